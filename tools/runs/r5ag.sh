# round-5 (session 2): grid SHA-1 blocks in flight per lane (2 shipped, 3, 4, 6)
set -e
export TMPDIR=/tmp
O=gpurun_out/r5ag
mkdir -p $O
for rep in 1 2; do
  for a in 2 3 4 6; do
    echo "ahead $a rep $rep" >> $O/sha_ahead.txt
    timeout -k 10 60 tools/ubench/sha_bench_a$a >> $O/sha_ahead.txt 2>&1
  done
done
echo ok
