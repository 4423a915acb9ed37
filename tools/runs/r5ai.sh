# round-5 final check (session 2): smoke() and the driver's default bench line
# on the committed build (the line should quote profiles/r05_scan_profile.json)
set -e
export TMPDIR=/tmp
O=gpurun_out/r5ai
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
timeout -k 10 300 python3 bench.py > $O/bench.jsonl 2> $O/bench.err
echo ok
