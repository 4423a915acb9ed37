#!/bin/bash
# Round profile set (run on the GPU box through gpurun; tooling only):
#   the build id of the libzchunk.so profiled (tools/collect_profiles.py keys
#   profiles/rNN_scan_profile.json on it; bench.py quotes only a matching one),
#   rocprofv3 kernel-trace summaries of C2/C3/C5 and of C2 with SHA-1 ids, the
#   scan's FETCH_SIZE and WRITE_SIZE passes and one SQ-counter pass (separate
#   runs), the bundle compressor's kernel trace (tools/lzo_rate.py), the host
#   CPU description, the static index at 2 M ids (trace + FETCH/WRITE), the LZO
#   dictionary-placement ubench's FETCH/WRITE per variant, and last the full
#   bench line (which then finds the profile
#   only after collect_profiles.py has run here -- it is re-run by the driver).
#   bash tools/profile_round.sh OUTDIR
set -e
set -o pipefail
OUT=${1:-gpurun_out/prof_round}
mkdir -p "$OUT"
export TMPDIR=/tmp
python3 -c "from zbackup_amd import _build, _lib; _lib.load(); print(_build.lib_build_id())" > "$OUT/build_id.txt"
for c in c2 c3 c5; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace_$c" -o $c -- \
    python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-extras > "$OUT/trace_$c.log" 2>&1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace_c2sha" -o c2sha -- \
  python3 bench.py --sha1 --steps 20 --warmup 5 --no-cpu-baseline --no-extras > "$OUT/trace_c2sha.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o f -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o w -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > "$OUT/pmc_write.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_sq" -o s -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > "$OUT/pmc_sq.log" 2>&1
if [ -z "$NO_LZO" ]; then
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace_lzo" -o lzo -- \
    python3 tools/lzo_rate.py 4 random text > "$OUT/trace_lzo.log" 2>&1
fi
if [ -z "$NO_STATIC" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace_static" -o st -- \
    python3 tools/static_scale.py 1 300000 2000000 > "$OUT/trace_static.log" 2>&1
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_static_fetch" -o f -- \
    python3 tools/static_scale.py 1 2000000 > "$OUT/pmc_static_fetch.log" 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_static_write" -o w -- \
    python3 tools/static_scale.py 1 2000000 > "$OUT/pmc_static_write.log" 2>&1
fi
if [ -z "$NO_LZO" ] && [ -x tools/ubench/lzo_dict_bench ]; then
  python3 -c "from tests.lzo_inputs import payload; payload('text', 128 << 20, 21).tofile('/tmp/text.bin')"
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_lzo_fetch" -o f -- \
    tools/ubench/lzo_dict_bench /tmp/text.bin 4 1 > "$OUT/pmc_lzo_fetch.log" 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_lzo_write" -o w -- \
    tools/ubench/lzo_dict_bench /tmp/text.bin 4 1 > "$OUT/pmc_lzo_write.log" 2>&1
fi
(lscpu; echo; echo "nproc: $(nproc)") > "$OUT/host_cpu.txt"
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 300 python3 bench.py > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
fi
echo done
