#!/bin/bash
# Round 3, first pass: GPU tests, then a decomposition of the decode kernel's time on config 2 and a
# config-5 shard (product library, diagnostic modes 1 = no decode, 2 = no output stores), SQ counters
# of the product on a config-5 shard, and the bench line. Each GPU step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3a; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
for wl in config2 config5; do
  timeout -k 10 240 python scripts/dec_time.py $wl 20 >> $OUT/dec_time.jsonl 2>>$OUT/dec_time.err || { echo "dec_time $wl failed"; exit 1; }
  for m in 1 2; do
    HPK_LIB=loona_amd/libhpk_diag.so HPK_DEBUG_MODE=$m timeout -k 10 240 python scripts/dec_time.py $wl 20 >> $OUT/dec_time.jsonl 2>>$OUT/dec_time.err || { echo "dec_time $wl mode $m failed"; exit 1; }
  done
done
cat $OUT/dec_time.jsonl
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --output-format csv -d $OUT/pmc_sq -o run -- python3 scripts/dec_time.py config5 3 > $OUT/pmc_sq.log 2>&1 || { echo "pmc failed"; exit 1; }
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo "exit 0"
