#!/bin/bash
# Round 3: decomposition of the decode kernel's time (product library; diagnostic modes 1 = no decode,
# 2 = no output stores) on config 2 and a config-5 shard, the vector-memory probe for per-lane
# streams, SQ counters of the product on a config-5 shard, and the bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3b; mkdir -p $OUT
timeout -k 10 120 ./bench/ta_probe > $OUT/ta_probe.jsonl 2>&1 || { echo "ta_probe failed"; cat $OUT/ta_probe.jsonl; exit 1; }
cat $OUT/ta_probe.jsonl
for wl in config2 config5; do
  for m in 0 1 2; do
    HPK_LIB=loona_amd/libhpk_diag.so HPK_DEBUG_MODE=$m timeout -k 10 240 python scripts/dec_time.py $wl 20 >> $OUT/dec_time.jsonl 2>>$OUT/dec_time.err || { echo "dec_time $wl mode $m failed"; tail $OUT/dec_time.err; exit 1; }
  done
  timeout -k 10 240 python scripts/dec_time.py $wl 20 >> $OUT/dec_time.jsonl 2>>$OUT/dec_time.err || { echo "dec_time $wl failed"; exit 1; }
done
cat $OUT/dec_time.jsonl
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-trace --output-format csv -d $OUT/pmc_sq -o run -- python3 scripts/dec_time.py config5 3 > $OUT/pmc_sq.log 2>&1 || { echo "pmc failed"; tail $OUT/pmc_sq.log; exit 1; }
python3 scripts/pmc_sq.py $OUT/pmc_sq 32000000 config5 hpk_decode12 > $OUT/pmc_sq_config5.json || exit 1
cat $OUT/pmc_sq_config5.json
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo "exit 0"
