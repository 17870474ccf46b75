#!/bin/bash
# Round 3: v25 wave kernel: per-wave phase stamps (config 5, config 2) and SQ counters on config 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3d; mkdir -p $OUT
for wl in config5 config2; do
  timeout -k 10 180 python scripts/wave_stamps.py $wl >> $OUT/stamps.jsonl 2>>$OUT/stamps.err || { echo "stamps $wl failed"; tail -20 $OUT/stamps.err; exit 1; }
done
cat $OUT/stamps.jsonl
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-trace --output-format csv -d $OUT/pmc_sq -o run -- python3 scripts/dec_time.py config5 3 > $OUT/pmc_sq.log 2>&1 || { echo "pmc failed"; tail $OUT/pmc_sq.log; exit 1; }
python3 scripts/pmc_sq.py $OUT/pmc_sq 32000000 config5 hpk_decode_wave > $OUT/pmc_sq_config5.json || exit 1
cat $OUT/pmc_sq_config5.json
echo "exit 0"
