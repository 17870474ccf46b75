#!/bin/bash
# hpk_decode_long study: GPU tests (product library), decode time of config 3 / config 2, then the
# diagnostic variants (HPK_LONG_VAR, HPK_LONG_MIN / HPK_LONG_BIG from the env) with per-wave counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-lv}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1 || { echo "pytest failed"; exit 1; }
fi
timeout -k 10 200 python3 scripts/dec_time.py config3 10 > $OUT/dt_$TAG.jsonl 2> $OUT/dt_$TAG.err || exit 2
timeout -k 10 200 python3 scripts/dec_time.py config2 20 >> $OUT/dt_$TAG.jsonl 2>> $OUT/dt_$TAG.err || exit 3
if [ -n "$TRACE" ]; then
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/tr_$TAG -o run -- python3 scripts/dec_time.py config3 5 > $OUT/tr_$TAG.log 2>&1 || exit 6
fi
for v in ${VARS:-0 1 2 3 4}; do
  HPK_DEBUG_MODE=5 HPK_LONG_VAR=$v DIAG_CONFIG=config3 timeout -k 10 200 python3 scripts/diag_decode.py >> $OUT/lv_$TAG.jsonl 2>> $OUT/lv_$TAG.err || exit 4
  HPK_DEBUG_MODE=0 HPK_LONG_VAR=$v DIAG_CONFIG=config3 timeout -k 10 200 python3 scripts/diag_decode.py >> $OUT/lv_$TAG.jsonl 2>> $OUT/lv_$TAG.err || exit 5
done
echo "exit 0"
