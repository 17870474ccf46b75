#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for n in 142773 400000 1000000; do
  HPK_DEBUG_MODE=4 DIAG_N=$n timeout -k 10 300 python scripts/diag_decode.py >> $OUT/diag4.jsonl 2>> $OUT/diag4.err || exit $?
done
