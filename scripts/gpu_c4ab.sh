#!/bin/bash
# Config 4 A/B of library builds (host passes of hpk_hdec_decode_blocks), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-c4ab}; mkdir -p $OUT
for r in $(seq ${ROUNDS:-2}); do
  for lib in ${LIBS:-libhpk.so}; do
    HPK_LIB=loona_amd/$lib timeout -k 10 300 python scripts/config4_time.py >> $OUT/config4.jsonl 2>>$OUT/config4.err || { echo "config4 $lib failed"; tail -20 $OUT/config4.err; exit 1; }
    tail -1 $OUT/config4.jsonl
  done
done
echo "exit 0"
