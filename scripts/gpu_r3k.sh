#!/bin/bash
# Round 3: wave-kernel decomposition on config 5: product, mode 1 (fills without the lane walk),
# mode 2 (walk without output stores), each twice, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3k}; mkdir -p $OUT
for rep in 1 2; do
  for m in 0 1 2; do
    HPK_DEBUG_MODE=$m HPK_LIB=loona_amd/libhpk_diag.so HPK_DECODE_KERNEL=wave timeout -k 10 180 python scripts/dec_time.py config5 20 >> $OUT/dec_time.jsonl 2>>$OUT/dec_time.err || { echo "dec_time mode $m failed"; tail -20 $OUT/dec_time.err; exit 1; }
  done
done
cat $OUT/dec_time.jsonl
echo "exit 0"
