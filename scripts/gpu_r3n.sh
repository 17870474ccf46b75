#!/bin/bash
# Round 3: wave-kernel per-wave stamps (sums in LDS) on config 5, and the stamped vs product time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3n}; mkdir -p $OUT
for m in 0 3; do
  HPK_DEBUG_MODE=$m HPK_LIB=loona_amd/libhpk_diag.so HPK_DECODE_KERNEL=wave timeout -k 10 180 python scripts/dec_time.py config5 20 >> $OUT/dec_time.jsonl 2>>$OUT/dec_time.err || { echo "dec_time mode $m failed"; tail -20 $OUT/dec_time.err; exit 1; }
done
for wl in config5 c2_4m; do
  timeout -k 10 180 python scripts/wave_stamps.py $wl >> $OUT/stamps.jsonl 2>>$OUT/stamps.err || { echo "stamps failed"; tail -20 $OUT/stamps.err; exit 1; }
done
cat $OUT/dec_time.jsonl $OUT/stamps.jsonl
echo "exit 0"
