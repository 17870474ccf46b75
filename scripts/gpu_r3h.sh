#!/bin/bash
# Round 3: wave-kernel A/B over the chunk hand-out (static / guided) x the queue order (LDS counting
# sort, 16- or 32-class ballots), config 5 and config 2, each run checked once; the fill kernel beside.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3h}; mkdir -p $OUT
for wl in config5 config2; do
  HPK_LIB=loona_amd/libhpk_diag.so HPK_DECODE_KERNEL=fill timeout -k 10 180 python scripts/dec_time.py $wl 20 >> $OUT/dec_time.jsonl 2>>$OUT/dec_time.err || { echo "dec_time $wl fill failed"; tail -20 $OUT/dec_time.err; exit 1; }
  for v in ${VARIANTS:-0 1 2 3 4 5}; do
    HPK_WAVE_VARIANT=$v HPK_LIB=loona_amd/libhpk_diag.so HPK_DECODE_KERNEL=wave timeout -k 10 180 python scripts/dec_time.py $wl 20 >> $OUT/dec_time.jsonl 2>>$OUT/dec_time.err || { echo "dec_time $wl $v failed"; tail -20 $OUT/dec_time.err; exit 1; }
  done
done
cat $OUT/dec_time.jsonl
echo "exit 0"
