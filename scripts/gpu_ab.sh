#!/bin/bash
# A/B of library builds in one box: for each workload, LIBS (loona_amd/libhpk*.so) alternate ROUNDS
# times, each run one dec_time.py process (timed launches checked once against the strings).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}; mkdir -p $OUT
for wl in ${WLS:-config3}; do
  for r in $(seq ${ROUNDS:-2}); do
    for lib in ${LIBS:-libhpk.so}; do
      HPK_LIB=loona_amd/$lib timeout -k 10 180 python scripts/dec_time.py $wl 20 >> $OUT/dec_time.jsonl 2>>$OUT/dec_time.err || { echo "dec_time $wl $lib failed"; tail -20 $OUT/dec_time.err; exit 1; }
    done
  done
done
python3 -c "
import json
for l in open('$OUT/dec_time.jsonl'):
    d = json.loads(l); print(d['workload'], d['lib'], d['decode_us'], d['checked'])"
echo "exit 0"
