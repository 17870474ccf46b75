#!/bin/bash
# A/B of library builds on the device encode (config 3 by default), alternating, each run checked.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abenc}; mkdir -p $OUT
for wl in ${WLS:-config3}; do
  for r in $(seq ${ROUNDS:-2}); do
    for lib in ${LIBS:-libhpk.so}; do
      HPK_LIB=loona_amd/$lib timeout -k 10 180 python scripts/enc_time.py $wl 20 >> $OUT/enc_time.jsonl 2>>$OUT/enc_time.err || { echo "enc_time $wl $lib failed"; tail -20 $OUT/enc_time.err; exit 1; }
    done
  done
done
python3 -c "
import json
for l in open('$OUT/enc_time.jsonl'):
    d = json.loads(l); print(d['workload'], d['lib'], d['encode_us'], d['bytes_equal_workload_encoding'])"
echo "exit 0"
