#!/bin/bash
# (round 6, development) config-2 and small-call timings of library variants (LIBS), alternating rounds
set -o pipefail
OUT=gpurun_out/${TAG:-c2}; mkdir -p $OUT
for r in $(seq ${ROUNDS:-3}); do for lib in $LIBS; do
  HPK_LIB=loona_amd/$lib timeout -k 10 120 python scripts/dec_time.py config2 ${REPS:-50} >> $OUT/dec_time.jsonl 2>>$OUT/dec_time.err || { echo "dec_time $lib failed"; tail $OUT/dec_time.err; exit 1; }
done; done
for lib in $LIBS; do HPK_LIB=loona_amd/$lib timeout -k 10 120 python scripts/lat_trace.py 200 2>/dev/null | sed "s/^/$lib /" >> $OUT/lat.jsonl || { echo "lat $lib failed"; exit 1; }; done
python3 -c "
import json
for l in open('$OUT/dec_time.jsonl'):
    d = json.loads(l); print(d['workload'], d['lib'], d['decode_us'], d['checked'])"
cat $OUT/lat.jsonl
