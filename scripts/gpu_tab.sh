#!/bin/bash
# A/B of the paired LDS-table loads: parity subset, config-2 decode, small-call latency, config 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-tab}; mkdir -p $OUT
TAG=${TAG:-tab}/w LIBS="$LIBS" WLS=config2 ROUNDS=4 bash scripts/gpu_r3w.sh || exit 1
for r in 1 2; do for lib in $LIBS; do
  HPK_LIB=loona_amd/$lib timeout -k 10 120 python scripts/lat_trace.py 200 >> $OUT/lat.jsonl 2>>$OUT/lat.err || { echo "lat $lib failed"; tail $OUT/lat.err; exit 1; }
  echo "$lib $(tail -2 $OUT/lat.jsonl | tr '\n' ' ' | cut -c1-300)"
done; done
TAG=${TAG:-tab}/c5 LIBS="$LIBS" WLS=config5 ROUNDS=2 bash scripts/gpu_ab.sh || exit 1
echo "exit 0"
