#!/bin/bash
# Round 3: long-literal phase geometry (waves, ring, steps per period) — parity subset per variant
# library, then an alternating A/B of the config-3 decode.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3w}; mkdir -p $OUT
for lib in ${LIBS:-libhpk.so}; do
  HPK_LIB=loona_amd/$lib timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "long or config3 or bad or interop or kats or error" > $OUT/pytest_$lib.log 2>&1 || { echo "pytest $lib failed"; tail -40 $OUT/pytest_$lib.log; exit 1; }
  echo "$lib: $(tail -1 $OUT/pytest_$lib.log)"
done
TAG=${TAG:-r3w}/ab WLS=${WLS:-config3} ROUNDS=${ROUNDS:-3} LIBS="${LIBS:-libhpk.so}" scripts/gpu_ab.sh || exit 1
echo "exit 0"
