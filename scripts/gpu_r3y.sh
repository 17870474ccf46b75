#!/bin/bash
# Round 3: wave-kernel chunk claims (late claim, least chunk) — parity of the wave kernel per variant
# library, then an alternating A/B on config 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3y}; mkdir -p $OUT
for lib in ${LIBS:-libhpk.so}; do
  HPK_LIB=loona_amd/$lib timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "wave" > $OUT/pytest_$lib.log 2>&1 || { echo "pytest $lib failed"; tail -40 $OUT/pytest_$lib.log; exit 1; }
  echo "$lib: $(tail -1 $OUT/pytest_$lib.log)"
done
TAG=${TAG:-r3y}/ab WLS=${WLS:-config5} ROUNDS=${ROUNDS:-3} LIBS="${LIBS:-libhpk.so}" scripts/gpu_ab.sh || exit 1
echo "exit 0"
