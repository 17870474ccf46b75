#!/bin/bash
# (round 6, development) parity of long-literal variants, then a config-3 A/B: LIBS_T (tested), LIBS_AB (timed)
set -o pipefail
OUT=gpurun_out/${TAG:-ltest}; mkdir -p $OUT
for lib in ${LIBS_T:-libhpk.so}; do
  HPK_LIB=loona_amd/$lib timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "${PYK:-long or config3 or large or huge or dense or kats or error_vectors or random_and_edge or interop}" > $OUT/pytest_$lib.log 2>&1 || { echo "pytest $lib failed"; tail -40 $OUT/pytest_$lib.log; exit 1; }
  echo "$lib: $(tail -1 $OUT/pytest_$lib.log)"
done
[ -n "$LIBS_AB" ] && TAG=${TAG:-ltest} STEPS=ab WLS="${WLS:-config3}" ROUNDS=${ROUNDS:-3} REPS=10 LIBS="$LIBS_AB" bash scripts/gpu_run.sh
exit 0
