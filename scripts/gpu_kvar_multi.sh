#!/bin/bash
# Decode-kernel harness over several inputs: one variant per process, each GPU step time-limited;
# the chain stops at the first failure. INPUTS="config2 config3", VARIANTS="coop1_snake ...".
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-km}
for inp in ${INPUTS:-config2}; do
  timeout -k 10 300 python scripts/kinput.py $inp /tmp/k_$inp.bin > $OUT/kvar_${TAG}_$inp.log 2>&1 || exit 1
  for v in ${VARIANTS:-coop1_snake}; do
    timeout -k 5 60 ./bench/kvariants /tmp/k_$inp.bin ${ITERS:-20} $v >> $OUT/kvar_${TAG}_$inp.log 2>&1 || { echo "$v exit $?" >> $OUT/kvar_${TAG}_$inp.log; exit 1; }
  done
done
echo "exit 0"
