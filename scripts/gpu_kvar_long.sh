#!/bin/bash
# Decode-kernel harness on long literals (cooperative path): one variant per process, each GPU
# step time-limited; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-kl}
timeout -k 10 300 python scripts/kinput.py ${KINPUT:-interop_long} /tmp/kil.bin ${KN:-} > $OUT/kvar_$TAG.log 2>&1 || exit 1
for v in ${VARIANTS:-coop0 coop2 coop1_checked coop1}; do
  timeout -k 5 30 ./bench/kvariants /tmp/kil.bin 5 $v >> $OUT/kvar_$TAG.log 2>&1 || { echo "$v exit $?" >> $OUT/kvar_$TAG.log; exit 1; }
done
echo "exit 0" >> $OUT/kvar_$TAG.log
