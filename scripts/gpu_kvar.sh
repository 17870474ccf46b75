#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-kv}
timeout -k 10 300 python scripts/kinput.py config2 /tmp/kin2.bin > $OUT/kvar_$TAG.log 2>&1 &&
timeout -k 10 300 ./bench/kvariants /tmp/kin2.bin 20 >> $OUT/kvar_$TAG.log 2>&1
echo "exit $?"
