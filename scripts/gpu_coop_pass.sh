#!/bin/bash
# GPU pass after enabling the cooperative long-literal path: parity tests, harness, configs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-coop}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; exit 1; }
VARIANTS="coop0 coop1" TAG=$TAG bash scripts/gpu_kvar_long.sh || { echo "kvar long failed"; exit 1; }
timeout -k 10 600 python -u scripts/bench_configs.py > $OUT/configs_$TAG.jsonl 2> $OUT/configs_$TAG.err || { echo "configs failed"; exit 1; }
echo "all done"
