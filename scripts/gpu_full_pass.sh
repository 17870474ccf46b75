#!/bin/bash
# Full GPU-box pass for a product build: parity tests, bench, rocprofv3 kernel trace, checked-store
# mode, PMC HBM traffic, host-inclusive rate and the other configs. Every GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-full}
TAG=$TAG bash scripts/gpu_check.sh > $OUT/check_$TAG.log 2>&1 || { echo "check failed"; exit 1; }
rm -f $OUT/diag4.jsonl
bash scripts/gpu_diag4.sh || { echo "diag4 failed"; exit 1; }
mv $OUT/diag4.jsonl $OUT/diag4_$TAG.jsonl
TAG=$TAG bash scripts/gpu_pmc_traffic.sh > $OUT/pmc_$TAG.out 2>&1 || { echo "pmc failed"; exit 1; }
timeout -k 10 300 python scripts/host_rate.py > $OUT/host_rate_$TAG.jsonl 2> $OUT/host_rate_$TAG.err || { echo "host_rate failed"; exit 1; }
timeout -k 10 600 python -u scripts/bench_configs.py > $OUT/configs_$TAG.jsonl 2> $OUT/configs_$TAG.err || { echo "configs failed"; exit 1; }
echo "all done"
