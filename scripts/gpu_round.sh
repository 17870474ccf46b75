#!/bin/bash
# Full GPU-box pass: parity tests, bench, kernel-trace profile, host-inclusive rate, PMC traffic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out; mkdir -p $OUT
TAG=$TAG bash scripts/gpu_check.sh || exit $?
timeout -k 10 300 python scripts/host_rate.py > $OUT/host_rate_$TAG.jsonl 2> $OUT/host_rate_$TAG.err || exit $?
TAG=$TAG bash scripts/gpu_pmc_traffic.sh
