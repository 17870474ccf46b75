#!/bin/bash
# One GPU-box pass: parity tests, bench, kernel-trace profile. Every GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r01}
rocm-smi --showproductname > $OUT/gpu_info.txt 2>&1 || true
nproc >> $OUT/gpu_info.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1 &&
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/prof_$TAG -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu > $OUT/prof_$TAG.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
