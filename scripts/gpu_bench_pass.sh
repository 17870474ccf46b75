#!/bin/bash
# GPU-box pass for the bench workload: parity tests, bench.py (default: config 5 at N=1), a rocprofv3
# kernel trace of the same command, and the PMC HBM traffic of its decode launches (FETCH_SIZE and
# WRITE_SIZE in separate passes, kernel trace only). Every GPU step has its own time limit and the
# chain stops at the first failure. TAG names the outputs; SKIP_TESTS=1 skips pytest.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r02}
WL=${WL:-config5}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; exit 1; }
fi
timeout -k 10 600 python bench.py --workload $WL > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/prof_$TAG -o run -- \
    python3 bench.py --workload $WL --steps 5 --warmup 1 --no-cpu --no-config2 > $OUT/prof_$TAG.log 2>&1 || { echo "prof failed"; exit 1; }
if [ -z "$SKIP_PMC" ]; then
  rm -rf $OUT/pmc_${TAG}
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_$TAG/fetch -o run -- \
      python3 bench.py --workload $WL --steps 3 --warmup 1 --no-cpu --no-config2 > $OUT/pmc_$TAG.log 2>&1 &&
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_$TAG/write -o run -- \
      python3 bench.py --workload $WL --steps 3 --warmup 1 --no-cpu --no-config2 >> $OUT/pmc_$TAG.log 2>&1 || { echo "pmc failed"; exit 1; }
  LIT=$([ "$WL" = config5 ] && echo 32000000 || echo 1000000)
  python3 scripts/pmc_traffic.py $OUT/pmc_$TAG $LIT $WL hpk_decode12 > $OUT/pmc_${WL}_$TAG.json
fi
echo "exit 0"
