#!/bin/bash
# Round-end GPU pass for the bench workload: parity tests + smoke, the PMC HBM traffic of the decode
# launches (FETCH_SIZE and WRITE_SIZE in separate kernel-trace passes) written where bench.py reads it,
# then bench.py (config 5 at N=1, its line carrying that traffic) and a rocprofv3 kernel trace of the
# same command. Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-final}
WL=config5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo "smoke failed"; exit 1; }
rm -rf $OUT/pmc_$TAG
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_$TAG/fetch -o run -- \
    python3 bench.py --workload $WL --steps 3 --warmup 1 --no-cpu --no-config2 > $OUT/pmc_$TAG.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_$TAG/write -o run -- \
    python3 bench.py --workload $WL --steps 3 --warmup 1 --no-cpu --no-config2 >> $OUT/pmc_$TAG.log 2>&1 || { echo "pmc write failed"; exit 1; }
python3 scripts/pmc_traffic.py $OUT/pmc_$TAG 32000000 $WL hpk_decode12 > $OUT/pmc_${WL}_$TAG.json || exit 1
cp $OUT/pmc_${WL}_$TAG.json profiles/pmc_config5.json
timeout -k 10 600 python bench.py --workload $WL > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/prof_$TAG -o run -- \
    python3 bench.py --workload $WL --steps 5 --warmup 1 --no-cpu --no-config2 > $OUT/prof_$TAG.log 2>&1 || { echo "prof failed"; exit 1; }
echo "exit 0"
