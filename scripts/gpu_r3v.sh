#!/bin/bash
# Round 3 (session 2): GPU parity suite, host-inclusive rate and per-call latency on the current
# library, then A/B of the long-phase priority and encode OR-when-full variants (config 3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3v}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u scripts/host_rate.py 1000000 10 > $OUT/host_rate.jsonl 2> $OUT/host_rate.err || { echo "host_rate failed"; tail $OUT/host_rate.err; exit 1; }
cat $OUT/host_rate.jsonl
timeout -k 10 300 python -u scripts/latency.py > $OUT/latency.jsonl 2> $OUT/latency.err || { echo "latency failed"; tail $OUT/latency.err; exit 1; }
cat $OUT/latency.jsonl
TAG=${TAG:-r3v}/abdec WLS=config3 ROUNDS=3 LIBS="libhpk.so libhpk_prio.so libhpk_prio16k.so" scripts/gpu_ab.sh || exit 1
TAG=${TAG:-r3v}/abenc WLS=config3 ROUNDS=3 LIBS="libhpk.so libhpk_orfull.so" scripts/gpu_ab_enc.sh || exit 1
echo "exit 0"
