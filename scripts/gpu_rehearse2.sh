#!/bin/bash
# Rehearsal of bench.py's N > 1 path on a one-GPU box: two ranks on device 0 over gloo (RCCL refuses
# two ranks per GPU): the timed decode and the max-over-ranks timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HPK_BENCH_DEVICE=0 HPK_BENCH_BACKEND=gloo
OUT=gpurun_out/${TAG:-rehearse2}; mkdir -p $OUT
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --no-config2 --no-config3 --no-config4 --no-e2e > $OUT/n2_noe2e.json 2> $OUT/n2_noe2e.err || { echo "n2 (no e2e) failed"; tail -30 $OUT/n2_noe2e.err; exit 1; }
cut -c1-600 $OUT/n2_noe2e.json
# (the scatter + decode + gather leg cannot be rehearsed here: gloo has no device-tensor send/recv
# (the run hung) and RCCL refuses two ranks on one GPU)
echo "exit 0"
