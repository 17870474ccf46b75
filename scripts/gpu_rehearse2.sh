#!/bin/bash
# Rehearsal of bench.py's N = 2 path on a ONE-GPU box: two ranks under torch.distributed.run, both on
# device 0 (HPK_BENCH_DEVICE) over gloo (HPK_BENCH_BACKEND: RCCL refuses two ranks on one GPU). The
# scatter + decode + gather leg is skipped (gloo carries no device tensors). Checks shard ownership,
# both ranks' output checks, the barriers and the max-over-ranks timing; the value is NOT a scaling
# number (the ranks share one GPU). Output: gpurun_out/rehearse/n2.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rehearse
HPK_BENCH_DEVICE=0 HPK_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 \
  --no-cpu --no-config2 --no-config3 --no-config4 --no-compact --no-e2e \
  > gpurun_out/rehearse/n2.json 2> gpurun_out/rehearse/n2.err
