#!/bin/bash
# config 2 (1M literals): workgroup-fill kernel vs wave kernel with guided (variant 3) and static 1/16
# hand-out (variant 0), diagnostic library, alternating runs. Output gpurun_out/c2w/dec_time.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c2w
for r in 1 2 3; do
  HPK_LIB=loona_amd/libhpk_diag.so HPK_DECODE_KERNEL=fill timeout -k 10 180 python scripts/dec_time.py config2 100 >> gpurun_out/c2w/dec_time.jsonl || exit 1
  for v in 3 0; do
    HPK_LIB=loona_amd/libhpk_diag.so HPK_DECODE_KERNEL=wave HPK_WAVE_VARIANT=$v timeout -k 10 180 python scripts/dec_time.py config2 100 >> gpurun_out/c2w/dec_time.jsonl || exit 1
  done
done
