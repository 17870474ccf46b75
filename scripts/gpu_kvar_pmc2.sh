#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-kp}
timeout -k 10 300 python scripts/kinput.py config2 /tmp/kin2.bin > $OUT/kvp_$TAG.log 2>&1 || exit 1
timeout -k 10 300 ./bench/kvariants /tmp/kin2.bin 20 >> $OUT/kvp_$TAG.log 2>&1 || exit 1
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "GRBM_GUI_ACTIVE SQ_IFETCH SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/kvp_$TAG/p$i -o run -- ./bench/kvariants /tmp/kin2.bin 3 >> $OUT/kvp_$TAG.pmc.log 2>&1 || exit 2
done
echo "exit 0"
