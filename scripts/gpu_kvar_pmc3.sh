#!/bin/bash
# One PMC pass (SQ counters) over the harness variants; each pass time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-kp3}
timeout -k 10 300 python scripts/kinput.py config2 /tmp/kin2.bin > $OUT/kvp_$TAG.log 2>&1 || exit 1
timeout -k 10 120 ./bench/kvariants /tmp/kin2.bin 10 >> $OUT/kvp_$TAG.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/kvp_$TAG/p1 -o run -- ./bench/kvariants /tmp/kin2.bin 3 >> $OUT/kvp_$TAG.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/kvp_$TAG/p2 -o run -- ./bench/kvariants /tmp/kin2.bin 3 >> $OUT/kvp_$TAG.log 2>&1 || exit 3
echo "exit 0"
