#!/bin/bash
# Two PMC passes (SQ counters) over the decode kernel on config 3 (diag_decode.py, mode 0); each
# pass time-limited, the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-dec3pmc}
export DIAG_CONFIG=${DIAG_CONFIG:-config3}
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex hpk_decode --output-format csv -d $OUT/$TAG/p1 -o run -- python3 scripts/diag_decode.py > $OUT/$TAG.log 2>&1 || exit 2
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-include-regex hpk_decode --output-format csv -d $OUT/$TAG/p2 -o run -- python3 scripts/diag_decode.py >> $OUT/$TAG.log 2>&1 || exit 3
echo "exit 0"
