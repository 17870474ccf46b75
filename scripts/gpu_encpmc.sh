#!/bin/bash
# SQ counters of the config-3 device encode (hpk_encode2), two passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-encpmc}; mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY"
P2="SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES"
timeout -k 10 300 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $OUT/p1 -o run -- python3 scripts/enc_time.py config3 10 > $OUT/p1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc $P2 --kernel-trace --output-format csv -d $OUT/p2 -o run -- python3 scripts/enc_time.py config3 10 > $OUT/p2.log 2>&1 || { echo "pmc failed"; tail $OUT/p1.log $OUT/p2.log; exit 1; }
python3 scripts/pmc_sq.py $OUT/p1 1000000 config3 hpk_encode2 > $OUT/sq1.json && python3 scripts/pmc_sq.py $OUT/p2 1000000 config3 hpk_encode2 > $OUT/sq2.json && echo "exit 0"
