#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root):
#   kernel trace + stats, then separate PMC passes (FETCH_SIZE / WRITE_SIZE /
#   SQ counter groups) — never combined with trace domains (gpurun refuses that).
# Usage: tools/profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-prof}; shift
ARGS=${@:---steps 3 --warmup 1 --no-cpu-baseline}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 300 rocprofv3 "$@" --output-format csv -d $OUT/$name -o $name -- python3 bench.py $ARGS > $OUT/$name.log 2>&1; }
run kt --kernel-trace --stats || exit 11
run fetch --pmc FETCH_SIZE || exit 12
run write --pmc WRITE_SIZE || exit 13
run sqa --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY || exit 14
run sqb --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU || exit 15
run misc --pmc GRBM_GUI_ACTIVE GRBM_TA_BUSY TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT || exit 16
echo profile done
