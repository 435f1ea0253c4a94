#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root):
#   kernel trace + stats, then separate PMC passes (FETCH_SIZE / WRITE_SIZE /
#   SQ counter groups) restricted to the ipp kernels — never combined with
#   trace domains (gpurun refuses that).  Bulky per-dispatch CSVs are pruned
#   after summarising so the output stays small.
# Usage: tools/profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-prof}; shift
ARGS=${@:---steps 3 --warmup 1 --no-cpu-baseline --no-stream}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
FILTER='k_pipe|k_rotate|k_lanczos|k_paste|k_hsv|k_ccl|k_copy|k_alpha'
run() { local name=$1; shift; timeout -k 10 300 rocprofv3 "$@" --output-format csv -d $OUT/$name -o $name -- python3 bench.py $ARGS > $OUT/$name.log 2>&1; }
pmc() { local name=$1; shift; run $name --kernel-include-regex "$FILTER" --pmc "$@"; }
run kt --kernel-trace --stats || exit 11
find $OUT/kt -name '*kernel_trace.csv' -delete
[ -n "$KT_ONLY" ] && exit 0
if [ -z "$SQ_ONLY" ]; then
pmc fetch FETCH_SIZE || exit 12
pmc write WRITE_SIZE || exit 13
fi
pmc sqa SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY || exit 14
pmc sqb SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU || exit 15
pmc misc GRBM_GUI_ACTIVE GRBM_TA_BUSY TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT || exit 16
echo profile done
