#!/bin/bash
# PMC probe of the H pass for library variants: tools/gpu_pmcprobe.sh <tag> name...
# ('base' = in-tree library, else variants/<name>/libipp.so).  One pass per
# counter group, each under its own time limit; the first failure ends it.
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
FILTER='k_pipe_hpass'
for name in "$@"; do
  lib=$PWD/image_processor_pipeline_amd/libipp.so; [ "$name" != base ] && lib=$PWD/variants/$name/libipp.so
  export IPP_LIB_PATH=$lib IPP_AB_EXPERIMENT=1
  OUT=gpurun_out/$TAG/$name; mkdir -p $OUT
  i=0
  for grp in "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE TD_TD_BUSY_sum TD_TC_STALL_sum" \
             "TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_ADDR_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum" \
             "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-include-regex "$FILTER" --pmc $grp --output-format csv -d $OUT/p$i -o p$i -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-copy-ceiling --no-stream > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 31; }
  done
  python tools/prof_summary.py $OUT > $OUT/summary.txt 2>&1 || true
  find $OUT -name '*counter_collection.csv' -size +4M -delete
  echo "== $name"; grep -v calls= $OUT/summary.txt
done
