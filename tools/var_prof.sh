#!/bin/bash
# Kernel time + SQ counters of library variants (variants/<name>/libipp.so;
# 'base' = the in-tree library).  Usage: tools/var_prof.sh <tag> name...
set -o pipefail
TAG=$1; shift
ARGS=${ARGS:---steps 2 --warmup 1 --batch 1024 --no-cpu-baseline --no-copy-ceiling}
CNT=${CNT:-SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE}
export TMPDIR=/tmp
for name in "$@"; do
  lib=$PWD/image_processor_pipeline_amd/libipp.so; [ "$name" != base ] && lib=$PWD/variants/$name/libipp.so
  OUT=gpurun_out/$TAG/$name; mkdir -p $OUT
  IPP_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py $ARGS > $OUT/kt.log 2>&1 || exit 11
  find $OUT/kt -name '*kernel_trace.csv' -delete
  IPP_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-include-regex 'k_pipe' --pmc $CNT --output-format csv -d $OUT/pmc -o pmc -- python3 bench.py $ARGS > $OUT/pmc.log 2>&1 || exit 12
  echo "== $name"; python3 tools/prof_summary.py $OUT | grep -E "${PAT:-hpass}"
done
