#!/bin/bash
# A/B of library variants on one box: tools/ab.sh "<bench args>" name[:ENV=V,...] ...
# 'base' = the in-tree library; other names = variants/<name>/libipp.so.
ARGS=$1; shift
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; envs=""; [ "$spec" != "$name" ] && envs=${spec#*:}
  lib=$PWD/image_processor_pipeline_amd/libipp.so; [ "$name" != base ] && lib=$PWD/variants/${name%%+*}/libipp.so
  out=$(env $(echo $envs | tr ',' ' ') IPP_AB_EXPERIMENT=1 IPP_LIB_PATH=$lib timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline --no-copy-ceiling --no-stream 2>gpurun_out/ab_err_${name}.log | tail -1)
  echo "$spec $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernels_ms"])')"
done
