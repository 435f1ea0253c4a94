#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for g in 1 2 4 8 16; do
  IPP_VB_GROUP=$g timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/vb_$g.log 2>&1 || { tail -20 gpurun_out/vb_$g.log; exit 22; }
  python -c "import json; d=json.loads(open('gpurun_out/vb_$g.log').read().strip().splitlines()[-1]); print('G=$g', d['value'], d['kernels_ms'])"
done
