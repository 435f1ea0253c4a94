#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for p in 2 9 10 11; do
  IPP_VB_STORE=$p timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/vb_$p.log 2>&1 || { tail -20 gpurun_out/vb_$p.log; exit 22; }
  python -c "import json; d=json.loads(open('gpurun_out/vb_$p.log').read().strip().splitlines()[-1]); print('pol=$p', d['value'], d['kernels_ms'])"
done
