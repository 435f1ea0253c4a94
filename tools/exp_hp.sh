#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for d in ${DBGS:-0 1 2 3 4 7}; do
  IPP_DBG_HPASS=$d timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/hp_$d.log 2>&1 || { tail -20 gpurun_out/hp_$d.log; exit 22; }
  python -c "import json; d=json.loads(open('gpurun_out/hp_$d.log').read().strip().splitlines()[-1]); print('dbg=$d', d['kernels_ms'])"
done
