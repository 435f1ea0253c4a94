#!/bin/bash
set -o pipefail
for e in "$@"; do
  env $e timeout -k 10 300 python bench.py --workload rotflip --batch 1024 --no-cpu-baseline > gpurun_out/rf.log 2>&1 || { tail -5 gpurun_out/rf.log; exit 3; }
  python -c "import json; d=json.loads(open('gpurun_out/rf.log').read().strip().splitlines()[-1]); print('$e', d['value'], d['kernels_ms'], d['roofline']['frac'])"
done
