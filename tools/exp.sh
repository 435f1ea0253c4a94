#!/bin/bash
# Quick GPU experiment: pipe parity subset, then the bench under each
# IPP_VB_STORE policy.  Each GPU step has its own limit; stops at first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -k "pipe or hsv" > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 21; }
tail -1 gpurun_out/t.log
for p in ${POLICIES:-1 0 2}; do
  IPP_VB_STORE=$p timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_$p.log 2>&1 || { tail -20 gpurun_out/b_$p.log; exit 22; }
  echo "policy $p: $(python -c "import json,sys; d=json.loads(open('gpurun_out/b_$p.log').read().strip().splitlines()[-1]); print(d['value'], d['kernels_ms'])")"
done
