#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -k "pipe" > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 21; }
tail -1 gpurun_out/t.log
for f in mfma dot4; do
  IPP_TAPS=$f timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/taps_$f.log 2>&1 || { tail -20 gpurun_out/taps_$f.log; exit 22; }
  python -c "import json; d=json.loads(open('gpurun_out/taps_$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['kernels_ms'])"
done
