#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -k "pipe" > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 21; }
tail -1 gpurun_out/t.log
for c in 0 64 128 256 512; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --chunk $c > gpurun_out/ch_$c.log 2>&1 || { tail -20 gpurun_out/ch_$c.log; exit 22; }
  python -c "import json; d=json.loads(open('gpurun_out/ch_$c.log').read().strip().splitlines()[-1]); print('chunk=$c', d['value'], d['kernels_ms'])"
done
