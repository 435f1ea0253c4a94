#!/bin/bash
# GPU session: the GPU test suite, then the pipe5 and video4k benches.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${TESTS:+-k "$TESTS"} > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 21; }
tail -1 gpurun_out/t.log
for w in ${WORKLOADS:-pipe5 video4k}; do
  timeout -k 10 400 python bench.py --no-cpu-baseline --workload $w > gpurun_out/b_$w.log 2>&1 || { tail -20 gpurun_out/b_$w.log; exit 22; }
  python -c "import json; d=json.loads(open('gpurun_out/b_$w.log').read().strip().splitlines()[-1]); print('$w', d['value'], d['kernels_ms'], d['roofline']['frac'])"
done
