#!/bin/bash
# A/B session: GPU parity tests, then the default bench under each env setting
# given as arguments (e.g. "IPP_HPASS=1" "IPP_HPASS=2").
set -o pipefail
mkdir -p gpurun_out
[ -n "$NO_TESTS" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${TESTS:+-k "$TESTS"} > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 21; }
[ -n "$NO_TESTS" ] || tail -1 gpurun_out/t.log
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-10} ${BENCH_ARGS} > gpurun_out/ab_$i.log 2>&1 || { tail -20 gpurun_out/ab_$i.log; exit 22; }
  python -c "import json; d=json.loads(open('gpurun_out/ab_$i.log').read().strip().splitlines()[-1]); print('$e', d['value'], d['kernels_ms'], d['roofline']['frac'])"
done
