#!/bin/bash
# Round-3 GPU session: pipe parity tests first (fast fail), then the whole GPU
# suite, smoke, and the default bench line.  Each GPU step has its own limit;
# the first failure ends the script.
set -o pipefail
TAG=${1:-r03}
FULL=${FULL:-1}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k pipe -x -v --timeout 120 --timeout-method thread > gpurun_out/pt_pipe_${TAG}.log 2>&1 || { tail -60 gpurun_out/pt_pipe_${TAG}.log; exit 21; }
tail -1 gpurun_out/pt_pipe_${TAG}.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_pipe5.json.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_pipe5.json.log; exit 23; }
tail -1 gpurun_out/bench_${TAG}_pipe5.json.log | cut -c1-1200
[ "$FULL" = 1 ] || exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_${TAG}.log; exit 22; }
tail -1 gpurun_out/pytest_gpu_${TAG}.log
