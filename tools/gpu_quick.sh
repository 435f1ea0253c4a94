#!/bin/bash
# Quick GPU session: parity tests, smoke, the default bench line.  Every GPU
# step has its own time limit; the first failure ends the script.
set -o pipefail
TAG=${1:-r02}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 21; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 22; }
echo smoke ok
timeout -k 10 600 python bench.py --stream > gpurun_out/bench_${TAG}_pipe5.json.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_pipe5.json.log; exit 23; }
tail -1 gpurun_out/bench_${TAG}_pipe5.json.log
