#!/bin/bash
# Device tap planner + streaming bench session: new tests first, then the
# pipe parity suite (now fed by device-built taps), bench-scale checks and
# the bench with --stream.  The first failing GPU step ends the script.
set -o pipefail
TAG=${1:-r03f}
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1 || { echo "FAILED: $*"; tail -40 "gpurun_out/$log"; exit 21; }; tail -1 "gpurun_out/$log" | cut -c1-600; }
run 300 pt_taps_${TAG}.log python -u -m pytest tests/test_gpu_taps.py -x -v -s --timeout 240 --timeout-method thread
run 300 pt_pipe_${TAG}.log python -u -m pytest tests/test_gpu_parity.py -k pipe -x -v --timeout 120 --timeout-method thread
run 400 pt_new_${TAG}.log python -u -m pytest tests/test_gpu_benchscale.py tests/test_transforms_gpu.py -k "benchscale or alpha_one or fit_crop or keep_largest" -x -v --timeout 300 --timeout-method thread
run 400 bench_${TAG}_stream.json.log python bench.py --no-cpu-baseline --stream
