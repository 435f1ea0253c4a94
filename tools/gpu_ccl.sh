#!/bin/bash
# CCL iteration on the GPU: parity tests of the CCL paths, the video4k bench
# line, and its kernel trace.  tools/gpu_ccl.sh <tag>
set -o pipefail
TAG=${1:-ccl}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_transforms_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "keep_largest or video or ccl" > gpurun_out/$TAG.log 2>&1 || { tail -30 gpurun_out/$TAG.log; exit 21; }
tail -3 gpurun_out/$TAG.log
timeout -k 10 300 python bench.py --workload video4k --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 22; }
tail -1 gpurun_out/bench_$TAG.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
KT_ONLY=1 timeout -k 10 300 bash tools/profile.sh ${TAG}_kt --workload video4k --steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling || exit 23
python tools/prof_summary.py gpurun_out/${TAG}_kt > gpurun_out/${TAG}_kt/summary.txt
grep k_ccl gpurun_out/${TAG}_kt/summary.txt
