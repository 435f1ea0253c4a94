#!/bin/bash
# Round-end style GPU session: parity tests, smoke, the default bench line
# (with CPU baseline), the config-2 and config-5 bench lines, then the
# rocprofv3 kernel-trace + PMC passes of the default bench.  Every GPU step has
# its own time limit; the first failure ends the script.
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 21; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 22; }
echo smoke ok
timeout -k 10 600 python bench.py > gpurun_out/bench_${TAG}_pipe5.json.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_pipe5.json.log; exit 23; }
tail -1 gpurun_out/bench_${TAG}_pipe5.json.log
timeout -k 10 300 python bench.py --workload rotflip --batch 1024 --no-cpu-baseline > gpurun_out/bench_${TAG}_rotflip.json.log 2>&1 || exit 24
tail -1 gpurun_out/bench_${TAG}_rotflip.json.log
timeout -k 10 400 python bench.py --workload video4k --no-cpu-baseline > gpurun_out/bench_${TAG}_video4k.json.log 2>&1 || exit 25
tail -1 gpurun_out/bench_${TAG}_video4k.json.log
bash tools/gpu_prof.sh prof_${TAG} --steps 3 --warmup 1 --no-cpu-baseline || exit 26
echo all done
