#!/bin/bash
# Round-end style GPU session (run through gpurun from the repo root):
#   tools/gpu_session.sh <tag> [quick|tests|prof]
# the GPU test suite, smoke(), the default bench line (config 3 with its
# streaming leg, CPU baseline and the config-2 / config-5 legs), config 5 on
# noisy frames, then the kernel traces and PMC passes of the three workloads
# (tools/profile_workload.sh).
# Every GPU step has its own time limit; the first failure ends the script.
# With "quick": only the pipe parity tests and the default bench line; with
# "prof": only the profiles (and the RCCL probe when RCCL_PROBE is set).
set -o pipefail
TAG=${1:-session}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" = prof ]; then
  :
elif [ "$2" = quick ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_benchscale.py -k "pipe or benchscale" -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 21; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 21; }
fi
if [ "$2" != prof ]; then
tail -1 $OUT/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 22; }
echo smoke ok
timeout -k 10 600 python bench.py > $OUT/bench_pipe5.json.log 2>&1 || { tail -20 $OUT/bench_pipe5.json.log; exit 23; }
tail -c 1500 $OUT/bench_pipe5.json.log
[ "$2" = quick ] && exit 0
timeout -k 10 400 python bench.py --workload video4k --frame-noise 2 --no-cpu-baseline > $OUT/bench_video4k_noise2.json.log 2>&1 || exit 25
tail -c 600 $OUT/bench_video4k_noise2.json.log
[ "$2" = tests ] && exit 0
fi
bash tools/profile_workload.sh ${TAG}/prof_pipe5 pipe5 4096 || exit 26
bash tools/profile_workload.sh ${TAG}/prof_rotflip rotflip 1024 || exit 27
bash tools/profile_workload.sh ${TAG}/prof_video4k video4k 256 || exit 28
echo all done
# last: can two RCCL ranks share the box's one GPU? (a failure here ends nothing above)
[ -n "$RCCL_PROBE" ] && { timeout -k 10 120 python tools/probes/rccl_same_gpu.py > $OUT/rccl_same_gpu.log 2>&1; echo "rccl probe rc=$?"; tail -5 $OUT/rccl_same_gpu.log; }
exit 0
