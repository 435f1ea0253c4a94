#!/bin/bash
# Round-end style GPU session: parity tests, smoke, the three bench lines,
# then kernel-trace + PMC profiles (and PMC traffic) of each workload.
# Every GPU step has its own time limit; the first failure ends the script.
#   tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-r02}
export TMPDIR=/tmp
bash tools/gpu_quick.sh $TAG || exit $?
for wl in rotflip video4k; do
  timeout -k 10 600 python bench.py --workload $wl > gpurun_out/bench_${TAG}_$wl.json.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_$wl.json.log; exit 24; }
  tail -1 gpurun_out/bench_${TAG}_$wl.json.log
done
bash tools/gpu_prof2.sh ${TAG}_pipe5 pipe5 4096 || exit 26
bash tools/gpu_prof2.sh ${TAG}_rotflip rotflip 1024 || exit 27
bash tools/gpu_prof2.sh ${TAG}_video4k video4k 256 || exit 28
echo round session done
