#!/bin/bash
# Round-3 checkpoint session: the whole GPU suite (failures reported, the
# session goes on unless the run itself died), smoke, the default bench line
# with the streaming figure, the pipe5 kernel trace + PMC passes, then the
# config-5 (video4k) line and profile when VIDEO is set.  Every GPU step has its own time limit.
set -o pipefail
TAG=${1:-r03g}
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1 || { echo "FAILED: $*"; tail -40 "gpurun_out/$log"; exit 21; }; tail -1 "gpurun_out/$log" | cut -c1-900; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu_${TAG}.log | tail -15
[ $rc -le 1 ] || { echo "pytest died rc=$rc"; exit 20; }
run 300 smoke_${TAG}.log python -c "import __graft_entry__ as g; g.smoke()"
run 400 bench_${TAG}_pipe5.json.log python bench.py --stream
bash tools/gpu_prof2.sh ${TAG}_pipe5 pipe5 4096 || exit 26
[ -n "$VIDEO" ] && run 400 bench_${TAG}_video4k.json.log python bench.py --workload video4k
[ -n "$VIDEO" ] && { bash tools/gpu_prof2.sh ${TAG}_video4k video4k 256 || exit 27; }
echo session done
