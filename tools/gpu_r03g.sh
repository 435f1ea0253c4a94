#!/bin/bash
# Round-3 checkpoint session: the whole GPU suite, smoke, the default bench
# line with the streaming figure, then the pipe5 kernel trace + PMC passes.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
TAG=${1:-r03g}
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1 || { echo "FAILED: $*"; tail -40 "gpurun_out/$log"; exit 21; }; tail -1 "gpurun_out/$log" | cut -c1-900; }
[ -x tools/probes/gather_probe ] && run 120 gather_probe_${TAG}.txt tools/probes/gather_probe
run 900 pytest_gpu_${TAG}.log python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread
run 300 smoke_${TAG}.log python -c "import __graft_entry__ as g; g.smoke()"
run 400 bench_${TAG}_pipe5.json.log python bench.py --stream
bash tools/gpu_prof2.sh ${TAG}_pipe5 pipe5 4096 || exit 26
echo session done
