set -o pipefail
mkdir -p gpurun_out/r04a
export TMPDIR=/tmp
timeout -k 10 240 tools/probes/stage_probe > gpurun_out/r04a/stage_probe.txt 2>&1 || { tail -20 gpurun_out/r04a/stage_probe.txt; exit 21; }
cat gpurun_out/r04a/stage_probe.txt
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r04a/bench_pipe5.json.log 2>&1 || { tail -20 gpurun_out/r04a/bench_pipe5.json.log; exit 23; }
tail -1 gpurun_out/r04a/bench_pipe5.json.log
bash tools/gpu_pmcprobe.sh r04a base
