#!/bin/bash
# Quick A/B session: pipe parity tests, then bench lines for the given
# variants: "[<variant library>[@VAR=val,...]|]<bench.py args>" (a library path
# runs that experiment build through IPP_LIB_PATH; @ exports its env vars).  tools/gpu_ab.sh <tag> "<A>" "<B>" ...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_benchscale.py tests/test_transforms_gpu.py -k "${PT:-pipe or benchscale}" -x -q --timeout 240 --timeout-method thread > gpurun_out/pt_${TAG}.log 2>&1 || { tail -30 gpurun_out/pt_${TAG}.log; exit 21; }
tail -1 gpurun_out/pt_${TAG}.log
i=0
for a in "$@"; do
  lib=""; args="$a"; envs=""
  case "$a" in *"|"*) lib="${a%%|*}"; args="${a#*|}";; esac
  case "$lib" in *"@"*) envs="${lib#*@}"; lib="${lib%%@*}";; esac
  if [ -n "$lib" ]; then export IPP_LIB_PATH=$lib IPP_AB_EXPERIMENT=1; else unset IPP_LIB_PATH IPP_AB_EXPERIMENT; fi
  timeout -k 10 300 env ${envs//,/ } python bench.py --no-cpu-baseline $args > gpurun_out/bench_${TAG}_$i.json.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_$i.json.log; exit 22; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['value'], d['kernels_ms'])" gpurun_out/bench_${TAG}_$i.json.log "$a"
  i=$((i+1))
done
