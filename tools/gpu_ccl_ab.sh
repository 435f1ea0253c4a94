set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -k "video or keep_largest or ccl" -x -q --timeout 240 --timeout-method thread > gpurun_out/pt_ccl.log 2>&1 || { tail -30 gpurun_out/pt_ccl.log; exit 21; }
tail -1 gpurun_out/pt_ccl.log
for v in base vf cur base vf cur; do
  if [ $v = cur ]; then unset IPP_LIB_PATH; else export IPP_LIB_PATH=variants/$v/libipp.so; fi
  timeout -k 10 300 python bench.py --workload video4k --no-cpu-baseline > gpurun_out/bench_ccl_$v.json.log 2>&1 || { tail -20 gpurun_out/bench_ccl_$v.json.log; exit 22; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['value'], d['roofline']['frac'])" gpurun_out/bench_ccl_$v.json.log $v
done
