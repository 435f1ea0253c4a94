set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base e2; do
  lib=$PWD/image_processor_pipeline_amd/libipp.so; [ $v != base ] && lib=$PWD/variants/$v/libipp.so
  IPP_LIB_PATH=$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "pipe" -x -q --timeout 180 --timeout-method thread > gpurun_out/pt_$v.log 2>&1 || { tail -30 gpurun_out/pt_$v.log; exit 21; }
  echo "$v $(tail -1 gpurun_out/pt_$v.log)"
done
bash tools/ab.sh "" old base e2 old base e2 || exit 20
