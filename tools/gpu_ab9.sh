set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base d3; do
  lib=$PWD/image_processor_pipeline_amd/libipp.so; [ $v != base ] && lib=$PWD/variants/$v/libipp.so
  IPP_LIB_PATH=$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "pipe" -q --timeout 180 --timeout-method thread > gpurun_out/pt_$v.log 2>&1
  echo "$v $(tail -1 gpurun_out/pt_$v.log)"
done
bash tools/ab.sh "" base d3 base d3 || exit 20
