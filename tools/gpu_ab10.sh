set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in b44 m0; do
  IPP_LIB_PATH=$PWD/variants/$v/libipp.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "pipe" -q --timeout 180 --timeout-method thread > gpurun_out/pt_$v.log 2>&1
  echo "$v $(tail -1 gpurun_out/pt_$v.log)"
done
bash tools/ab.sh "" base b44 m0 base b44 m0 || exit 20
bash tools/gpu_pmcprobe.sh probe4 b44 || exit $?
