set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
IPP_LIB_PATH=$PWD/variants/w6/libipp.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "keep_largest or video" -q --timeout 180 --timeout-method thread > gpurun_out/pt_w6.log 2>&1
echo "w6 $(tail -1 gpurun_out/pt_w6.log)"
bash tools/ab.sh "--workload video4k" base w6 w8 base w6 w8 || exit 20
