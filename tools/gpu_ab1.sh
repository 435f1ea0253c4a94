set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "pipe" -x -q --timeout 180 --timeout-method thread > gpurun_out/pt_new.log 2>&1 || { tail -30 gpurun_out/pt_new.log; exit 21; }
tail -1 gpurun_out/pt_new.log
IPP_LIB_PATH=$PWD/variants/nw8/libipp.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "pipe" -x -q --timeout 180 --timeout-method thread > gpurun_out/pt_nw8.log 2>&1 || { tail -30 gpurun_out/pt_nw8.log; exit 22; }
tail -1 gpurun_out/pt_nw8.log
bash tools/ab.sh "" old base early nw8 old base early nw8
