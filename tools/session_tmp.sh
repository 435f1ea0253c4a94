set -o pipefail
mkdir -p gpurun_out/r05m
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_benchscale.py -k "pipe or benchscale" -x -q --timeout 240 --timeout-method thread > gpurun_out/r05m/pt.log 2>&1 || { tail -30 gpurun_out/r05m/pt.log; exit 21; }
tail -1 gpurun_out/r05m/pt.log
export IPP_LIB_PATH=$PWD/variants/vdb2/libipp.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_benchscale.py -k "pipe or benchscale" -x -q --timeout 240 --timeout-method thread > gpurun_out/r05m/pt_vdb2.log 2>&1 || { tail -30 gpurun_out/r05m/pt_vdb2.log; exit 22; }
tail -1 gpurun_out/r05m/pt_vdb2.log
unset IPP_LIB_PATH
timeout -k 10 800 bash tools/ab.sh "--steps 20 --warmup 5" base vdb2 base vdb2 base vdb2 > gpurun_out/r05m/ab.txt 2>&1; cat gpurun_out/r05m/ab.txt
