set -o pipefail
mkdir -p gpurun_out/r05p
export TMPDIR=/tmp
export IPP_LIB_PATH=$PWD/variants/cx3/libipp.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -k "video or keep_largest" -x -q --timeout 240 --timeout-method thread > gpurun_out/r05p/pt.log 2>&1 || { tail -30 gpurun_out/r05p/pt.log; exit 21; }
tail -1 gpurun_out/r05p/pt.log
unset IPP_LIB_PATH
timeout -k 10 600 bash tools/ab.sh "--workload video4k --steps 20 --warmup 5" base cx3 base cx3 > gpurun_out/r05p/ab.txt 2>&1; cat gpurun_out/r05p/ab.txt
