set -o pipefail
mkdir -p gpurun_out/r05v
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_benchscale.py -k "pipe or benchscale" -x -q --timeout 240 --timeout-method thread > gpurun_out/r05v/pt.log 2>&1 || { tail -30 gpurun_out/r05v/pt.log; exit 21; }
tail -1 gpurun_out/r05v/pt.log
for v in w4h1 w4h2; do
export IPP_LIB_PATH=$PWD/variants/$v/libipp.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_benchscale.py -k "pipe or benchscale" -x -q --timeout 240 --timeout-method thread > gpurun_out/r05v/pt_$v.log 2>&1 || { tail -30 gpurun_out/r05v/pt_$v.log; exit 22; }
tail -1 gpurun_out/r05v/pt_$v.log
done
unset IPP_LIB_PATH
timeout -k 10 800 bash tools/ab.sh "--steps 20 --warmup 5" base w4h1 w4h2 base w4h1 w4h2 > gpurun_out/r05v/ab.txt 2>&1; cat gpurun_out/r05v/ab.txt
