set -o pipefail
mkdir -p gpurun_out/r05r
export TMPDIR=/tmp
for v in tbuf vbuf; do
export IPP_LIB_PATH=$PWD/variants/$v/libipp.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_benchscale.py -k "pipe or benchscale" -x -q --timeout 240 --timeout-method thread > gpurun_out/r05r/pt_$v.log 2>&1 || { tail -30 gpurun_out/r05r/pt_$v.log; exit 21; }
tail -1 gpurun_out/r05r/pt_$v.log
done
unset IPP_LIB_PATH
timeout -k 10 800 bash tools/ab.sh "--steps 20 --warmup 5" base tbuf vbuf base tbuf vbuf > gpurun_out/r05r/ab.txt 2>&1; cat gpurun_out/r05r/ab.txt
