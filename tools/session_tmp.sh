set -o pipefail
mkdir -p gpurun_out/r05o
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -k "video or keep_largest" -x -q --timeout 240 --timeout-method thread > gpurun_out/r05o/pt.log 2>&1 || { tail -30 gpurun_out/r05o/pt.log; exit 21; }
tail -1 gpurun_out/r05o/pt.log
