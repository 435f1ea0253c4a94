set -o pipefail
mkdir -p gpurun_out/r05a
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_benchscale.py tests/test_gpu_taps.py -k "pipe or benchscale or taps" -x -q --timeout 240 --timeout-method thread > gpurun_out/r05a/pt.log 2>&1 || { tail -30 gpurun_out/r05a/pt.log; exit 21; }
tail -1 gpurun_out/r05a/pt.log
timeout -k 10 900 bash tools/ab.sh "--steps 20 --warmup 5" r4base base g16 g4 g8s16 g8u2 vb3 r4base base > gpurun_out/r05a/ab.txt 2>&1; cat gpurun_out/r05a/ab.txt
timeout -k 10 400 bash tools/ab.sh "--workload rotflip --steps 20 --warmup 5" r4base base r4base base > gpurun_out/r05a/ab_rot.txt 2>&1; cat gpurun_out/r05a/ab_rot.txt
