set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "keep_largest or video" -q --timeout 180 --timeout-method thread > gpurun_out/pt_ccl.log 2>&1
echo "ccl $(tail -1 gpurun_out/pt_ccl.log)"
bash tools/ab.sh "--workload video4k" cclold base cclold base || exit 20
