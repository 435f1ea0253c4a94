set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_transforms_gpu.py tests/test_gpu_dropin.py -k "rotat or flip or gather or rgba or window" -q --timeout 180 --timeout-method thread > gpurun_out/pt_rot.log 2>&1
echo "rot $(tail -1 gpurun_out/pt_rot.log)"; grep FAILED gpurun_out/pt_rot.log | head
bash tools/ab.sh "--workload rotflip --batch 1024" rot2 base rot2 base || exit 20
