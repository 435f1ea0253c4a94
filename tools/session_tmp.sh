set -o pipefail
mkdir -p gpurun_out/r05q
export TMPDIR=/tmp
timeout -k 10 800 bash tools/ab.sh "--steps 20 --warmup 5" base st1 st2 st3 st16 st18 base st1 st2 st3 st16 st18 > gpurun_out/r05q/ab.txt 2>&1; cat gpurun_out/r05q/ab.txt
