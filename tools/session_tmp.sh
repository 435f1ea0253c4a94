set -o pipefail
mkdir -p gpurun_out/r05w
export TMPDIR=/tmp
timeout -k 10 800 bash tools/ab.sh "--steps 20 --warmup 5" diag0 x3 nogather diag0 x3 nogather > gpurun_out/r05w/ab.txt 2>&1; cat gpurun_out/r05w/ab.txt
