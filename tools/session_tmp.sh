set -o pipefail
mkdir -p gpurun_out/r05h
export TMPDIR=/tmp
timeout -k 10 600 bash tools/ab.sh "--workload video4k --steps 20 --warmup 5" cswz0 cswz2 base cswz0 cswz2 base > gpurun_out/r05h/ab.txt 2>&1; cat gpurun_out/r05h/ab.txt
