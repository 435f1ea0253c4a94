set -o pipefail
mkdir -p gpurun_out/r05d
export TMPDIR=/tmp
timeout -k 10 1000 bash tools/ab.sh "--steps 20 --warmup 5" r4base g8s8 g8s4 g8s6 g12s8 g8s8vb3 r4base g8s8 g8s4 g8s6 g12s8 g8s8vb3 > gpurun_out/r05d/ab.txt 2>&1; cat gpurun_out/r05d/ab.txt
