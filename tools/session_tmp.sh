set -o pipefail
mkdir -p gpurun_out/r05j
export TMPDIR=/tmp
for rep in 1 2; do
for c in 0 32 64 128 256 512; do
  echo -n "chunk=$c " >> gpurun_out/r05j/ab.txt
  timeout -k 10 200 bash tools/ab.sh "--steps 10 --warmup 3 --chunk $c" base >> gpurun_out/r05j/ab.txt 2>&1 || exit 3
done; done
cat gpurun_out/r05j/ab.txt
