set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab.sh "" prev base prev base || exit 20
