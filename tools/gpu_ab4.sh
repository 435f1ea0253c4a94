set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab.sh "" old q22 asmg asmgq old q22 asmg asmgq || exit 20
