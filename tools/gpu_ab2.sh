set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab.sh "" old base liveskip oldnobreak old base liveskip oldnobreak || exit 20
bash tools/gpu_pmcprobe.sh probe1 old base || exit $?
