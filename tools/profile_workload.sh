#!/bin/bash
# Profile one bench workload (kernel trace + PMC passes) and record its PMC
# traffic: tools/profile_workload.sh <tag> <workload> <batch-or-frames> [bench args...]
set -o pipefail
TAG=$1; WL=$2; NB=$3; shift 3
export TMPDIR=/tmp
bash tools/profile.sh $TAG --workload $WL --steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling "$@" || exit 25
python tools/prof_summary.py gpurun_out/$TAG > gpurun_out/$TAG/summary.txt
python tools/pmc_traffic.py gpurun_out/$TAG $WL $NB gpurun_out/pmc_traffic.json
# raw per-dispatch counters and agent listings: summarised above, not kept
find gpurun_out/$TAG \( -name "*_agent_info.csv" -o -name "*counter_collection.csv" \) -delete
