#!/bin/bash
# Profile-only GPU session: tools/profile.sh on the default bench, summaries
# and PMC traffic; per-dispatch counter CSVs are removed afterwards.
set -o pipefail
TAG=${1:-prof}
shift
bash tools/profile.sh $TAG "$@" || exit 25
python tools/prof_summary.py gpurun_out/$TAG > gpurun_out/$TAG/summary.txt
python tools/pmc_traffic.py gpurun_out/$TAG pipe5 4096 gpurun_out/pmc_traffic.json
find gpurun_out/$TAG -name '*counter_collection.csv' -size +4M -delete
du -sh gpurun_out
cat gpurun_out/$TAG/summary.txt
