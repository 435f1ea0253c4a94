set -o pipefail
mkdir -p gpurun_out/r04b
export TMPDIR=/tmp
timeout -k 10 240 tools/probes/pair_probe > gpurun_out/r04b/pair_probe.txt 2>&1 || { tail -20 gpurun_out/r04b/pair_probe.txt; exit 21; }
cat gpurun_out/r04b/pair_probe.txt
for v in 0 1 2; do
  timeout -s KILL 60 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum --output-format csv -d gpurun_out/r04b/pmc$v -o p -- tools/probes/pair_probe $v > gpurun_out/r04b/pmc$v.log 2>&1 || exit 31
done
bash tools/ab.sh "--steps 10 --warmup 3" base tapsc1 copysc1 bothsc1 base 2>&1 | tee gpurun_out/r04b/ab.txt
