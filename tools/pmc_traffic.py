"""Per-launch HBM traffic from rocprofv3 PMC passes → profiles/pmc_traffic.json.

Input: a tools/profile.sh output directory holding the separate `fetch`
(--pmc FETCH_SIZE) and `write` (--pmc WRITE_SIZE) passes of one bench
command.  Units and corrections (MI355X_MICROARCH.md §HBM): rocprofv3
reports both counters in KiB; on gfx950 FETCH_SIZE tallies half the bytes
of wide coalesced streaming reads, so it is doubled.  Infinity-cache hits
are counted by these memory-side counters, so the figure is an upper
bound on true HBM bytes.

  python tools/pmc_traffic.py <profile_dir> <workload> <batch> [profiles/pmc_traffic.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = {  # C-ABI entry point → predicate on the (demangled) device kernel name
    "ipp_pipe_hpass_bgcopy": lambda k: "k_pipe_hpass" in k,
    "ipp_pipe_vblend_bands": lambda k: "k_pipe_vblend" in k,
    "ipp_rotate_flip_nearest": lambda k: "k_rotate_flip_nearest" in k,
    "ipp_video_keep_largest": lambda k: "k_ccl" in k or "k_video" in k,
}


def per_dispatch(d: str, counter: str):
    vals = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            vals[r["Kernel_Name"]][r.get("Dispatch_Id", r.get("Correlation_Id", ""))] += float(r["Counter_Value"])
    return vals


def main():
    prof, workload, batch = sys.argv[1], sys.argv[2], int(sys.argv[3])
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join("profiles", "pmc_traffic.json")
    fetch = per_dispatch(os.path.join(prof, "fetch"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(prof, "write"), "WRITE_SIZE")
    res = {"_batch": batch}
    for api, sym in KERNELS.items():
        fk = [k for k in fetch if sym(k)]
        wk = [k for k in write if sym(k)]
        if not fk or not wk:
            continue
        # one entry point may launch several kernels (ipp_video_keep_largest):
        # per kernel the mean over its dispatches, summed over the kernels
        f_bytes = 2 * 1024 * sum(sum(fetch[k].values()) / len(fetch[k]) for k in fk)
        w_bytes = 1024 * sum(sum(write[k].values()) / len(write[k]) for k in wk)
        res[api] = {"hbm_bytes": int(f_bytes + w_bytes), "fetch_bytes_x2": int(f_bytes), "write_bytes": int(w_bytes),
                    "kernels": len(fk), "dispatches": sum(len(fetch[k]) for k in fk)}
    data = json.load(open(out)) if os.path.exists(out) else {}
    data[workload] = res
    json.dump(data, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
