"""Summarise tools/gpu.sh pmc_xfer's passes into profiles/r02_pmc_xfer.json:
HBM bytes per push (per iteration for the pair cases) of the pair kernel,
against its B.  FETCH_SIZE is doubled and WRITE_SIZE taken as is
(MI355X_MICROARCH.md §HBM, gfx950); both are the L2's memory-side request
counters, device-wide, so a pair case counts both halves' traffic.

    python tools/pmc_xfer_summary.py gpurun_out/<tag> profiles/<round>_pmc_xfer.json

(cases are the pmc_<name>_{FETCH,WRITE}_SIZE pass directories with their
.log; other passes in the same directory, e.g. the bench's, are skipped)
"""
import csv
import glob
import json
import os
import re
import statistics
import sys


def kb(path, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if "k_xfer" in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return statistics.median(vals), len(vals), sorted({r["Kernel_Name"].split("(")[0] for r in csv.DictReader(open(path))
                                                       if "k_xfer" in r["Kernel_Name"]})


def workload_line(log):
    for line in open(log):
        if line.startswith("{"):
            return json.loads(line)
    return {}


src, out = sys.argv[1], sys.argv[2]
cases = sorted({re.sub(r"_(FETCH|WRITE)_SIZE$", "", os.path.basename(d)) for d in glob.glob(os.path.join(src, "*_SIZE"))
                if os.path.isdir(d)})
res = []
for name in cases:
    f = glob.glob(os.path.join(src, f"{name}_FETCH_SIZE", "*counter_collection.csv"))
    w = glob.glob(os.path.join(src, f"{name}_WRITE_SIZE", "*counter_collection.csv"))
    if not f or not w or not os.path.exists(os.path.join(src, f"{name}_WRITE_SIZE.log")):
        continue
    fkb, nf, kname = kb(f[0], "FETCH_SIZE")
    wkb, nw, _ = kb(w[0], "WRITE_SIZE")
    wl = workload_line(os.path.join(src, f"{name}_WRITE_SIZE.log"))
    B, iters = wl["bytes"], wl["iters"]
    read_pp = 2 * fkb * 1024 / iters
    write_pp = wkb * 1024 / iters
    pair = "mode" in wl
    res.append(dict(case=name, kernel=kname, bytes=B, iters_per_launch=iters, dispatches=[nf, nw],
                    protocol=wl.get("protocol"), nwg=wl.get("nwg"), check=bool(wl.get("check", "check" in name)),
                    scope="pair (both halves, device-wide counters)" if pair else "one kernel (rank paired with itself)",
                    hbm_read_bytes_per_iter=round(read_pp, 1), hbm_write_bytes_per_iter=round(write_pp, 1),
                    read_over_B=round(read_pp / B, 3) if B else None, write_over_B=round(write_pp / B, 3) if B else None,
                    us_per_iter=wl.get("us_per_push", wl.get("us_per_iter"))))
doc = dict(source="rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes (tools/gpu.sh pmc_xfer); "
                  "FETCH_SIZE x2 per MI355X_MICROARCH.md HBM section; median of 3 dispatches of 'iters' iterations",
           cases=res)
json.dump(doc, open(out, "w"), indent=1)
for r in res:
    print(f"{r['case']:24s} B={r['bytes']:>8d} read/B={r['read_over_B']} write/B={r['write_over_B']} "
          f"us/iter={r['us_per_iter']} {r['protocol']} nwg={r['nwg']}")
