"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over
tools/pmc_copy.py into profiles/pmc_<workload>.json: HBM bytes per launch of
the copy kernel, corrected as MI355X_MICROARCH.md §HBM prescribes (gfx950
FETCH_SIZE counts 128-B streaming requests at 64 B: doubled; WRITE_SIZE
exact for 16-B-per-lane stores).  bench.py reads it as roofline.traffic."""
import csv
import json
import statistics
import sys


def per_launch(path, counter, kernel="k_copy"):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return statistics.median(vals), len(vals)


fetch_csv, write_csv, out, nbytes = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
f_kb, nf = per_launch(fetch_csv, "FETCH_SIZE")
w_kb, nw = per_launch(write_csv, "WRITE_SIZE")
read_b = 2 * f_kb * 1024
write_b = w_kb * 1024
res = {
    "workload": "local_d2d_copy", "bytes": nbytes, "kernel": "k_copy",
    "fetch_size_kb_raw": f_kb, "write_size_kb_raw": w_kb, "launches": [nf, nw],
    "hbm_read_bytes_per_launch": read_b, "hbm_write_bytes_per_launch": write_b,
    "hbm_bytes_per_launch": read_b + write_b,
    "algorithmic_bytes_per_launch": 2 * nbytes,
    "traffic_over_algorithmic": round((read_b + write_b) / (2 * nbytes), 4),
    "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), FETCH_SIZE x2 per "
              "MI355X_MICROARCH.md HBM section",
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
