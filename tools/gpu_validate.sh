#!/bin/bash
# Bit-exact payload validation sweep on one GPU with the drop-in host:
# mpx_perf -c 2 (seeded per-(src,dst,run) patterns, every received payload
# checksummed) over 1 B .. 64 MiB for each engine x mode, one loopback pair,
# then four concurrent pairs; summary rows in gpurun_out/validate_summary.csv.
set -o pipefail
mkdir -p gpurun_out/validate
rm -rf gpurun_out/validate/*
echo vm > gpurun_out/validate/group1
for eng in kernel sdma; do
  for m in pp uni nb; do
    flag=""; [ $m = uni ] && flag="-u 1"; [ $m = nb ] && flag="-x 1"
    MPX_PROCESSOR_NAMES=vm,runsc timeout -k 10 240 mpi-perf_amd/bin/mpx_perf -w 2 -g 0,0 -e $eng -c 2 -t 10000 \
      -f gpurun_out/validate/group1 -n 1 -p 1 -r 2 -i 7 -S 1:67108864 $flag -l gpurun_out/validate/${eng}_$m \
      > gpurun_out/validate/${eng}_$m.log 2>&1 || { echo "FAIL $eng $m"; exit 1; }
  done
  MPX_PROCESSOR_NAMES=vm,vm,vm,vm,runsc,runsc,runsc,runsc timeout -k 10 240 mpi-perf_amd/bin/mpx_perf -w 8 -g 0,0,0,0,0,0,0,0 \
    -e $eng -c 2 -t 10000 -f gpurun_out/validate/group1 -n 1 -p 4 -u 1 -r 2 -i 7 -S 1024:4194304 \
    -l gpurun_out/validate/${eng}_4pairs > gpurun_out/validate/${eng}_4pairs.log 2>&1 || { echo "FAIL $eng 4pairs"; exit 1; }
done
python - <<'PY'
import csv, glob, os
rows = []
for d in sorted(glob.glob("gpurun_out/validate/*/")):
    tag = os.path.basename(d.rstrip("/"))
    for f in sorted(glob.glob(d + "gpu-*.csv")):
        for r in csv.DictReader(open(f)):
            rows.append(dict(run=tag, engine=r["Engine"], mode=r["Mode"], rank=r["Rank"], bytes=r["BufferSize"],
                             iters=r["NumOfBuffers"], protocol=r["Protocol"], checked=r["CheckedPayloads"],
                             failures=r["CheckFailures"], GBps=r["GBps"], run_id=r["RunId"]))
with open("gpurun_out/validate_summary.csv", "w") as out:
    w = csv.DictWriter(out, fieldnames=list(rows[0]))
    w.writeheader()
    w.writerows(rows)
bad = [r for r in rows if r["failures"] != "0"]
print(f"{len(rows)} transfer records, {sum(int(r['checked']) for r in rows)} payloads checked, {len(bad)} with failures")
PY
