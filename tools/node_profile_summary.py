"""Summarise tools/node_profile.sh: per rank, the timed sender launches of the
pair kernel (k_xfer<unidir, G1>) — their average duration (kernel-trace pass)
and their EA write requests (PMC pass): link bytes = (WRREQ - WRREQ_DRAM) x 64,
local-HBM writes = WRREQ_DRAM x 64, against the algorithmic B x iters.

    python tools/node_profile_summary.py gpurun_out/node_prof_n<N> <N>

The timed launches of a rank are its last k sender launches (bench.py
--no-extras runs nothing after the timed steps), k = the timed steps whose
round makes it the sender (timed step s runs round s mod (N-1))."""
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
from mpx.schedule import all_pairs_rounds, round_role  # noqa: E402

SENDER = "k_xfer<2, 1>"
PULLER = "k_xfer_pull<2, 0>"   # pull passes: the receiver moves the bytes


def per_dispatch(path, kernel):
    per = {}
    for x in csv.DictReader(open(path)):
        if kernel in x["Kernel_Name"]:
            per.setdefault(int(x["Dispatch_Id"]), {})[x["Counter_Name"]] = float(x["Counter_Value"])
    return per


def bench_line(path):
    try:
        with open(path) as f:
            lines = [x for x in f.read().splitlines() if x.startswith("{")]
        return json.loads(lines[-1]) if lines else None
    except OSError:
        return None


def main():
    out_dir, n = sys.argv[1], int(sys.argv[2])
    rounds = all_pairs_rounds(n)
    line = bench_line(os.path.join(out_dir, "trace_rank0.json")) or {}
    steps = line.get("steps", 2 * (n - 1))
    B = line.get("config", {}).get("bytes", 4 << 20)
    iters = line.get("config", {}).get("iters_per_step", 500)
    ranks = []
    for r in range(n):
        timed = [s for s in range(steps) if round_role(rounds, s % (n - 1), r)[0] == 1]
        k = len(timed)
        rec = dict(rank=r, timed_sender_launches=k)
        tr = glob.glob(os.path.join(out_dir, "trace", f"rank{r}_kernel_trace.csv"))
        if tr and k:
            rows = [x for x in csv.DictReader(open(tr[0])) if SENDER in x["Kernel_Name"]]
            rows.sort(key=lambda x: int(x["Start_Timestamp"]))
            d = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) * 1e-9 for x in rows[-k:]]
            if d:
                rec["avg_launch_us"] = round(statistics.mean(d) * 1e6, 2)
                rec["algorithmic_GBps"] = round(B * iters / statistics.mean(d) / 1e9, 2)
        pm = glob.glob(os.path.join(out_dir, "pmc", f"rank{r}_counter_collection.csv"))
        if pm and k:
            per = {}
            for x in csv.DictReader(open(pm[0])):
                if SENDER in x["Kernel_Name"]:
                    per.setdefault(int(x["Dispatch_Id"]), {})[x["Counter_Name"]] = float(x["Counter_Value"])
            last = [per[i] for i in sorted(per)[-k:]]
            if last:
                wr = statistics.median(v.get("TCC_EA0_WRREQ_sum", 0) for v in last)
                dram = statistics.median(v.get("TCC_EA0_WRREQ_DRAM_sum", 0) for v in last)
                rec["link_write_bytes_per_launch"] = round((wr - dram) * 64)
                rec["local_dram_write_bytes_per_launch"] = round(dram * 64)
                rec["algorithmic_bytes_per_launch"] = B * iters
                rec["link_over_algorithmic"] = round((wr - dram) * 64 / (B * iters), 4)
                if "avg_launch_us" in rec:
                    rec["achieved_link_GBps"] = round((wr - dram) * 64 / (rec["avg_launch_us"] * 1e-6) / 1e9, 2)
        fb = glob.glob(os.path.join(out_dir, "fabric", f"rank{r}_counter_collection.csv"))
        if fb and k:
            per = {}
            for x in csv.DictReader(open(fb[0])):
                if SENDER in x["Kernel_Name"]:
                    per.setdefault(int(x["Dispatch_Id"]), {})[x["Counter_Name"]] = float(x["Counter_Value"])
            last = [per[i] for i in sorted(per)[-k:]]
            if last:
                rec["gmi_write_bytes_per_launch"] = round(
                    statistics.median(v.get("TCC_EA0_WRREQ_WRITE_GMI_32B_sum", 0) for v in last) * 32)
                rec["io_write_bytes_per_launch"] = round(
                    statistics.median(v.get("TCC_EA0_WRREQ_WRITE_IO_32B_sum", 0) for v in last) * 32)
        # pull passes: this rank's timed RECEIVER launches (rounds where it is
        # group 0) load the peer's tx over the link
        kp = sum(1 for s in range(steps) if round_role(rounds, s % (n - 1), r)[0] == 0)
        tr = glob.glob(os.path.join(out_dir, "pull_trace", f"rank{r}_kernel_trace.csv"))
        if tr and kp:
            rows = [x for x in csv.DictReader(open(tr[0])) if PULLER in x["Kernel_Name"]]
            rows.sort(key=lambda x: int(x["Start_Timestamp"]))
            d = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) * 1e-9 for x in rows[-kp:]]
            if d:
                rec["pull_avg_launch_us"] = round(statistics.mean(d) * 1e6, 2)
                rec["pull_algorithmic_GBps"] = round(B * iters / statistics.mean(d) / 1e9, 2)
        pf = glob.glob(os.path.join(out_dir, "pull_fabric", f"rank{r}_counter_collection.csv"))
        if pf and kp:
            per = per_dispatch(pf[0], PULLER)
            last = [per[i] for i in sorted(per)[-kp:]]
            if last:
                rd = statistics.median(v.get("TCC_EA0_RDREQ_sum", 0) for v in last)
                dram = statistics.median(v.get("TCC_EA0_RDREQ_DRAM_sum", 0) for v in last)
                gmi = statistics.median(v.get("TCC_EA0_RDREQ_GMI_32B_sum", 0) for v in last)
                rec["pull_gmi_read_bytes_per_launch"] = round(gmi * 32)
                rec["pull_read_requests_per_launch"] = round(rd)
                rec["pull_dram_read_requests_per_launch"] = round(dram)
                rec["pull_gmi_over_algorithmic"] = round(gmi * 32 / (B * iters), 4)
                if "pull_avg_launch_us" in rec:
                    rec["pull_achieved_link_GBps"] = round(gmi * 32 / (rec["pull_avg_launch_us"] * 1e-6) / 1e9, 2)
        ranks.append(rec)
    doc = dict(n=n, bytes=B, iters_per_step=iters, steps=steps, kernel=SENDER,
               source="tools/node_profile.sh: rocprofv3 --kernel-trace --stats, then --pmc TCC_EA0_WRREQ_sum "
                      "TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum, every rank under its own profiler",
               one_gpu_rehearsal=bool(os.environ.get("MPX_BENCH_ONE_GPU")), ranks=ranks)
    with open(os.path.join(out_dir, "summary.json"), "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc))


if __name__ == "__main__":
    main()
