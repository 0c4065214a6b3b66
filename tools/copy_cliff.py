"""Config 2's 512 KiB - 16 MiB range: where a copy's time goes (VERDICT r02,
"Next round" item 4).

    python tools/copy_cliff.py run <out.jsonl>            (on the GPU box,
        under `rocprofv3 --kernel-trace --output-format csv -d <dir> -o cliff --`)
    python tools/copy_cliff.py summary <out.jsonl> <kernel_trace.csv>

`run` measures every size with each form of mpx_copy, in two states of the
process: "fresh", and "after_headline" (200 back-to-back 1 GiB copies, the
headline's load, just before).  Per (state, size, form): one warm call, then
5 calls of 10 copies, per-copy time from HIP events (best and median).  Forms:
  steps  : all copies in one k_copy_steps launch (MPX_COPY_STEPS_MAX raised)
  launch : one k_copy launch per copy (MPX_COPY_STEPS_MAX=0)
  pipe*  : all copies in one k_copy_pipe launch (MPX_COPY_PIPE_MAX raised;
           pipeN: N units per lane)
(MPX_CLIFF_FORMS=steps,launch,pipe,... picks them; default steps,launch)
and the in-kernel shader clock (tools/libclock_probe.so: delta s_memtime /
delta s_memrealtime, MI355X_MICROARCH.md "DVFS give-back" item 6) before and
after each state: one workgroup for 2 ms, and one per CU.

`summary` walks the kernel trace in dispatch order against the schedule `run`
wrote and splits each launch-per-copy call into kernel time and the gap
between one copy's end and the next copy's start (the dispatch cost), and
each steps call into its per-copy kernel time.
"""
import ctypes
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIZES = [512 << 10, 1 << 20, 2 << 20, 3 << 20, 4 << 20, 8 << 20, 16 << 20]
# form -> environment of mpx_copy (read per call); MPX_CLIFF_FORMS=a,b,... selects
FORMS = {
    "steps": {"MPX_COPY_STEPS_MAX": str(16 << 20), "MPX_COPY_PIPE_MAX": "0"},
    "launch": {"MPX_COPY_STEPS_MAX": "0", "MPX_COPY_PIPE_MAX": "0"},
    "pipe": {"MPX_COPY_PIPE_MAX": str(16 << 20), "MPX_COPY_PIPE_UPL": ""},
    "pipe2": {"MPX_COPY_PIPE_MAX": str(16 << 20), "MPX_COPY_PIPE_UPL": "2"},
    "pipe8": {"MPX_COPY_PIPE_MAX": str(16 << 20), "MPX_COPY_PIPE_UPL": "8"},
    "pipe16": {"MPX_COPY_PIPE_MAX": str(16 << 20), "MPX_COPY_PIPE_UPL": "16"},
}
CALLS, COPIES, WARM = 5, 10, 2
EMPTY, EMPTY_COUNT = ((1, 64), (128, 256), (1024, 256), (4096, 256)), 20   # (grid, lanes) of empty launches
G = 1 << 30


def run(out_path):
    sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
    import mpx

    probe = ctypes.CDLL(os.path.join(ROOT, "tools", "libclock_probe.so"))
    probe.clock_probe.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    probe.empty_kernels.argtypes = [ctypes.c_int] * 4

    def clock(wgs):
        g = ctypes.c_double(0)
        rc = probe.clock_probe(0, 2.0, wgs, ctypes.byref(g))
        return round(g.value, 3) if rc == 0 else f"rc {rc}"

    out = open(out_path, "w")

    def emit(d):
        out.write(json.dumps(d) + "\n")
        out.flush()
        print(json.dumps(d), flush=True)

    schedule = []
    with mpx.Context(1) as c:
        src, dst = c.alloc(0, G), c.alloc(0, G)
        c.fill(src, G, mpx.FILL_SPLITMIX, 11)
        for state in ("fresh", "after_headline"):
            if state == "after_headline":
                os.environ.update(FORMS["launch"])
                for _ in range(20):
                    c.copy(0, dst, src, G, 10)
                schedule.append(dict(state=state, what="headline", dispatches=200))
            emit(dict(state=state, clock_ghz_1wg=clock(1), clock_ghz_per_cu=clock(256)))
            for grid, threads in EMPTY:
                probe.empty_kernels(0, grid, threads, EMPTY_COUNT)
            schedule.append(dict(state=state, what="empty"))
            for n in SIZES:
                for form in os.environ.get("MPX_CLIFF_FORMS", "steps,launch").split(","):
                    for k, v in FORMS[form].items():
                        os.environ[k] = v
                    c.copy(0, dst, src, n, WARM)
                    per = []
                    for _ in range(CALLS):
                        t = c.copy(0, dst, src, n, COPIES)
                        per.append(t.device_s / COPIES)
                    assert c.checksum(dst, n) == c.checksum(src, n), (n, form)
                    path = mpx.PROTOCOLS.get(t.protocol, t.protocol)
                    schedule.append(dict(state=state, n=n, form=form, path=path, grid=t.nwg))
                    emit(dict(state=state, bytes=n, form=form, path=path, grid=t.nwg,
                              us_per_copy_best=round(min(per) * 1e6, 3),
                              us_per_copy_median=round(statistics.median(per) * 1e6, 3)))
            emit(dict(state=state, clock_ghz_1wg_after=clock(1), clock_ghz_per_cu_after=clock(256)))
    out.write(json.dumps(dict(schedule=schedule)) + "\n")
    out.close()


def summary(lab_path, trace_path):
    lines = [json.loads(x) for x in open(lab_path)]
    schedule = next(x["schedule"] for x in lines if "schedule" in x)
    every = sorted(csv.DictReader(open(trace_path)), key=lambda r: int(r["Dispatch_Id"]))
    rows = [r for r in every if "k_copy" in r["Kernel_Name"]]
    empty = [r for r in every if "k_empty" in r["Kernel_Name"]]
    k = 0
    res = []
    for item in schedule:
        if item.get("what") == "headline":
            k += item["dispatches"]
            continue
        if item.get("what") == "empty":
            mine, empty = empty[:len(EMPTY) * EMPTY_COUNT], empty[len(EMPTY) * EMPTY_COUNT:]
            for j, (grid, threads) in enumerate(EMPTY):
                d = mine[j * EMPTY_COUNT:(j + 1) * EMPTY_COUNT]
                dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in d]
                gap = [(int(d[i + 1]["Start_Timestamp"]) - int(d[i]["End_Timestamp"])) / 1e3 for i in range(len(d) - 1)]
                res.append(dict(state=item["state"], empty_kernel=dict(grid=grid, lanes=threads),
                                kernel_us_median=round(statistics.median(dur), 3),
                                gap_us_median=round(statistics.median(gap), 3)))
            continue
        steps = item["path"] in ("copy_steps", "copy_pipe")
        calls = []
        for copies in [WARM] + [COPIES] * CALLS:
            nd = 1 if steps else copies
            d = rows[k:k + nd]
            k += nd
            assert all(("k_copy_steps" in r["Kernel_Name"] or "k_copy_pipe" in r["Kernel_Name"]) == steps
                       for r in d), (item, d[0]["Kernel_Name"])
            s = [int(r["Start_Timestamp"]) for r in d]
            e = [int(r["End_Timestamp"]) for r in d]
            calls.append(dict(copies=copies, span_ns=e[-1] - s[0], kernel_ns=[b - a for a, b in zip(s, e)],
                              gaps_ns=[s[i + 1] - e[i] for i in range(len(d) - 1)]))
        timed = calls[1:]
        per_copy = [cl["span_ns"] / COPIES / 1e3 for cl in timed]
        kern = [x / (COPIES if steps else 1) / 1e3 for cl in timed for x in cl["kernel_ns"]]
        gaps = [x / 1e3 for cl in timed for x in cl["gaps_ns"]]
        res.append(dict(state=item["state"], bytes=item["n"], form=item["form"], grid=item["grid"],
                        trace_us_per_copy_best=round(min(per_copy), 3),
                        trace_us_per_copy_median=round(statistics.median(per_copy), 3),
                        kernel_us_per_copy_median=round(statistics.median(kern), 3),
                        gap_us_median=round(statistics.median(gaps), 3) if gaps else None,
                        gap_share=round(statistics.median(gaps) / statistics.median(per_copy), 3) if gaps else None))
    assert k == len(rows), (k, len(rows))
    for r in res:
        print(json.dumps(r))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        summary(sys.argv[2], sys.argv[3])
