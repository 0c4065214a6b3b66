"""In-process counter probe (libmpxprof, mpx/counters.py) on one GPU: does the
device counting service initialise in THIS process, in which load order
relative to torch, and do its numbers agree with the rocprofv3 --pmc passes
committed in profiles/pmc_local_d2d_copy.json (k_copy 1 GiB: 1.0004 x
algorithmic) and profiles/r02_pmc_xfer_ea.json (a loopback push writes one
64-B request per 64 B pushed, all to local DRAM)?

    python tools/counters_probe.py torch_first | prof_first | no_torch [shutdown] [nopair]

shutdown: mpx_shutdown() (pooled rank streams destroyed) before exit.
nopair: the copy passes only (no rank attached: no rank streams exist).

Prints one JSON line.
"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))

order = sys.argv[1]
out = {"order": order}
from mpx import counters  # noqa: E402  (no HIP)

if order == "torch_first":
    import torch  # noqa: F401
try:
    counters.register()
    out["register"] = "ok"
except counters.CounterError as e:
    out["register"] = str(e)
if order == "prof_first":
    import torch  # noqa: F401
import mpx  # noqa: E402

if order != "no_torch":
    torch.cuda.set_device(0)
    torch.cuda.synchronize()
mpx.device_count()
out["ready"] = counters.ready()
out["error"] = counters.error()
bus = mpx.bus_id(0)
out["bus"] = bus

N = 1 << 30
COPIES = 30
with mpx.Context(2, "kernel") as c:
    src, dst = c.alloc(0, N), c.alloc(0, N)
    c.fill(src, N, mpx.FILL_SPLITMIX, 7)
    c.copy(0, dst, src, N, 3)
    res = {}
    for name in ("FETCH_SIZE", "WRITE_SIZE", "TCC_EA0_RDREQ_sum,TCC_EA0_WRREQ_sum,TCC_EA0_WRREQ_64B_sum"):
        try:
            t0 = time.perf_counter()
            with counters.Pass(bus, name.split(",")) as p:
                t = c.copy(0, dst, src, N, COPIES)
            res[name] = dict(values=p.values, reads_reset=p.reads_reset, launches=t.launches,
                             pass_s=round(time.perf_counter() - t0, 3))
        except Exception as e:  # noqa: BLE001
            res[name] = f"{type(e).__name__}: {e}"
    out["copy_1GiB_x30"] = res
    try:
        f = res["FETCH_SIZE"]["values"][0] * 1024 * 2 / COPIES     # FETCH_SIZE KiB, x2 (MI355X_MICROARCH.md HBM)
        w = res["WRITE_SIZE"]["values"][0] * 1024 / COPIES
        out["copy_traffic_per_launch"] = f + w
        out["copy_traffic_over_algorithmic"] = round((f + w) / (2 * N), 5)
    except Exception as e:  # noqa: BLE001
        out["copy_traffic_error"] = str(e)
    c.free(src)
    c.free(dst)
    # a loopback pair (two ranks on GPU 0, one thread each): unidir 4 MiB x 500
    B, IT = 4 << 20, (0 if "nopair" in sys.argv[2:] else 500)
    bufs = []
    for r in range(2 if IT else 0):
        tx, rx = c.alloc(0, B), c.alloc(0, B)
        c.fill(tx, B, mpx.FILL_SPLITMIX, r + 1)
        c.attach(r, 0, tx, rx, B)
        bufs.append((tx, rx))

    def run_pair(iters):
        errs = []

        def side(r):
            try:
                c.xfer(mpx.MODE_UNIDIR, 1 - r, r, 1 - r, iters, bufs[r][0], bufs[r][1], B)
            except Exception as e:  # noqa: BLE001
                errs.append(str(e))
        th = [threading.Thread(target=side, args=(r,)) for r in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errs, errs

    if IT:
        run_pair(20)
    try:
        assert IT, "nopair: no rank streams in this process"
        with counters.Pass(bus, ["TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum", "TCC_EA0_WRREQ_DRAM_sum"]) as p:
            run_pair(IT)
        wr, w64, dram = p.values
        out["pair_unidir_4MiB_x500"] = dict(values=p.values, reads_reset=p.reads_reset,
                                            wrreq_64B_bytes_over_pushed=round(w64 * 64 / (B * IT), 5),
                                            dram_req_over_wrreq=round(dram / wr, 5) if wr else None,
                                            link_req=wr - dram)
    except Exception as e:  # noqa: BLE001
        out["pair_unidir_4MiB_x500"] = f"{type(e).__name__}: {e}"
if "shutdown" in sys.argv[2:]:
    mpx.shutdown()
    out["shutdown"] = "pooled rank streams destroyed before exit"
print(json.dumps(out), flush=True)
