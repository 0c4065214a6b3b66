"""Diagnostic: repeated context lifecycles with IPC imports, one process per
rank, every rank on GPU 0 (torch.distributed.run, gloo for the exchange).
Reports which call fails in which cycle."""
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import torch.distributed as dist  # noqa: E402

import mpx  # noqa: E402

dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
nbytes = 4 << 20
for cyc, engine in enumerate(["kernel", "sdma", "kernel", "sdma"]):
    err, step = "", "create"
    c = None
    try:
        c = mpx.Context(world, engine)
        step = "alloc"
        tx, rx = c.alloc(0, nbytes), c.alloc(0, nbytes)
        step = "fill"
        c.fill(tx, nbytes, mpx.FILL_BYTE, 0x61 + rank)
        step = "attach"
        c.attach(rank, 0, tx, rx, nbytes)
        step = "export"
        d = c.export(rank)
    except Exception as e:  # noqa: BLE001
        err = f"{step}: {e}"
        d = None
    descs = [None] * world
    dist.all_gather_object(descs, d)
    if not err and all(descs):
        try:
            step = "import"
            for r in range(world):
                if r != rank:
                    c.import_rank(r, descs[r])
        except Exception as e:  # noqa: BLE001
            err = f"{step}: {e}"
    if not err and engine == "kernel":
        try:  # a few transfers, as the bench does before closing
            step = "xfer"
            peer = rank ^ 1
            c.xfer(mpx.MODE_UNIDIR, 1 if rank % 2 == 0 else 0, rank, peer, 10, tx, rx, nbytes)
        except Exception as e:  # noqa: BLE001
            err = f"{step}: {e}"
    print(f"cycle {cyc} {engine} rank {rank} rx=0x{rx.ptr if c else 0:x} -> {err or 'ok'}", flush=True)
    dist.barrier()
    if c is not None:
        try:
            c.close()
        except Exception:  # noqa: BLE001
            traceback.print_exc()
    if os.environ.get("DIAG_BARRIER_AFTER_CLOSE", "1") == "1":
        dist.barrier()
dist.destroy_process_group()
