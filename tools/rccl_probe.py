"""Does RCCL accept two ranks (two processes) on one GPU?  Worker mode:
rccl_probe.py <dir> <rank>."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-perf_amd"))
import mpx  # noqa: E402

d, rank = sys.argv[1], int(sys.argv[2])
c = mpx.Context(2, "rccl")
tx, rx = c.alloc(0, 1 << 20), c.alloc(0, 1 << 20)
c.fill(tx, 1 << 20, mpx.FILL_BYTE, 98 - rank)
c.attach(rank, 0, tx, rx, 1 << 20)
if rank == 0:
    open(os.path.join(d, "uid.tmp"), "wb").write(mpx.rccl_unique_id())
    os.rename(os.path.join(d, "uid.tmp"), os.path.join(d, "uid"))
while not os.path.exists(os.path.join(d, "uid")):
    time.sleep(0.01)
c.rccl_init_rank(rank, 2, open(os.path.join(d, "uid"), "rb").read())
t = c.xfer(2, 1 - rank, rank, 1 - rank, 10, tx, rx, 1 << 20)
print(f"rank {rank}: rccl unidir ok {t.wall_s / 10 * 1e6:.1f} us/iter; rx ok:",
      c.checksum(rx, 1 if rank == 0 else 1 << 20) != 0, flush=True)
c.close()
