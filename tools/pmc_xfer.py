"""Workloads for rocprofv3 --pmc passes over the pair kernel k_xfer, sized so
one launch moves `iters` pushes of B bytes (DESIGN.md §7 "Counter evidence").

  self <variant> <B> <iters>
      one rank paired with itself on GPU 0: the non-blocking loop as ONE
      kernel (k_xfer<1,0>, or k_xfer_nbcheck with check) — nothing for the
      profiler's dispatch serialisation to deadlock.  variant: nb (bulk, LDS-
      staged tx), nb_hbm (bulk, tx read from HBM: the call flag
      MPX_XFER_NOSTAGE), nbcheck (bulk + every payload checksummed and poisoned),
      nbpull / nbpullcheck (pull mode, MPX_XFER_PULL: k_xfer_pull loads its
      own tx every iteration — whether each iteration's bytes come from
      memory or from the L2 is what FETCH_SIZE shows).
  pair <dir> <rank> <mode> <B> <iters> <check> [pull]
      rank 0 or 1 of a loopback pair in two processes (IPC, like
      tests/ipc_worker.py); only rank 0 runs under the profiler, so its
      dispatch window spans the whole co-running loop and the device-wide
      TCC counters see both halves' traffic (a pair total).  mode: pingpong |
      unidir; B <= 2 KiB on one GPU is the LL protocol.

Each workload makes 3 identical calls (the first is a warm-up); the summary
(tools/pmc_xfer_summary.py) takes the median of the k_xfer dispatches.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402

MODES = {"pingpong": mpx.MODE_PINGPONG, "unidir": mpx.MODE_UNIDIR, "nonblocking": mpx.MODE_NONBLOCKING}


def self_pair(variant, B, iters):
    with mpx.Context(1, "kernel") as c:
        tx, rx = c.alloc(0, max(B, 1)), c.alloc(0, max(B, 1))
        c.fill(tx, B, mpx.FILL_SPLITMIX, 99)
        c.attach(0, 0, tx, rx, max(B, 1))
        want = c.checksum(tx, B)
        check = variant in ("nbcheck", "nbpullcheck")
        pull = variant.startswith("nbpull")
        for _ in range(3):
            t = c.xfer(mpx.MODE_NONBLOCKING, 0, 0, 0, iters, tx, rx, B, check_payload=check, expect=want, pull=pull,
                       stage=variant != "nb_hbm")
        assert c.checksum(rx, B) == want
        print(json.dumps(dict(variant=variant, bytes=B, iters=iters, nwg=t.nwg, protocol=mpx.PROTOCOLS[t.protocol],
                              us_per_push=round(t.device_s / iters * 1e6, 3), check_iters=t.check_iters)))


def pair(d, rank, mode, B, iters, check, pull=False):
    peer = 1 - rank
    cap = max(B, 1)
    c = mpx.Context(2, "kernel")
    tx, rx = c.alloc(0, cap), c.alloc(0, cap)
    c.fill(tx, cap, mpx.FILL_SPLITMIX, mpx.pattern_key(mpx.PATTERN_SEED, rank, peer, 0))
    c.attach(rank, 0, tx, rx, cap)
    sums = (c.checksum(tx, B), c.checksum(tx, 1))
    with open(os.path.join(d, f"desc_{rank}.tmp"), "wb") as f:
        f.write(c.export(rank) + json.dumps(sums).encode().ljust(64))
    os.rename(os.path.join(d, f"desc_{rank}.tmp"), os.path.join(d, f"desc_{rank}.bin"))
    path = os.path.join(d, f"desc_{peer}.bin")
    t0 = time.time()
    while not os.path.exists(path):
        if time.time() - t0 > 60:
            raise SystemExit("peer never published its descriptor")
        time.sleep(0.01)
    blob = open(path, "rb").read()
    c.import_rank(peer, blob[:mpx.RANK_DESC_BYTES])
    peer_sums = json.loads(blob[mpx.RANK_DESC_BYTES:].decode().strip())
    group = 1 if rank == 0 else 0
    for _ in range(3):
        t = c.xfer(MODES[mode], group, rank, peer, iters, tx, rx, B, check_payload=check, expect=peer_sums[0],
                   expect_ack=peer_sums[1], timeout_ms=20000, pull=pull)
    print(json.dumps(dict(mode=mode, rank=rank, bytes=B, iters=iters, check=check,
                          protocol=mpx.PROTOCOLS[t.protocol], nwg=t.nwg,
                          us_per_iter=round(t.device_s / iters * 1e6, 3), check_iters=t.check_iters)))
    c.close()


if __name__ == "__main__":
    if sys.argv[1] == "self":
        self_pair(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
    else:
        pair(sys.argv[2], int(sys.argv[3]), sys.argv[4], int(sys.argv[5]), int(sys.argv[6]), sys.argv[7] == "1",
             len(sys.argv) > 8 and sys.argv[8] == "pull")
    # every context is finalized: the pooled rank streams go before exit (a
    # profiler's exit-time finalizer faulted on them: r04_exit_segv_stack.txt)
    mpx.shutdown()
