"""One rank of the 2-process IPC test (tests/test_gpu_ipc.py).

Each process owns one mpx context with one local rank on GPU 0, exports its
descriptor to a file, imports the other rank's, then runs every loop mode
with every payload checksummed.  Results go to <dir>/result_<rank>.json.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402


# 8191 / 8192 / 8193: both sides of the cross-GPU LL threshold (ll_max_bytes)
SIZES = (1, 8, 4097, 8191, 8192, 8193, 65541, 1 << 20)


def main():
    d, rank = sys.argv[1], int(sys.argv[2])
    engine = sys.argv[3] if len(sys.argv) > 3 else "kernel"
    pull = engine.endswith("-pull")   # kernel-pull / sdma-pull: that engine in pull mode (MPX_XFER_PULL)
    engine = engine[:-len("-pull")] if pull else engine
    # "cross": rank r on GPU r (the pair moves its bytes over xGMI); else GPU 0
    dev = rank if len(sys.argv) > 4 and sys.argv[4] == "cross" and not os.environ.get("MPX_MULTI_REHEARSE") else 0
    peer = 1 - rank
    group = 1 if rank == 0 else 0
    cap = 1 << 20
    c = mpx.Context(2, engine)
    tx, rx = c.alloc(dev, cap), c.alloc(dev, cap)
    c.fill(tx, cap, mpx.FILL_SPLITMIX, mpx.pattern_key(mpx.PATTERN_SEED, rank, peer, 0))
    c.attach(rank, dev, tx, rx, cap)
    with open(os.path.join(d, f"desc_{rank}.tmp"), "wb") as f:
        f.write(c.export(rank))
    os.rename(os.path.join(d, f"desc_{rank}.tmp"), os.path.join(d, f"desc_{rank}.bin"))
    # my tx checksums, for the peer's expectations
    sums = {str(n): c.checksum(tx, n) for n in SIZES}
    with open(os.path.join(d, f"sums_{rank}.tmp"), "w") as f:
        json.dump(sums, f)
    os.rename(os.path.join(d, f"sums_{rank}.tmp"), os.path.join(d, f"sums_{rank}.json"))
    t0 = time.time()
    while not (os.path.exists(os.path.join(d, f"desc_{peer}.bin")) and os.path.exists(os.path.join(d, f"sums_{peer}.json"))):
        if time.time() - t0 > 60:
            raise SystemExit("peer never published its descriptor")
        time.sleep(0.01)
    c.import_rank(peer, open(os.path.join(d, f"desc_{peer}.bin"), "rb").read())
    peer_sums = json.load(open(os.path.join(d, f"sums_{peer}.json")))
    results = []
    for mode in (mpx.MODE_PINGPONG, mpx.MODE_UNIDIR, mpx.MODE_NONBLOCKING):
        for n in SIZES:
            iters = 300 if mode == mpx.MODE_NONBLOCKING else 9
            t = c.xfer(mode, group, rank, peer, iters, tx, rx, n, check_payload=True,
                       expect=peer_sums[str(n)], expect_ack=peer_sums["1"], timeout_ms=5000, pull=pull)
            m = 1 if (mode == mpx.MODE_UNIDIR and group == 1) else n
            results.append(dict(mode=mode, n=n, iters=iters, check_iters=t.check_iters,
                                check_failures=t.check_failures, recv_done=t.recv_done,
                                final_rx_ok=c.checksum(rx, m) == peer_sums[str(m)], protocol=t.protocol,
                                us_per_iter=t.wall_s / iters * 1e6))
    with open(os.path.join(d, f"result_{rank}.json"), "w") as f:
        json.dump(results, f)
    c.close()


if __name__ == "__main__":
    main()
