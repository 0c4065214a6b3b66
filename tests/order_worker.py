"""One rank of the two-process ordering tests (tests/test_gpu_ordering.py).

argv: <dir> <rank> <engine> <scenario> [mode check n iters]
engine "kernel-pull": the kernel engine in pull mode (MPX_XFER_PULL).
Each process owns one context with one rank on GPU 0, exports it, imports the
other rank over IPC, runs the scenario of tests/ordering.py and writes
<dir>/result_<rank>.json.
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "mpi-perf_amd"))
sys.path.insert(0, HERE)
import mpx  # noqa: E402
import ordering as O  # noqa: E402


def publish(d, name, data: bytes):
    with open(os.path.join(d, name + ".tmp"), "wb") as f:
        f.write(data)
    os.rename(os.path.join(d, name + ".tmp"), os.path.join(d, name))


def wait_for(d, name):
    t0 = time.time()
    while not os.path.exists(os.path.join(d, name)):
        if time.time() - t0 > 60:
            raise SystemExit(f"peer never published {name}")
        time.sleep(0.01)
    return open(os.path.join(d, name), "rb").read()


def main():
    d, rank, engine, scenario = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4]
    peer = 1 - rank
    # MPX_ORDER_CROSS=1: rank r on GPU r (the pair spans GPUs, bytes over xGMI)
    dev = rank if os.environ.get("MPX_ORDER_CROSS") and not os.environ.get("MPX_MULTI_REHEARSE") else 0
    pull = engine == "kernel-pull"
    c = mpx.Context(2, "kernel" if pull else engine)
    tx, rx, scratch = c.alloc(dev, O.CAP), c.alloc(dev, O.CAP), c.alloc(dev, O.CAP)
    sums = O.pattern_sums(c, scratch, rank, peer)
    c.fill(tx, O.CAP, mpx.FILL_SPLITMIX, O.key(rank, peer, 0))
    c.fill(rx, O.CAP, mpx.FILL_BYTE, 0)
    c.attach(rank, dev, tx, rx, O.CAP)
    publish(d, f"desc_{rank}.bin", c.export(rank))
    publish(d, f"sums_{rank}.json", json.dumps(sums).encode())
    c.import_rank(peer, wait_for(d, f"desc_{peer}.bin"))
    peer_sums = json.loads(wait_for(d, f"sums_{peer}.json"))
    if scenario == "lag":
        res = O.lag(c, rank, tx, rx, peer_sums, pull=pull)
    else:
        mode, check, n, iters = (int(x) for x in sys.argv[5:9])
        res = O.race(c, rank, tx, rx, peer_sums, mode, bool(check), n, iters, pull=pull)
    publish(d, f"result_{rank}.json", json.dumps(res).encode())
    c.close()


if __name__ == "__main__":
    main()
