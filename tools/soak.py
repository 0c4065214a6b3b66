"""Randomised soak of the kernel engine's pair protocol (push and pull, every
loop, check on and off, changing lengths and widths, tx rewritten between
calls): the class of cross-call race GPUTEST_r02 caught.  Both ranks draw the
same plan from one seed; after every call each rank compares its rx with the
peer's tx (the bytes the reference's last receive leaves in rx), and in check
mode every payload is checksummed on the device.

    python tools/soak.py threads <calls> <seed> [engine]   two ranks, one process
    python tools/soak.py procs <calls> <seed> [engine]     two processes over IPC
    python tools/soak.py worker <dir> <rank> <calls> <seed> <engine>   (one process of `procs`)

engine: kernel (default) or sdma; both with push and pull calls; half of the
calls armed (mpx_xfer_arm before the call; one in ten of those cancelled
with mpx_xfer_disarm and run unarmed).  With a
negative-control knob set (MPX_TEST=no_posted, MPX_TEST=no_pull_wait) the
soak must report failures: that is what shows it can see the races.

Prints one JSON line per form: calls run, failures (with the first few),
seconds.  Exit status 1 on any failure.
"""
import json
import os
import random
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402

CAP = (8 << 20) + 64
EDGES = [0, 1, 15, 16, 17, 2047, 2048, 2049, 4096, 8191, 8192, 8193, 65536, 65537, 456131, 1 << 20, (4 << 20) + 3,
         8 << 20]
MODES = [mpx.MODE_PINGPONG, mpx.MODE_NONBLOCKING, mpx.MODE_UNIDIR]


def plan(calls, seed, engine="kernel"):
    rng = random.Random(seed)
    out = []
    for k in range(calls):
        mode = rng.choice(MODES)
        n = rng.choice(EDGES) if rng.random() < 0.5 else rng.randint(0, 1 << rng.randint(4, 23))
        if mode == mpx.MODE_NONBLOCKING:
            iters = rng.choice([1, 2, 17, 255, 256, 257, 300]) if n <= (1 << 20) else rng.randint(1, 20)
        else:
            iters = rng.randint(1, 40) if n <= (1 << 20) else rng.randint(1, 8)
        pull = rng.random() < 0.5
        step = dict(mode=mode, n=n, iters=iters, check=rng.random() < 0.6, pull=pull,
                    nwg=rng.choice([0, 0, 1, 3, 8, 64, 128, 256]), stream=rng.random() < 0.3,
                    refill=rng.random() < 0.2, key=rng.getrandbits(32))
        # armed calls (mpx_xfer_arm, then the same call starts it), a few of
        # them cancelled first (mpx_xfer_disarm, then the call runs unarmed)
        step["armed"] = rng.random() < 0.5
        step["cancel"] = step["armed"] and rng.random() < 0.1
        out.append(step)
    return out


def run_rank(c, rank, tx, rx, steps, peer_sum):
    """one rank's side of the plan; peer_sum(k, n) -> checksum of the peer's
    tx prefix of n bytes during call k; my fills follow the plan"""
    peer, group = 1 - rank, 1 if rank == 0 else 0
    fails = []
    for k, s in enumerate(steps):
        if s["refill"]:
            c.fill(tx, CAP, mpx.FILL_SPLITMIX, mpx.pattern_key(mpx.PATTERN_SEED, rank, peer, s["key"] & 0xFFFF))
        m = 1 if (s["mode"] == mpx.MODE_UNIDIR and group == 1) else s["n"]
        kw = dict(check_payload=s["check"], expect=peer_sum(k, s["n"]), expect_ack=peer_sum(k, 1), timeout_ms=10000,
                  nwg=s["nwg"], stream=s["stream"], pull=s["pull"])
        try:
            if s.get("armed"):
                c.arm(s["mode"], group, rank, peer, s["iters"], tx, rx, s["n"], **kw)
                if s.get("cancel"):
                    c.disarm(rank)
            t = c.xfer(s["mode"], group, rank, peer, s["iters"], tx, rx, s["n"], **kw)
            if s["check"] and (t.check_failures or t.check_iters != s["iters"]):
                fails.append(dict(call=k, step=s, what="check", t=t.as_dict()))
            if c.checksum(rx, m) != peer_sum(k, m):
                fails.append(dict(call=k, step=s, what="final rx differs from the peer's tx"))
        except mpx.MpxError as e:
            fails.append(dict(call=k, step=s, what=str(e)[:300]))
            if e.status == mpx.ERR_TIMEOUT:
                break                     # the link state is unknown afterwards
    return fails


class Sums:
    """checksums of each rank's tx pattern (by fill key) at the sizes a call
    needs, computed on a scratch buffer"""

    def __init__(self, c, dev, steps):
        self.c, self.scratch = c, c.alloc(dev, CAP)
        self.cache = {}
        self.steps = steps
        self._filled = None

    def key_at(self, rank, k):
        key = None
        for j in range(k + 1):
            if self.steps[j]["refill"]:
                key = self.steps[j]["key"] & 0xFFFF
        return 0 if key is None else key

    def get(self, rank, k, n):
        key = self.key_at(rank, k)
        d = self.cache.setdefault((rank, key), {})
        if n not in d:
            if self._filled != (rank, key):
                self.c.fill(self.scratch, CAP, mpx.FILL_SPLITMIX, mpx.pattern_key(mpx.PATTERN_SEED, rank, 1 - rank, key))
                self._filled = (rank, key)
            d[n] = self.c.checksum(self.scratch, n)
        return d[n]


def threads(calls, seed, engine="kernel"):
    steps = plan(calls, seed, engine)
    t0 = time.time()
    with mpx.Context(2, engine) as c:
        bufs = []
        for r in range(2):
            tx, rx = c.alloc(0, CAP), c.alloc(0, CAP)
            c.fill(tx, CAP, mpx.FILL_SPLITMIX, mpx.pattern_key(mpx.PATTERN_SEED, r, 1 - r, 0))
            c.attach(r, 0, tx, rx, CAP)
            bufs.append((tx, rx))
        S = Sums(c, 0, steps)
        # precompute every sum the plan needs (the scratch fills must not
        # interleave with the ranks' calls)
        need = {}
        for r in range(2):
            for k, s in enumerate(steps):
                for n in (s["n"], 1):
                    need[(r, k, n)] = S.get(r, k, n)
        out = {}

        def side(r):
            out[r] = run_rank(c, r, bufs[r][0], bufs[r][1], steps, lambda k, n, p=1 - r: need[(p, k, n)])

        th = [threading.Thread(target=side, args=(r,)) for r in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    fails = out[0] + out[1]
    return dict(form="threads", engine=engine, calls=calls, seed=seed, failures=len(fails), first=fails[:4],
                seconds=round(time.time() - t0, 1))


def worker(d, rank, calls, seed, engine):
    steps = plan(calls, seed, engine)
    peer = 1 - rank
    c = mpx.Context(2, engine)
    tx, rx = c.alloc(0, CAP), c.alloc(0, CAP)
    c.fill(tx, CAP, mpx.FILL_SPLITMIX, mpx.pattern_key(mpx.PATTERN_SEED, rank, peer, 0))
    c.attach(rank, 0, tx, rx, CAP)
    S = Sums(c, 0, steps)
    need = {}
    for k, s in enumerate(steps):
        for n in (s["n"], 1):
            need[(k, n)] = S.get(peer, k, n)
    with open(os.path.join(d, f"desc_{rank}.tmp"), "wb") as f:
        f.write(c.export(rank))
    os.rename(os.path.join(d, f"desc_{rank}.tmp"), os.path.join(d, f"desc_{rank}.bin"))
    t0 = time.time()
    while not os.path.exists(os.path.join(d, f"desc_{peer}.bin")):
        if time.time() - t0 > 60:
            raise SystemExit("peer never published its descriptor")
        time.sleep(0.01)
    c.import_rank(peer, open(os.path.join(d, f"desc_{peer}.bin"), "rb").read())
    fails = run_rank(c, rank, tx, rx, steps, lambda k, n: need[(k, n)])
    with open(os.path.join(d, f"result_{rank}.json"), "w") as f:
        json.dump(fails, f)
    c.close()


def procs(calls, seed, engine="kernel"):
    import tempfile
    d = tempfile.mkdtemp(prefix="soak_")
    t0 = time.time()
    ps = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "worker", d, str(r), str(calls), str(seed),
                            engine])
          for r in (0, 1)]
    rcs = []
    for p in ps:
        try:
            rcs.append(p.wait(timeout=400))
        except subprocess.TimeoutExpired:
            p.kill()
            rcs.append(-9)
    fails = []
    for r in (0, 1):
        path = os.path.join(d, f"result_{r}.json")
        fails += json.load(open(path)) if os.path.exists(path) else [dict(rank=r, what=f"no result (rc {rcs[r]})")]
    return dict(form="procs", engine=engine, calls=calls, seed=seed, failures=len(fails), first=fails[:4], rcs=rcs,
                seconds=round(time.time() - t0, 1))


if __name__ == "__main__":
    if sys.argv[1] == "worker":
        worker(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), sys.argv[6])
        sys.exit(0)
    res = (threads if sys.argv[1] == "threads" else procs)(int(sys.argv[2]), int(sys.argv[3]),
                                                            sys.argv[4] if len(sys.argv) > 4 else "kernel")
    print(json.dumps(res), flush=True)
    sys.exit(1 if res["failures"] else 0)
