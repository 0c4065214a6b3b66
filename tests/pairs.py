"""Pairs of ranks of one process, for the -m gpu tests.

`npairs` pairs in the reference's -p layout (mpi_perf.c:437-450 with ppn =
npairs): ranks [0, np) are group 1, ranks [np, 2np) group 0, rank k is paired
with np + k.  Each rank runs its side of the loop on a host thread of its own,
like one MPI rank each.

`devs` maps rank -> GPU.  The default puts every rank on GPU 0 (loopback
pairs: the kernel, mailbox protocol and sequence bookkeeping of the cross-GPU
path, with the peer's HBM being local HBM); `cross_gpu_devs()` puts every
rank on a GPU of its own, so each pair moves its bytes over xGMI.
"""
from __future__ import annotations

import os
import threading

import mpx

def rehearsing() -> bool:
    """MPX_MULTI_REHEARSE=1: run the multi-GPU tests' code on one GPU (every
    rank on GPU 0) to shake out the tests themselves.  Read per call: on a
    one-GPU box tests/test_gpu_multi.py sets it per test (a fixture), so the
    driver's `pytest -m gpu` runs that rehearsal; subprocess workers inherit
    it through the environment."""
    return bool(os.environ.get("MPX_MULTI_REHEARSE"))


def cross_gpu_devs(nranks: int) -> list[int] | None:
    """rank r on GPU r, or None when fewer than nranks GPUs are visible
    (rehearsal: every rank on GPU 0)"""
    if rehearsing():
        return [0] * nranks
    return list(range(nranks)) if mpx.device_count() >= nranks else None


class Pairs:
    def __init__(self, engine, npairs, cap, fill="compat", devs=None):
        self.c = mpx.Context(2 * npairs, engine)
        self.np = npairs
        self.cap = cap
        self.devs = list(devs) if devs is not None else [0] * (2 * npairs)
        assert len(self.devs) == 2 * npairs
        self.bufs = []
        for r in range(2 * npairs):
            d = self.devs[r]
            tx, rx = self.c.alloc(d, cap), self.c.alloc(d, cap)
            if fill == "compat":   # mpi_perf.c:244-251: group 0 'a', group 1 'b'
                self.c.fill(tx, cap, mpx.FILL_BYTE, ord("b") if r < npairs else ord("a"))
            else:
                self.c.fill(tx, cap, mpx.FILL_SPLITMIX, mpx.pattern_key(mpx.PATTERN_SEED, r, 0, 0))
            self.c.fill(rx, cap, mpx.FILL_BYTE, 0)
            self.c.attach(r, d, tx, rx, cap)
            self.bufs.append((tx, rx))
        if self.c.engine == mpx.ENGINE_RCCL:
            self.c.rccl_init_all()

    def peer(self, r):
        return r + self.np if r < self.np else r - self.np

    def group(self, r):
        return 1 if r < self.np else 0

    def expect(self, r, n):
        tx = self.bufs[self.peer(r)][0]
        return self.c.checksum(tx, n), self.c.checksum(tx, 1)

    def run(self, mode, n, iters, check=True, timeout_ms=10000, ranks=None, nwg=0, stream=False, pull=False,
            armed=False):
        """every rank's side on a thread of its own; armed: each side arms
        its call (mpx_xfer_arm), all sides meet at a barrier (the hosts'
        mpi_perf.c:499), then start it"""
        ranks = list(range(2 * self.np)) if ranks is None else ranks
        exp = {r: self.expect(r, n) for r in ranks}
        out, errs = {}, {}
        bar = threading.Barrier(len(ranks))

        def side(r):
            kw = dict(check_payload=check, expect=exp[r][0], expect_ack=exp[r][1], timeout_ms=timeout_ms, nwg=nwg,
                      stream=stream, pull=pull)
            args = (mode, self.group(r), r, self.peer(r), iters, self.bufs[r][0], self.bufs[r][1], n)
            try:
                if armed:
                    self.c.arm(*args, **kw)
                    bar.wait()
                out[r] = self.c.xfer(*args, **kw)
            except mpx.MpxError as e:
                errs[r] = e
                if armed:
                    bar.abort()

        th = [threading.Thread(target=side, args=(r,)) for r in ranks]
        for t in th:
            t.start()
        for t in th:
            t.join()
        return out, errs

    def close(self):
        self.c.close()
