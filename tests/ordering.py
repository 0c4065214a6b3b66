"""Cross-call ordering scenarios (tests/test_gpu_ordering.py), shared by the
threads form (two ranks of one context) and the processes form
(tests/order_worker.py, one context per process, ranks mapped over IPC).

The reference's rx is written only under a posted receive: a payload of the
next loop can land only after the receiver's next MPI_Recv / MPI_Irecv
(/root/reference/mpi_perf.c:75,79,100,104,137,141).  In libmpx the receiver's
call posts its receives (Mailbox.posted) and the sender's first push of a call
waits for that post.  Two scenarios check it, each with rank 0 racing ahead of
rank 1 between two calls and changing its payload (pattern A, then B):

* race: rank 1 sleeps between the calls and then reads rx on the host; it
  must still hold call 1's last payload (pattern A), and after call 2 the
  new one (pattern B).
* lag: the non-blocking loop in check mode; one of rank 1's workgroups stalls
  (MPX_TEST lag_wg=...) before it checks call 1's last receive, and call 2 changes
  the length and the push width, so its chunks and receive slots cover bytes
  the stalled workgroup still owns under call 1's layout.  Every payload of
  both calls must pass its checksum.

Both run in pull mode too (`pull=True`, MPX_XFER_PULL): there the stalled
workgroup has not yet LOADED call 1's last payload from rank 0's tx when rank 0
would like to return and rewrite tx; rank 0's call must wait for it (MPI_Send's
buffer-reuse rule), so the lag scenario checks the sender side's order.
"""
from __future__ import annotations

import time

import mpx

CAP = 1 << 20
# call 2 of the lag scenario: another length (ragged) and width than call 1's
LAG_N1, LAG_N2, LAG_NWG2 = CAP, CAP - 4083, 8
LAG_ITERS = 300
LAG_US = 300_000
# rank 1's last workgroup of call 1 (-1: counted from the last; 1 MiB is 64
# workgroups of 16 KiB within one GPU, 32 of 32 KiB across GPUs, bulk_nwg);
# call 2's last workgroup (7 of 8) covers its bytes
LAG_WG = -1
RACE_DELAY_S = 0.3
SIZES = (1, 1024, 4097, 65536 + 13, 262144 + 13, LAG_N1, LAG_N2)


def lag_env(extra: str = "") -> dict:
    """libmpx's fault injection for the lag scenario (MPX_TEST lag_wg=...),
    plus `extra` knobs (e.g. "no_posted")"""
    return {"MPX_TEST": ",".join(x for x in (f"lag_wg=1:{LAG_WG}:{LAG_US}", extra) if x)}


def key(rank: int, peer: int, it: int) -> int:
    return mpx.pattern_key(mpx.PATTERN_SEED, rank, peer, it)


def pattern_sums(c: mpx.Context, scratch: mpx.Buffer, rank: int, peer: int) -> dict:
    """checksums of rank's patterns A (it 0) and B (it 1) at every size, keyed 'it:n'"""
    out = {}
    for it in (0, 1):
        c.fill(scratch, CAP, mpx.FILL_SPLITMIX, key(rank, peer, it))
        for n in SIZES:
            out[f"{it}:{n}"] = c.checksum(scratch, n)
    return out


def lag(c: mpx.Context, rank: int, tx: mpx.Buffer, rx: mpx.Buffer, peer_sums: dict, pull: bool = False) -> dict:
    peer, group = 1 - rank, 1 if rank == 0 else 0
    res = {}
    try:
        t = c.xfer(mpx.MODE_NONBLOCKING, group, rank, peer, LAG_ITERS, tx, rx, LAG_N1, check_payload=True,
                   expect=peer_sums[f"0:{LAG_N1}"], timeout_ms=10000, pull=pull)
        res["call1"] = dict(ok=True, check_iters=t.check_iters, nwg=t.nwg)
    except mpx.MpxError as e:
        res["call1"] = dict(ok=False, error=str(e))
    if rank == 0:
        c.fill(tx, CAP, mpx.FILL_SPLITMIX, key(0, 1, 1))
    it = 1 if rank == 1 else 0          # rank 1 receives rank 0's new pattern
    try:
        t = c.xfer(mpx.MODE_NONBLOCKING, group, rank, peer, LAG_ITERS, tx, rx, LAG_N2, check_payload=True,
                   expect=peer_sums[f"{it}:{LAG_N2}"], timeout_ms=10000, nwg=LAG_NWG2, pull=pull)
        res["call2"] = dict(ok=True, check_iters=t.check_iters, nwg=t.nwg)
    except mpx.MpxError as e:
        res["call2"] = dict(ok=False, error=str(e))
    return res


def race(c: mpx.Context, rank: int, tx: mpx.Buffer, rx: mpx.Buffer, peer_sums: dict, mode: int, check: bool,
         n: int, iters: int, pull: bool = False) -> dict:
    peer, group = 1 - rank, 1 if rank == 0 else 0
    m = 1 if (mode == mpx.MODE_UNIDIR and group == 1) else n   # what this rank receives
    res = {}
    for call in (1, 2):
        it = 1 if (rank == 1 and call == 2) else 0
        try:
            c.xfer(mode, group, rank, peer, iters, tx, rx, n, check_payload=check, expect=peer_sums[f"{it}:{n}"],
                   expect_ack=peer_sums["0:1"], timeout_ms=10000, pull=pull)
            res[f"call{call}"] = dict(ok=True)
        except mpx.MpxError as e:
            res[f"call{call}"] = dict(ok=False, error=str(e))
        if call == 1:
            if rank == 0:
                c.fill(tx, CAP, mpx.FILL_SPLITMIX, key(0, 1, 1))   # race ahead with a new payload
            else:
                time.sleep(RACE_DELAY_S)
                res["rx_between_is_call1"] = c.checksum(rx, m) == peer_sums[f"0:{m}"]
    res["rx_after_is_call2"] = c.checksum(rx, m) == peer_sums[f"{1 if rank == 1 else 0}:{m}"]
    return res
