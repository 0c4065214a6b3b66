"""ctypes binding of libmpx (include/mpx.h) for tests and bench.py.

This is plumbing over the C-ABI, not a second implementation: every call goes
to lib/libmpx.so, and importing this module fails loudly if the library is
missing (there is no CPU fallback — the CPU restatement lives in oracle/ and is
only ever used as a checker).

Reference mapping: see include/mpx.h (each entry point cites the
/root/reference/mpi_perf.c call it replaces).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
# MPX_LIB: load another build of the library (A/B of two builds in tools/)
LIB_PATH = os.environ.get("MPX_LIB") or os.path.join(PKG_ROOT, "lib", "libmpx.so")
HEADER_PATH = os.path.join(os.path.dirname(PKG_ROOT), "include", "mpx.h")

# enum values (include/mpx.h)
OK, ERR_INVALID, ERR_HIP, ERR_NOMEM, ERR_TIMEOUT, ERR_RCCL, ERR_UNSUPPORTED, ERR_STATE, ERR_CHECK = range(9)
ENGINE_KERNEL, ENGINE_SDMA, ENGINE_RCCL = 0, 1, 2
ENGINE_HOST = 3   # reserved: mpx_init refuses it, MPX_ERR_UNSUPPORTED
ENGINES = {"kernel": ENGINE_KERNEL, "sdma": ENGINE_SDMA, "rccl": ENGINE_RCCL}
MODE_PINGPONG, MODE_NONBLOCKING, MODE_UNIDIR = 0, 1, 2
MODES = {"pingpong": MODE_PINGPONG, "nonblocking": MODE_NONBLOCKING, "unidir": MODE_UNIDIR}
FILL_BYTE, FILL_SPLITMIX = 0, 1
XFER_STREAM = 1
XFER_PULL = 2
XFER_NOSTAGE = 4
ABI_VERSION = 7
PATTERN_SEED = 0x6D70695F70657266
MAX_RANKS = 64
RANK_DESC_BYTES = 512
RCCL_ID_BYTES = 128
PROTOCOLS = {0: "ll", 1: "bulk", 2: "sdma", 3: "rccl", 4: "copy", 5: "copy_steps", 6: "copy_pipe", 7: "pull", 8: "sdma_pull"}


class Timing(C.Structure):
    _fields_ = [
        ("wall_s", C.c_double),
        ("device_s", C.c_double),
        ("bytes", C.c_uint64),
        ("launches", C.c_int32),
        ("nwg", C.c_int32),
        ("protocol", C.c_int32),
        ("check_failures", C.c_int32),
        ("check_iters", C.c_uint64),
        ("recv_done", C.c_uint64),
        ("recv_digest", C.c_uint64),
    ]

    def as_dict(self) -> dict:
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["protocol"] = PROTOCOLS.get(self.protocol, self.protocol)
        return d


class XferOpts(C.Structure):
    _fields_ = [
        ("check", C.c_int32),
        ("flags", C.c_int32),
        ("expect_checksum", C.c_uint64),
        ("expect_ack", C.c_uint64),
        ("timeout_ms", C.c_uint32),
        ("nwg", C.c_int32),
    ]


class Phases(C.Structure):
    _fields_ = ([(k, C.c_double) for k in ("wall_s", "host_prep_s", "launch_to_start_s", "posted_wait_s", "kernel_s",
                                            "done_to_return_s")]
                + [("armed", C.c_int32), ("resident", C.c_int32), ("first_iter_s", C.c_double), ("tail_s", C.c_double)])

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


def pattern_key(seed: int, src: int, dst: int, it: int) -> int:
    """mpx_pattern_key (include/mpx.h)."""
    return (seed ^ (src << 56) ^ (dst << 48) ^ (it << 24)) & 0xFFFFFFFFFFFFFFFF


_SIGS = {
    "mpx_version": (C.c_int, []),
    "mpx_strerror": (C.c_char_p, [C.c_int]),
    "mpx_last_error": (C.c_char_p, []),
    "mpx_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "mpx_link_info": (C.c_int, [C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "mpx_device_bus_id": (C.c_int, [C.c_int, C.c_char_p, C.c_int]),
    "mpx_last_phases": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(Phases)]),
    "mpx_init": (C.c_int, [C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    "mpx_finalize": (C.c_int, [C.c_void_p]),
    "mpx_shutdown": (C.c_int, []),
    "mpx_live_events": (C.c_int, [C.POINTER(C.c_int)]),
    "mpx_alloc": (C.c_int, [C.c_void_p, C.c_int, C.c_size_t, C.POINTER(C.c_void_p)]),
    "mpx_free": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mpx_fill": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t, C.c_int, C.c_uint64]),
    "mpx_checksum": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t, C.POINTER(C.c_uint64)]),
    "mpx_read": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_size_t]),
    "mpx_copy": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.POINTER(Timing)]),
    "mpx_rank_attach": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_size_t]),
    "mpx_rank_export": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p]),
    "mpx_rank_import": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p]),
    "mpx_xfer": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                           C.c_int, C.POINTER(C.c_double)]),
    "mpx_xfer_ex": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                              C.c_int, C.POINTER(XferOpts), C.POINTER(Timing)]),
    "mpx_xfer_prepare": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                   C.POINTER(XferOpts)]),
    "mpx_xfer_arm": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                               C.c_int, C.POINTER(XferOpts)]),
    "mpx_xfer_disarm": (C.c_int, [C.c_void_p, C.c_int]),
    "mpx_barrier": (C.c_int, [C.c_void_p, C.c_int]),
    "mpx_rccl_version": (C.c_int, [C.POINTER(C.c_int), C.c_char_p, C.c_int]),
    "mpx_rccl_get_unique_id": (C.c_int, [C.c_void_p]),
    "mpx_rccl_init_rank": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    "mpx_rccl_init_all": (C.c_int, [C.c_void_p]),
}

_lib = None


def lib() -> C.CDLL:
    """Load lib/libmpx.so (raises if it was not built: no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libmpx not built: {LIB_PATH} missing (run __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.mpx_version() != ABI_VERSION:
            raise ImportError(f"{LIB_PATH}: ABI version {L.mpx_version()}, this binding needs {ABI_VERSION} "
                              "(stale build: run __graft_entry__.build())")
        _lib = L
    return _lib


class MpxError(RuntimeError):
    def __init__(self, status: int, what: str):
        self.status = status
        L = lib()
        super().__init__(f"{what}: {L.mpx_strerror(status).decode()} ({L.mpx_last_error().decode()})")


def check(status: int, what: str) -> None:
    if status != OK:
        raise MpxError(status, what)


def device_count() -> int:
    n = C.c_int(0)
    check(lib().mpx_device_count(C.byref(n)), "mpx_device_count")
    return n.value


LINK_TYPES = {0: "hypertransport", 1: "qpi", 2: "pcie", 3: "infiniband", 4: "xgmi"}


def link_info(dev_a: int, dev_b: int) -> dict:
    """mpx_link_info: the interconnect between two visible GPUs."""
    t, h = C.c_int(0), C.c_int(0)
    check(lib().mpx_link_info(dev_a, dev_b, C.byref(t), C.byref(h)), "mpx_link_info")
    return {"type": LINK_TYPES.get(t.value, t.value), "hops": h.value}


def shutdown() -> None:
    """mpx_shutdown: destroy the pooled rank streams (no context alive)."""
    check(lib().mpx_shutdown(), "mpx_shutdown")


def live_events() -> int:
    """mpx_live_events: HIP events libmpx holds right now (leak check)."""
    n = C.c_int(0)
    check(lib().mpx_live_events(C.byref(n)), "mpx_live_events")
    return n.value


def bus_id(dev: int) -> str:
    """mpx_device_bus_id: the GPU's PCI bus id, "DDDD:BB:DD.F"."""
    buf = C.create_string_buffer(64)
    check(lib().mpx_device_bus_id(dev, buf, 64), "mpx_device_bus_id")
    return buf.value.decode()


@dataclass
class Buffer:
    ptr: int
    dev: int
    size: int


class Context:
    """Thin object wrapper of an mpx_ctx."""

    def __init__(self, nranks: int, engine: int | str = ENGINE_KERNEL):
        if isinstance(engine, str):
            engine = ENGINES[engine]
        self.L = lib()
        self.h = C.c_void_p()
        check(self.L.mpx_init(nranks, engine, C.byref(self.h)), "mpx_init")
        self.nranks = nranks
        self.engine = engine

    def close(self) -> None:
        if self.h:
            check(self.L.mpx_finalize(self.h), "mpx_finalize")
            self.h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # buffers
    def alloc(self, dev: int, size: int) -> Buffer:
        p = C.c_void_p()
        check(self.L.mpx_alloc(self.h, dev, size, C.byref(p)), "mpx_alloc")
        return Buffer(p.value, dev, size)

    def free(self, b: Buffer) -> None:
        check(self.L.mpx_free(self.h, C.c_void_p(b.ptr)), "mpx_free")

    def fill(self, b: Buffer, n: int, pattern: int, arg: int) -> None:
        check(self.L.mpx_fill(self.h, b.dev, C.c_void_p(b.ptr), n, pattern, arg & 0xFFFFFFFFFFFFFFFF), "mpx_fill")

    def checksum(self, b: Buffer, n: int, offset: int = 0) -> int:
        out = C.c_uint64()
        check(self.L.mpx_checksum(self.h, b.dev, C.c_void_p(b.ptr + offset), n, C.byref(out)), "mpx_checksum")
        return out.value

    def read(self, b: Buffer, n: int, offset: int = 0) -> bytes:
        buf = C.create_string_buffer(max(n, 1))
        check(self.L.mpx_read(self.h, b.dev, buf, C.c_void_p(b.ptr + offset), n), "mpx_read")
        return buf.raw[:n]

    def copy(self, dev: int, dst: Buffer, src: Buffer, n: int, iters: int) -> Timing:
        t = Timing()
        check(self.L.mpx_copy(self.h, dev, C.c_void_p(dst.ptr), C.c_void_p(src.ptr), n, iters, C.byref(t)), "mpx_copy")
        return t

    # ranks
    def attach(self, rank: int, dev: int, tx: Buffer, rx: Buffer, length: int) -> None:
        check(self.L.mpx_rank_attach(self.h, rank, dev, C.c_void_p(tx.ptr), C.c_void_p(rx.ptr), length),
              "mpx_rank_attach")

    def export(self, rank: int) -> bytes:
        buf = C.create_string_buffer(RANK_DESC_BYTES)
        check(self.L.mpx_rank_export(self.h, rank, buf), "mpx_rank_export")
        return buf.raw

    def import_rank(self, rank: int, desc: bytes) -> None:
        buf = C.create_string_buffer(bytes(desc), RANK_DESC_BYTES)
        check(self.L.mpx_rank_import(self.h, rank, buf), "mpx_rank_import")

    def xfer(self, mode: int, group: int, my_rank: int, peer_rank: int, iters: int, tx: Buffer, rx: Buffer,
             length: int, check_payload: bool = False, expect: int = 0, expect_ack: int = 0,
             timeout_ms: int = 0, nwg: int = 0, stream: bool = False, pull: bool = False,
             stage: bool = True, after=None) -> Timing:
        """mpx_xfer_ex.  after: a spin barrier (mpx.spin.SpinBarrier) to wait
        on first, from C, so the call starts right as the barrier opens"""
        flags = (XFER_STREAM if stream else 0) | (XFER_PULL if pull else 0) | (0 if stage else XFER_NOSTAGE)
        o = XferOpts(check=1 if check_payload else 0, flags=flags, expect_checksum=expect,
                     expect_ack=expect_ack, timeout_ms=timeout_ms, nwg=nwg)
        t = Timing()
        if after is not None:
            st = after.wait_then(C.cast(self.L.mpx_xfer_ex, C.c_void_p), self.h, mode, group, my_rank, peer_rank,
                                 iters, C.c_void_p(tx.ptr), C.c_void_p(rx.ptr), length, C.byref(o), C.byref(t))
        else:
            st = self.L.mpx_xfer_ex(self.h, mode, group, my_rank, peer_rank, iters, C.c_void_p(tx.ptr),
                                    C.c_void_p(rx.ptr), length, C.byref(o), C.byref(t))
        check(st, "mpx_xfer_ex")
        return t

    def arm(self, mode: int, group: int, my_rank: int, peer_rank: int, iters: int, tx: Buffer, rx: Buffer,
            length: int, check_payload: bool = False, expect: int = 0, expect_ack: int = 0, timeout_ms: int = 0,
            nwg: int = 0, stream: bool = False, pull: bool = False, stage: bool = True) -> None:
        """mpx_xfer_arm: launch the next xfer with these arguments now; the
        xfer call with the same arguments starts it (kernel engine)"""
        flags = (XFER_STREAM if stream else 0) | (XFER_PULL if pull else 0) | (0 if stage else XFER_NOSTAGE)
        o = XferOpts(check=1 if check_payload else 0, flags=flags, expect_checksum=expect,
                     expect_ack=expect_ack, timeout_ms=timeout_ms, nwg=nwg)
        check(self.L.mpx_xfer_arm(self.h, mode, group, my_rank, peer_rank, iters, C.c_void_p(tx.ptr),
                                  C.c_void_p(rx.ptr), length, C.byref(o)), "mpx_xfer_arm")

    def disarm(self, rank: int) -> None:
        check(self.L.mpx_xfer_disarm(self.h, rank), "mpx_xfer_disarm")

    def prepare(self, mode: int, group: int, my_rank: int, peer_rank: int, iters: int, length: int,
                timeout_ms: int = 0, pull: bool = False) -> None:
        """mpx_xfer_prepare: before timing, build the SDMA engine's graph chunks
        (pull: its pulled form's) or set up the RCCL engine's channel to
        peer_rank (both ranks call it)"""
        o = XferOpts(timeout_ms=timeout_ms, flags=XFER_PULL if pull else 0)
        check(self.L.mpx_xfer_prepare(self.h, mode, group, my_rank, peer_rank, iters, length, C.byref(o)),
              "mpx_xfer_prepare")

    def phases(self, rank: int) -> dict:
        """mpx_last_phases: where rank's last kernel-engine call spent its time"""
        p = Phases()
        check(self.L.mpx_last_phases(self.h, rank, C.byref(p)), "mpx_last_phases")
        return p.as_dict()

    def rccl_init_all(self) -> None:
        check(self.L.mpx_rccl_init_all(self.h), "mpx_rccl_init_all")

    def rccl_init_rank(self, rank: int, nranks: int, uid: bytes) -> None:
        buf = C.create_string_buffer(bytes(uid), RCCL_ID_BYTES)
        check(self.L.mpx_rccl_init_rank(self.h, rank, nranks, buf), "mpx_rccl_init_rank")


def rccl_version() -> dict:
    """mpx_rccl_version: the RCCL this process runs and where it came from"""
    v, buf = C.c_int(0), C.create_string_buffer(512)
    check(lib().mpx_rccl_version(C.byref(v), buf, 512), "mpx_rccl_version")
    x = v.value
    return {"version": x, "release": f"{x // 10000}.{x // 100 % 100}.{x % 100}", "library": buf.value.decode()}


def rccl_unique_id() -> bytes:
    buf = C.create_string_buffer(RCCL_ID_BYTES)
    check(lib().mpx_rccl_get_unique_id(buf), "mpx_rccl_get_unique_id")
    return buf.raw


def header_symbols(path: str = HEADER_PATH) -> list[str]:
    """Every function name include/mpx.h declares (for the export test)."""
    import re

    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_]+\s*\*?\s*(mpx_[a-z_0-9]+)\s*\(", txt, flags=re.M)
    return sorted(set(n for n in names if n != "mpx_pattern_key"))
