"""ctypes binding of the node-local spin barrier (mpxb_spin_*, host/mpx_boot.h
in lib/libmpx_host.so) for bench.py's N > 1 path: the barrier in front of
every timed loop (the reference's MPI_Barrier, mpi_perf.c:499).  gloo's
barrier is a TCP round trip: ranks leave it tens of microseconds apart, and
each rank's timer starts at its own exit, so short loops (run-hbv3.sh's
-i 10) carried that skew; the spin barrier in shared memory lets them leave
within about a microsecond, as MPI's intra-node barrier does.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "libmpx_host.so")
_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        L = C.CDLL(LIB_PATH)
        L.mpxb_spin_open.restype = C.c_int
        L.mpxb_spin_open.argtypes = [C.POINTER(C.c_void_p), C.c_char_p, C.c_int, C.c_int]
        L.mpxb_spin_wait.restype = C.c_int
        L.mpxb_spin_wait.argtypes = [C.c_void_p, C.c_double]
        L.mpxb_spin_wait_xfer.restype = C.c_int
        L.mpxb_spin_wait_xfer.argtypes = [C.c_void_p, C.c_double, C.c_void_p, C.c_void_p] + [C.c_int] * 5 + [
            C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_int)]
        L.mpxb_spin_close.restype = None
        L.mpxb_spin_close.argtypes = [C.c_void_p, C.c_int]
        L.mpxb_error.restype = C.c_char_p
        _lib = L
    return _lib


class SpinBarrier:
    """`nranks` processes of one node; `name` a POSIX shm name ("/x"); one
    rank creates it (create=True) before the others open it."""

    def __init__(self, name: str, nranks: int, create: bool):
        self.h = C.c_void_p()
        if lib().mpxb_spin_open(C.byref(self.h), name.encode(), nranks, 1 if create else 0) != 0:
            raise OSError(lib().mpxb_error().decode())

    def wait(self, timeout_s: float = 180.0) -> None:
        if lib().mpxb_spin_wait(self.h, timeout_s) != 0:
            raise TimeoutError(lib().mpxb_error().decode())

    def wait_then(self, fn, ctx, mode, group, rank, peer, iters, tx, rx, length, opts, timing,
                  timeout_s: float = 180.0) -> int:
        """wait, then fn(ctx, ..., opts, timing) from C with nothing in
        between (mpxb_spin_wait_xfer); fn's return code"""
        rc = C.c_int(0)
        if lib().mpxb_spin_wait_xfer(self.h, timeout_s, fn, ctx, mode, group, rank, peer, iters, tx, rx, length,
                                     opts, timing, C.byref(rc)) != 0:
            raise TimeoutError(lib().mpxb_error().decode())
        return rc.value

    def close(self) -> None:
        if self.h:
            lib().mpxb_spin_close(self.h, 0)
            self.h = C.c_void_p()


def unlink(name: str) -> None:
    """remove the shm name (every rank keeps its mapping)"""
    try:
        os.unlink("/dev/shm" + name)
    except FileNotFoundError:
        pass
