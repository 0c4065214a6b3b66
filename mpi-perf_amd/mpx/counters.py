"""ctypes binding of libmpxprof.so (include/mpxprof.h): hardware counters of
this process's own GPU work, read in-process with rocprofiler-sdk's device
counting service.  bench.py uses it to put measured HBM / xGMI bytes into
its own JSON line (north_star: "rocprof counters (achieved xGMI and HBM
GB/s)"), sampling around untimed re-runs of the timed work.

register() must run before the process's first HIP call (the tool has to be
configured before the HSA runtime starts); everything else after.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "libmpxprof.so")

_lib = None


class CounterError(RuntimeError):
    pass


def register() -> None:
    """Load libmpxprof (global symbols: rocprofiler-sdk looks the tool up in
    the process) and register it.  Raises CounterError with the SDK's reason
    (e.g. rocprofiler already configured: HIP started, or rocprofv3 owns the
    process)."""
    global _lib
    if not os.path.exists(LIB_PATH):
        raise CounterError(f"{LIB_PATH} not built")
    L = C.CDLL(LIB_PATH, mode=os.RTLD_GLOBAL | os.RTLD_NOW)
    L.mpxprof_register.restype = C.c_int
    L.mpxprof_ready.restype = C.c_int
    L.mpxprof_error.restype = C.c_char_p
    L.mpxprof_begin.restype = C.c_int
    L.mpxprof_begin.argtypes = [C.c_char_p, C.c_char_p]
    L.mpxprof_end.restype = C.c_int
    L.mpxprof_end.argtypes = [C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_int)]
    if L.mpxprof_register() != 0:
        raise CounterError(L.mpxprof_error().decode())
    _lib = L


def ready() -> bool:
    return _lib is not None and _lib.mpxprof_ready() == 1


def error() -> str:
    return _lib.mpxprof_error().decode() if _lib is not None else "libmpxprof not registered"


class Pass:
    """One counter pass: `with Pass(bus_id, ["FETCH_SIZE"]) as p: ...work...`
    then p.values (one per counter, summed over instances) and
    p.reads_reset (how this SDK's samples behave, see mpxprof_end)."""

    def __init__(self, bus_id: str, counters: list[str]):
        self.bus_id, self.counters = bus_id, list(counters)
        self.values: list[float] | None = None
        self.reads_reset: int | None = None

    def __enter__(self):
        if _lib is None:
            raise CounterError("libmpxprof not registered")
        if _lib.mpxprof_begin(self.bus_id.encode(), ",".join(self.counters).encode()) != 0:
            raise CounterError(error())
        return self

    def __exit__(self, exc_type, *rest):
        vals = (C.c_double * len(self.counters))()
        reset = C.c_int(-1)
        rc = _lib.mpxprof_end(vals, len(self.counters), C.byref(reset))
        if exc_type is None:
            if rc != 0:
                raise CounterError(error())
            self.values, self.reads_reset = list(vals), reset.value
        return False
