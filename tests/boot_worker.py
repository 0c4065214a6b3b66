"""One rank of the mpx_boot collective test (tests/test_procs.py): joins the
job through libmpx_host.so's mpxb_* functions and prints what every
collective returned, as one JSON line.

    python boot_worker.py <rank> <size> <port> [timeout_s]
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = C.CDLL(os.path.join(ROOT, "mpi-perf_amd", "lib", "libmpx_host.so"))
L.mpxb_init.argtypes = [C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_char_p, C.c_int, C.c_double]
L.mpxb_allgather.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
L.mpxb_bcast0.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
L.mpxb_barrier.argtypes = [C.c_void_p]
L.mpxb_allreduce_f64.argtypes = [C.c_void_p, C.c_double] + [C.POINTER(C.c_double)] * 3
L.mpxb_rank.argtypes = L.mpxb_size.argtypes = L.mpxb_finalize.argtypes = [C.c_void_p]
L.mpxb_error.restype = C.c_char_p

rank, size, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
timeout = float(sys.argv[4]) if len(sys.argv) > 4 else 30.0
b = C.c_void_p()
if L.mpxb_init(C.byref(b), rank, size, b"127.0.0.1", port, timeout) != 0:
    print(json.dumps({"rank": rank, "error": L.mpxb_error().decode()}), flush=True)
    sys.exit(3)
out = {"rank": L.mpxb_rank(b), "size": L.mpxb_size(b)}
mine = (C.c_uint64 * 3)(rank, rank * rank, 0xABCD0000 + rank)
allv = (C.c_uint64 * (3 * size))()
assert L.mpxb_allgather(b, mine, allv, 24) == 0
out["allgather"] = list(allv)
buf = C.create_string_buffer(b"rank0-says-hello" if rank == 0 else b"\0" * 16, 16)
assert L.mpxb_bcast0(b, buf, 16) == 0
out["bcast"] = buf.raw.decode()
for _ in range(200):
    assert L.mpxb_barrier(b) == 0
mn, mx, sm = C.c_double(), C.c_double(), C.c_double()
assert L.mpxb_allreduce_f64(b, 0.25 + rank, C.byref(mn), C.byref(mx), C.byref(sm)) == 0
out["reduce"] = [mn.value, mx.value, sm.value]
big = (C.c_ubyte * (1 << 20))()
C.memset(big, rank & 0xFF, 1 << 20)
bigall = (C.c_ubyte * (size << 20))()
assert L.mpxb_allgather(b, big, bigall, 1 << 20) == 0
out["big_ok"] = all(bigall[(r << 20) + 12345] == (r & 0xFF) for r in range(size))
L.mpxb_finalize(b)
print(json.dumps(out), flush=True)
