"""ctypes view of oracle/liboracle.so (the CPU restatement) for tests.

TEST INFRASTRUCTURE: the checker only.
"""
import ctypes as C
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "liboracle.so")
GOLDEN = os.path.join(ROOT, "tests", "golden", "ref_runs.json")
MAX_HOST = 128


class RankStats(C.Structure):
    _fields_ = [("recv_done", C.c_uint64), ("recv_bytes", C.c_uint64), ("recv_digest", C.c_uint64),
                ("sent_bytes", C.c_uint64), ("time_s", C.c_double)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            import subprocess
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "all"], check=True)
        L = C.CDLL(LIB)
        L.oracle_mix64.restype = C.c_uint64
        L.oracle_mix64.argtypes = [C.c_uint64]
        L.oracle_checksum.restype = C.c_uint64
        L.oracle_checksum.argtypes = [C.c_void_p, C.c_size_t]
        L.oracle_fill.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_uint64]
        L.oracle_strnicmp.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t]
        L.oracle_in_group1.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_int]
        L.oracle_pairing.argtypes = [C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.oracle_nb_waited.restype = C.c_longlong
        L.oracle_nb_waited.argtypes = [C.c_longlong]
        L.oracle_run_pairs.argtypes = [C.c_int, C.c_int, C.c_int, C.c_size_t, C.POINTER(RankStats),
                                       C.POINTER(C.c_double)]
        L.oracle_format_record.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int,
                                           C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_double, C.c_longlong]
        L.oracle_log_name.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_char_p, C.c_int, C.c_char_p]
        L.oracle_gbps.restype = C.c_double
        L.oracle_gbps.argtypes = [C.c_int, C.c_int, C.c_int, C.c_double]
        _lib = L
    return _lib


def checksum(data: bytes) -> int:
    return lib().oracle_checksum(data, len(data))


def fill(n: int, pattern: int, arg: int) -> bytes:
    buf = C.create_string_buffer(max(n, 1))
    lib().oracle_fill(buf, n, pattern, arg & 0xFFFFFFFFFFFFFFFF)
    return buf.raw[:n]


def pattern_checksum(n: int, pattern: int, arg: int) -> int:
    return checksum(fill(n, pattern, arg))


def in_group1(name: str, lines: list[str]) -> int:
    blob = b"".join((ln + "\n").encode().ljust(MAX_HOST, b"\0")[:MAX_HOST] for ln in lines)
    return lib().oracle_in_group1(name.encode(), len(name), blob, len(lines))


def pairing(groups: list[int]):
    n = len(groups)
    g = (C.c_int * n)(*groups)
    gr, pe = (C.c_int * n)(), (C.c_int * n)()
    lib().oracle_pairing(n, g, gr, pe)
    return list(gr), list(pe)


def run_pairs(npairs: int, mode: int, iters: int, nbytes: int):
    st = (RankStats * (2 * npairs))()
    mx = C.c_double()
    assert lib().oracle_run_pairs(npairs, mode, iters, nbytes, st, C.byref(mx)) == 0
    return [dict(recv_done=s.recv_done, recv_bytes=s.recv_bytes, recv_digest=s.recv_digest,
                 sent_bytes=s.sent_bytes, time_s=s.time_s) for s in st], mx.value


def format_record(ts, uuid, rank, world, ppn, lip, rip, blen, iters, t_s, run):
    out = C.create_string_buffer(1024)
    lib().oracle_format_record(out, 1024, ts.encode(), uuid.encode(), rank, world, ppn, lip.encode(), rip.encode(),
                               blen, iters, t_s, run)
    return out.value.decode()


def golden():
    with open(GOLDEN) as f:
        return json.load(f)
