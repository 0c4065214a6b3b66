"""CPU checks of the diagnostic tools the round-5 root cause rests on
(profiles/r05_exit_stall_symbolized.txt): tools/symbolize_frames.py names the
stripped ROCm frames of profiles/r04_procs_exit_stall.txt by the strings and
calls of their enclosing functions.  Tied to the image's ROCm 7.2 build (the
offsets are that build's): skipped on another build."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIP = "/opt/rocm/lib/libamdhip64.so.7"
HSA = "/opt/rocm/lib/libhsa-runtime64.so.1"
HIP_BUILD_ID = "c7eeb80a2701f2525f81fea6b13c88cc5df7013c"


def build_id(path):
    r = subprocess.run(["readelf", "-n", path], capture_output=True, text=True)
    return next((ln.split()[-1] for ln in r.stdout.splitlines() if "Build ID" in ln), None)


def symbolize(lib, *offsets):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "symbolize_frames.py"), lib, *offsets],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-400:]
    return r.stdout


@pytest.mark.skipif(not os.path.exists(HIP) or build_id(HIP) != HIP_BUILD_ID, reason="not the image's HIP build")
def test_stall_frames_are_named():
    out = symbolize(HIP, "0x3ea90f", "0x3fff31", "0x3fd4f9", "0x4b499")
    assert "Deleting CG enabled hardware queue" in out            # roc::Device::releaseQueue
    assert "There was a timestamp that was not used; deleting." in out   # ~VirtualGPU
    assert "Handler: value(%d), timestamp(%p), handle(0x%lx)" in out      # the completion handler
    assert "removeFatBinary" in out                                # the exit-time unregistration
    assert "hsa_queue_destroy@plt" in out


@pytest.mark.skipif(not os.path.exists(HSA), reason="no HSA runtime")
def test_kfd_wait_ioctl_request():
    """the event thread's ioctl request is AMDKFD_IOC_WAIT_EVENTS:
    _IOWR('K', 0x0c, 24-byte struct)"""
    req = 0xc0184b0c
    assert (req >> 30) == 3 and ((req >> 16) & 0x3fff) == 24 and ((req >> 8) & 0xff) == ord("K") and (req & 0xff) == 0x0c
    r = subprocess.run(["objdump", "-d", "--no-show-raw-insn", "--start-address=0x135700", "--stop-address=0x1357f0",
                        HSA], capture_output=True, text=True)
    if "$0xc0184b0c" not in r.stdout:
        pytest.skip("not the image's HSA build")
    assert "call" in r.stdout


# ---- tools/link_counter_control.py's peer-HBM cases, with stand-ins ---------
class _Buf:
    def __init__(self, dev, n, ptr):
        self.dev, self.n, self.ptr = dev, n, ptr


class _Ctx:
    def __init__(self, *a):
        self.k = 0

    def alloc(self, dev, n):
        self.k += 1
        return _Buf(dev, n, 0x1000 * self.k)

    def fill(self, *a):
        pass

    def attach(self, *a):
        pass

    def copy(self, *a):
        pass

    def xfer(self, *a, **k):
        pass

    def checksum(self, b, n):
        return 7      # every copy "checks"

    def free(self, b):
        pass

    def close(self):
        pass


class _Mpx:
    MODE_UNIDIR, FILL_BYTE, FILL_SPLITMIX = 2, 0, 1
    Context = _Ctx


def _counters(per_byte):
    """a stand-in counter module whose passes read `per_byte` x the control's
    known bytes for each counter (in that counter's unit)"""
    import bench
    nbytes = bench.PEER_CONTROL_BYTES * bench.PEER_CONTROL_ITERS
    unit = {"TCC_EA0_WRREQ_sum": 64, "TCC_EA0_WRREQ_64B_sum": 64, "TCC_EA0_WRREQ_DRAM_sum": 64,
            "TCC_EA0_WRREQ_WRITE_GMI_32B_sum": 32, "TCC_EA0_WRREQ_WRITE_IO_32B_sum": 32,
            "TCC_EA0_WRREQ_WRITE_DRAM_32B_sum": 32}

    class Pass:
        def __init__(self, bus, names):
            self.names = names

        def __enter__(self):
            return self

        def __exit__(self, *e):
            self.values = [per_byte.get(n, 0.0) * nbytes / unit[n] for n in self.names]
            return False

    class Counters:
        pass
    Counters.Pass = Pass
    return Counters, nbytes, unit


class _Hip:
    @staticmethod
    def hipIpcGetMemHandle(h, p):
        return 0


def _tool():
    sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    sys.path.insert(0, ROOT)
    import link_counter_control as T
    return T


@pytest.mark.parametrize("peer,per_byte,want", [
    # a store into peer HBM classified as DRAM at the sender: the subtraction
    # reads 0, the GMI 32-B counter the bytes -> 'gmi'
    (1, {"TCC_EA0_WRREQ_sum": 1.0, "TCC_EA0_WRREQ_DRAM_sum": 1.0, "TCC_EA0_WRREQ_WRITE_GMI_32B_sum": 1.0}, "gmi"),
    # peer writes not DRAM-classified: the subtraction reads them (first choice)
    (1, {"TCC_EA0_WRREQ_sum": 1.0, "TCC_EA0_WRREQ_WRITE_GMI_32B_sum": 1.0}, "subtraction"),
    # nothing reads the bytes: no formula, with the reason
    (1, {"TCC_EA0_WRREQ_sum": 0.5, "TCC_EA0_WRREQ_DRAM_sum": 0.5}, None),
    # one GPU: the code path only
    (0, {"TCC_EA0_WRREQ_sum": 1.0, "TCC_EA0_WRREQ_WRITE_GMI_32B_sum": 1.0}, None),
])
def test_link_counter_control_peer_cases_pick_the_formula(peer, per_byte, want):
    """the tool's peer-HBM cases — GPU 0 writing known
    bytes into an IPC-imported buffer of GPU 1 (a child process) and
    bench.peer_link_control's identical in-process case — report every EA
    write counter as a multiple of the bytes, and the formula is picked from
    that table."""
    T = _tool()
    counters, nbytes, unit = _counters(per_byte)
    seen = []

    def run_child(handle_hex):
        seen.append(handle_hex)
        vals = {n: per_byte.get(n, 0.0) * nbytes / u for n, u in unit.items()}
        return dict(T.summarise(dict(vals, TCC_EA0_WRREQ_64B_sum=0.0), nbytes), copy_checked=True, src_checksum=7)

    c = _Ctx()
    r = T.peer_cases(_Mpx, counters, _Hip, c, c.alloc(0, 16), "bus0", peer, run_child)
    assert len(seen) == 1 and set(r["peer_table"]) == {"peer_hbm_ipc", "peer_hbm"}
    for row in r["peer_table"].values():
        for k in ("TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_DRAM_sum", "TCC_EA0_WRREQ_WRITE_GMI_32B_sum",
                  "TCC_EA0_WRREQ_WRITE_IO_32B_sum"):
            assert row[k] == pytest.approx(per_byte.get(k, 0.0), abs=1e-4), (k, row)
        assert row["checked"] is True and set(row["formulas"]) == {"subtraction", "gmi", "io"}
    f = r["peer_formula"]
    assert f["formula"] == want, f
    if want is None:
        assert f["reason"].startswith("one GPU" if peer == 0 else "no formula")
    assert r["cases"]["copy->peer_hbm_ipc"]["copy_checked_by_owner"] is True
