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
