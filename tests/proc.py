"""Bounded subprocess runs for the GPU tests.

A child that outlives its limit is killed and the test fails with the tail
of what it printed, instead of pytest-timeout (120 s per test) ending the
whole session with only the parent's stack.  Limits stay below 120 s."""
import subprocess


def run_bounded(cmd, timeout=90, **kw):
    try:
        return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, **kw)
    except subprocess.TimeoutExpired as e:
        def tail(b):
            if b is None:
                return ""
            s = b.decode(errors="replace") if isinstance(b, bytes) else b
            return s[-3000:]
        raise AssertionError(f"{cmd[:3]}... still running after {timeout} s; stderr tail:\n{tail(e.stderr)}\n"
                             f"stdout tail:\n{tail(e.stdout)}") from None
