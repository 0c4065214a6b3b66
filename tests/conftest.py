"""pytest configuration: the `gpu` marker, paths, and shared helpers.

`-m "not gpu"` runs here (no GPU): oracle vs golden fixtures, host logic, and
the C-ABI symbol check.  `-m gpu` runs on an MI355X box and calls libmpx
through its C-ABI, checking every result against the oracle.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mpi-perf_amd")
for p in (PKG, os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)

# libmpx's fault-injection knobs (MPX_TEST="skip_push=k,lag_wg=r:w:us,
# no_posted,no_pull_wait") are looked at only in a process that starts with
# MPX_TEST set — this one, and the workers it spawns, which inherit it.  The
# tests change its value between calls.
os.environ.setdefault("MPX_TEST", "")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
