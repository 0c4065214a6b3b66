"""A short randomised soak of the pair protocol on every run of the GPU suite
(tools/soak.py: push and pull calls in every loop, 0 B - 8 MiB around the LL
and unit edges, check on and off, push widths, the streaming hint, tx
rewritten between calls).  After every call each rank's rx must equal the
peer's tx, and every checked payload must pass.  profiles/r03_soak.jsonl
holds the long runs (39 600 calls) and the negative controls that show the
soak sees the cross-call races it is there for."""
import importlib.util
import os

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _soak():
    spec = importlib.util.spec_from_file_location("soak", os.path.join(ROOT, "tools", "soak.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("form,engine,calls,seed", [("threads", "kernel", 400, 101), ("procs", "kernel", 200, 102),
                                                    ("threads", "sdma", 200, 103)])
def test_randomised_calls_keep_every_payload(form, engine, calls, seed):
    S = _soak()
    res = (S.threads if form == "threads" else S.procs)(calls, seed, engine)
    assert res["failures"] == 0, res
