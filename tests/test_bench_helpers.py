"""bench.py's transfer helpers on CPU, with stand-in objects (no GPU, no
libmpx calls): the failure paths the advisor flagged in round 4."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import bench  # noqa: E402


class Ctx:
    """records the calls bench.safe_wall makes on an mpx context"""

    def __init__(self, fail_xfer=None):
        self.log, self.fail_xfer = [], fail_xfer

    def xfer(self, mode, group, me, peer, iters, tx, rx, n, **kw):
        self.log.append(("xfer", me))
        if self.fail_xfer:
            raise self.fail_xfer

        class T:
            wall_s = 0.5
        return T()

    def disarm(self, r):
        self.log.append(("disarm", r))


class Dist:
    def __init__(self, fail=None):
        self.fail = fail

    def barrier(self):
        if self.fail:
            raise self.fail


def test_safe_wall_disarms_when_the_start_never_came():
    """The barrier in front of an armed transfer fails (a spin-barrier
    TimeoutError): the call is cancelled, so the rank is not left armed."""
    c, errs = Ctx(), []
    w = bench.safe_wall(c, errs, 2, 1, 3, 4, 10, None, None, 4096, barrier=Dist(TimeoutError("spin barrier")))
    assert w == float("inf") and ("disarm", 3) in c.log and ("xfer", 3) not in c.log
    assert errs and "TimeoutError" in errs[0]


def test_safe_wall_disarm_after_a_failed_transfer_is_harmless():
    """The transfer itself fails (the call was started: libmpx already
    dropped it): disarm is still issued and is a no-op there."""
    c, errs = Ctx(fail_xfer=RuntimeError("device wait timed out")), []
    assert bench.safe_wall(c, errs, 2, 1, 0, 1, 10, None, None, 8) == float("inf")
    assert c.log == [("xfer", 0), ("disarm", 0)]


def test_safe_wall_success_does_not_disarm():
    c, errs = Ctx(), []
    assert bench.safe_wall(c, errs, 2, 1, 0, 1, 10, None, None, 8, barrier=Dist()) == 0.5
    assert c.log == [("xfer", 0)] and not errs


def test_config1_pingpong_baseline_shape():
    """The compiled reference's 2-rank ping-pong (BASELINE config 1) that
    bench.py puts beside its N = 1 and N >= 2 lines: 8 B half round trip and
    4 MiB rate, two cores, median of runs 1..5."""
    pp = bench.cpu_baseline_pingpong()
    assert pp is not None, "oracle/_ref not built (python -c 'import __graft_entry__ as g; g.build()')"
    assert pp["cores"] == 2 and pp["kind"] == "reference" and pp["loop"].startswith("ping-pong")
    assert 0 < pp["half_rtt_us_8B"] < 100 and 0 < pp["GBps_4MiB"] < 1000, pp
