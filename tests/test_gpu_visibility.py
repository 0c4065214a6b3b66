"""Mid-kernel visibility of bytes written by another memory client — the
cross-GPU check-mode case on one GPU ("Cross-GPU visibility").

tools/stale_l2_probe: one workgroup per CU reads its chunk of a buffer, then
spins; a copy engine (hipMemcpyDeviceToDeviceNoCU) or a kernel on another
stream replaces the buffer; the workgroups read again after an acquire of
each kind.  k_xfer's check reads (system acquire, sc0|sc1 loads, sum_chunk in
csrc/mpx_kernels.hip) must see none of the old words, and the positive
control (plain loads, no acquire: the CU's L1) must see some, or the probe
would prove nothing.
"""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "tools", "stale_l2_probe")

pytestmark = pytest.mark.gpu


@pytest.mark.skipif(not os.path.exists(PROBE), reason="tools/stale_l2_probe not built (make -C tools)")
def test_check_reads_never_see_bytes_replaced_mid_kernel():
    p = subprocess.run([PROBE, str(4 << 20), "1"], capture_output=True, text=True, timeout=90)
    assert p.returncode == 0, (p.stdout[-800:], p.stderr[-800:])
    rows = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(rows) == 36, p.stdout[-800:]
    for r in rows:
        assert r["lost_flag"] == 0 and r["load1_bad"] == 0 and r["other_words"] == 0, r
        control = r["load1"] == "plain" and r["acquire"] == "none" and r["load2"] == "plain"
        if not control:
            assert r["stale_words"] == 0, r
    # the check form itself, for every writer
    check = [r for r in rows if r["acquire"] == "system" and r["load2"] == "sys"]
    assert {r["writer"] for r in check} == {"sdma", "ksc1", "kplain"}
    assert sum(r["stale_words"] for r in rows if r["load1"] == "plain" and r["acquire"] == "none"
               and r["load2"] == "plain") > 0, "the L1 control saw nothing: the probe cannot detect staleness"
