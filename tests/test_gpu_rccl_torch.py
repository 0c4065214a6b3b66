"""The RCCL engine in bench.py's process layout (round 5).

libmpx opens the image's /opt/rocm/lib/librccl.so.1 itself (RTLD_LOCAL |
RTLD_DEEPBIND).  bench.py imports torch before libmpx, so in its processes
the HIP runtime is torch's bundled one (soname libamdhip64.so.7, already
loaded), and that RCCL runs on it.  The -m gpu suite never imports torch,
so this runs the RCCL self pair in a child that does, with torch's CUDA
context live first, and checks the transfers as test_gpu_engine does
(oracle-derived checksums and receive counts)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))

CHILD = """
import sys, json
sys.path.insert(0, {pkg!r}); sys.path.insert(0, {here!r})
import torch
torch.zeros(1, device="cuda:0").add_(1)        # torch's HIP runtime is live first
torch.cuda.synchronize()
import mpx
import oracle_py as O
v = mpx.rccl_version()
cap = 65541
c = mpx.Context(1, "rccl")
try:
    key = mpx.pattern_key(mpx.PATTERN_SEED, 0, 0, 7)
    tx, rx = c.alloc(0, cap), c.alloc(0, cap)
    c.fill(tx, cap, mpx.FILL_SPLITMIX, key)
    c.fill(rx, cap, mpx.FILL_BYTE, 0)
    c.attach(0, 0, tx, rx, cap)
    c.rccl_init_all()
    c.prepare(mpx.MODE_NONBLOCKING, 0, 0, 0, 300, cap)
    res = []
    for n, iters in ((1, 3), (4097, 257), (cap, 300)):
        want = O.pattern_checksum(n, mpx.FILL_SPLITMIX, key)
        t = c.xfer(mpx.MODE_NONBLOCKING, 0, 0, 0, iters, tx, rx, n, check_payload=True, expect=want, timeout_ms=20000)
        k = O.lib().oracle_nb_waited(iters)
        res.append(dict(n=n, iters=iters, ok=t.check_iters == iters and t.check_failures == 0 and t.recv_done == k
                        and t.recv_digest == (k * want) & 0xFFFFFFFFFFFFFFFF and c.checksum(rx, n) == want,
                        protocol=t.protocol))
finally:
    c.close()
mpx.shutdown()
print(json.dumps(dict(rccl=v, hip=torch.version.hip, cases=res)))
"""


# the first `import torch` on a fresh box pages the image in (1-2 minutes)
@pytest.mark.timeout(330)
def test_rccl_self_pair_in_a_torch_first_process():
    code = CHILD.format(pkg=os.path.join(os.path.dirname(HERE), "mpi-perf_amd"), here=HERE)
    r = subprocess.run([sys.executable, "-u", "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-400:], r.stderr[-1200:])
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["rccl"]["library"] == "/opt/rocm/lib/librccl.so.1", d
    assert all(x["ok"] and x["protocol"] == 3 for x in d["cases"]), d
