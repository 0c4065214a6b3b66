"""Two PROCESSES on GPU 0 exchange payloads through libmpx's IPC path
(mpx_rank_export / mpx_rank_import), the path bench.py uses for one process
per GPU.  Every payload is checksummed; the final rx must equal the peer's tx.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("engine", ["kernel", "sdma", "kernel-pull", "sdma-pull"])
def test_two_process_ipc_pair(tmp_path, engine):
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "ipc_worker.py"), str(tmp_path), str(r), engine],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in (0, 1)]
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=100)[0])
        except subprocess.TimeoutExpired:
            p.kill()
            outs.append(p.communicate()[0])
    assert all(p.returncode == 0 for p in procs), outs
    for r in (0, 1):
        res = json.load(open(tmp_path / f"result_{r}.json"))
        assert len(res) == 3 * 8
        for x in res:
            assert x["final_rx_ok"], (r, x)
            # every payload checked, the non-blocking loop's 300 included
            # (receive slots in the peer's IPC-mapped ring)
            assert x["check_failures"] == 0 and x["check_iters"] == x["iters"], (r, x)
            assert x["recv_done"] == (x["iters"] - x["iters"] // 256 if x["mode"] == 1 else x["iters"]), (r, x)
            if engine == "kernel-pull":   # B-byte payloads pulled (protocol 7) above the 2 KiB LL threshold
                ll = x["mode"] != 1 and x["n"] <= 2048
                assert x["protocol"] == (0 if ll else 7), (r, x)
            if engine == "sdma-pull":     # every size pulled by the receiver's stream
                assert x["protocol"] == 8, (r, x)
