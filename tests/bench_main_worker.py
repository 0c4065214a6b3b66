"""One rank of tests/test_bench_main.py: bench.py's main() end to end at
N > 1 on CPU (gloo), with the TEST-ONLY stand-in for the mpx binding from
bench_dist_worker.py and torch.cuda's device calls stubbed out.  Checks the
JSON line contract and the comparison-engine watchdog without a GPU.

    RANK=r WORLD_SIZE=n LOCAL_RANK=r MASTER_ADDR=127.0.0.1 MASTER_PORT=p \\
        python bench_main_worker.py <scenario> --gpus n --steps K --warmup W
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402

import bench  # noqa: E402
import bench_dist_worker as W  # noqa: E402

W.rank = int(os.environ["RANK"])
W.scenario = sys.argv[1]
from mpx import spin as _spin  # noqa: E402  (the real node-local spin barrier: host code, no GPU)

W.FakeMpx.spin = _spin
sys.modules["mpx"] = W.FakeMpx          # bench.main's `import mpx` gets the stand-in
torch.cuda.set_device = lambda d: None
torch.cuda.synchronize = lambda *a: None
# one GPU per rank (bench.main then describes every pair's link: link_table)
torch.cuda.device_count = lambda: int(os.environ["WORLD_SIZE"])
bench.EXTRAS_DEADLINE_S = 5
sys.argv = ["bench.py"] + sys.argv[2:]
bench.main()
# main() returns through the normal exit after destroying the rank streams
# (mpx_shutdown), profiled or not (round 5: no os._exit after the line)
print(f"MAIN_RETURNED shutdown={any(x[0] == 'shutdown' for x in W.FakeMpx.log)}", file=sys.stderr, flush=True)
