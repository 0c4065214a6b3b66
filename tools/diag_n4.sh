#!/bin/bash
# N=4 rehearsal on one GPU (every rank on GPU 0): kernel engine headline,
# then the SDMA / RCCL comparison contexts, with libmpx debug output.
set -o pipefail
mkdir -p gpurun_out
MPX_DEBUG=1 MPX_BENCH_ONE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 4 --steps 6 --warmup 2 > gpurun_out/n4_kernel.json 2> gpurun_out/n4_kernel.err
echo "rc=$?"
