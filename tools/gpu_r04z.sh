mkdir -p gpurun_out/r04z
MPX_BENCH_ONE_GPU=1 timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 > gpurun_out/r04z/bench_n2.json 2> gpurun_out/r04z/bench_n2.err
echo rc=$?
