set -x
mkdir -p gpurun_out
{ rocminfo | grep -E 'Marketing|gfx|Compute Unit' | head -20; rocm-smi --showtopo 2>&1 | head -40; nproc; free -g; ls /opt/conda/bin/mpicc; python -c 'import torch;print(torch.cuda.device_count(), torch.cuda.get_device_name(0))'; } > gpurun_out/probe.txt 2>&1
timeout -k 10 120 rocprofv3 -L > gpurun_out/rocprof_L.txt 2>&1 || true
grep -i -E 'xgmi|TCC_EA0_RDREQ|FETCH_SIZE|WRITE_SIZE' gpurun_out/rocprof_L.txt | head -60 > gpurun_out/counters_grep.txt || true
echo done
