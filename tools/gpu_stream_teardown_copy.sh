#!/bin/bash
# Round-2 follow-up of tools/gpu_stream_teardown.sh: does a device-to-device
# hipMemcpyAsync (a runtime blit kernel) on a CU-masked stream leave the
# process exit hanging even when every buffer is freed before the stream is
# destroyed (mpx's teardown order)?  Each scenario twice, 20 s limit each.
mkdir -p gpurun_out
out=gpurun_out/stream_teardown_copy.txt
: > $out
while IFS= read -r sc; do
    [ -z "$sc" ] && continue
    for rep in 1 2; do
        timeout -k 5 20 tools/stream_teardown "$sc" > gpurun_out/st_last.txt 2>&1
        rc=$?
        echo "[$sc] rep$rep rc=$rc: $(tr '\n' ' ' < gpurun_out/st_last.txt)" | tee -a $out
    done
done <<'LIST'
a0 a1 m0 k0.0 f0 f1 d0
a0 a1 m0 c0.0.1 f0 f1 d0
a0 a1 m0 c0.0.1 f0 f1
a0 a1 p0 c0.0.1 f0 f1 d0
a0 a1 m0 s0.0 f0 f1 d0
a0 a1 m0 m1 c0.0.1 c1.1.0 f0 f1 d0 d1
a0 a1 m0 m1 c0.0.1 c1.1.0 f0 f1
LIST
