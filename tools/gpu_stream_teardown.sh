#!/bin/bash
# Runs tools/stream_teardown scenarios, each in a process of its own with a
# 20 s limit (rc 124 after "exit" = a hang in the runtime's process teardown).
# After a failure the next scenario runs only if a plain control still passes.
mkdir -p gpurun_out
out=gpurun_out/stream_teardown.txt
: > $out
while IFS= read -r sc; do
    [ -z "$sc" ] && continue
    timeout -k 5 20 tools/stream_teardown "$sc" > gpurun_out/st_last.txt 2>&1
    rc=$?
    echo "[$sc] rc=$rc: $(tr '\n' ' ' < gpurun_out/st_last.txt)" | tee -a $out
    if [ $rc -ne 0 ]; then
        timeout -k 5 20 tools/stream_teardown "a0 p0 k0.0 d0 f0" > /dev/null 2>&1 || { echo "control failed: stop" | tee -a $out; exit 1; }
    fi
done <<'LIST'
a0 m0 k0.0 d0 f0
a0 a1 m0 k0.0 d0 f1
a0 m0 k0.0 d0
a0 m0 k0.0 f0 d0
m0 a0 k0.0 d0 f0
a0 m0 m1 k0.0 d0 f0 d1
a0 m0 m1 k0.0 d0 f0
a0 m0 m1 k0.0 k1.0 d0 f0 d1
a0 m0 k0.0 f0 d0 a1 m1 k1.1 f1 d1 a2 f2
a0 p0 k0.0 d0 f0
a0 m0 k0.0 d0 y f0
a0 m0 k0.0 d0 a1 f1
a0 m0 d0 f0
a0 m0 k0.0 d0 f0 m1
a0 m0 k0.0 d0 f0 m1 a1 k1.1
LIST
