#!/bin/bash
# Diagnoses the intermittent exit stall of `mpx_perf -e sdma -x 1 -c 1` with
# two ranks on GPU 0 (tests/test_scripts.py::test_pair_script_on_gpu[sdma]).
# Up to N attempts; an attempt still alive 30 s after start is asked for
# every thread's stack (SIGUSR1, MPX_DEBUG), killed, and the script stops.
mkdir -p gpurun_out/exit_hang
cd gpurun_out/exit_hang || exit 1
echo "node-0" > group1
N=${N:-6}
for a in $(seq 1 $N); do
    rm -rf logs
    MPX_DEBUG=1 MPX_POOL_EXIT=${MPX_POOL_EXIT:-} MPX_PROCESSOR_NAMES= MPX_HOSTNAME=node ../../mpi-perf_amd/bin/mpx_perf -w 2 -g 0,0 -e ${ENGINE:-sdma} \
        -f group1 -n 1 -p 1 -r 3 -i 300 -b 65536 -l logs -x 1 -c 1 -t 5000 > out_$a.txt 2> err_$a.txt &
    pid=$!
    t=0
    while kill -0 $pid 2>/dev/null && [ $t -lt 300 ]; do sleep 0.1; t=$((t + 1)); done
    if kill -0 $pid 2>/dev/null; then
        echo "attempt $a: still running after 30 s; stacks:" | tee -a summary.txt
        for tk in /proc/$pid/task/*; do echo "$(basename $tk) $(cat $tk/comm) wchan=$(cat $tk/wchan)"; done >> summary.txt
        kill -USR1 $pid; sleep 3
        kill -9 $pid; wait $pid 2>/dev/null
        tail -5 err_$a.txt | tee -a summary.txt
        exit 3
    fi
    wait $pid; rc=$?
    echo "attempt $a: rc=$rc $(grep -c . err_$a.txt) stderr lines" | tee -a summary.txt
    [ $rc -ne 0 ] && exit $rc
done
exit 0
