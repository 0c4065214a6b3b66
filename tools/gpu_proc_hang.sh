#!/bin/bash
# Diagnoses a stall of mpx_perf in processes mode (one process per rank, IPC;
# tests/test_gpu_host.py::test_processes_mode_*): N attempts of the 2-rank
# ping-pong case on GPU 0; a process still alive 40 s after the start is
# asked for every thread's stack (SIGUSR1 under MPX_DEBUG), then killed, and
# the script stops.  Output: gpurun_out/proc_hang/.
OUT=gpurun_out/proc_hang${TAG:+_$TAG}
mkdir -p $OUT
cd $OUT || exit 1
echo "vm" > group1
N=${N:-3}
ENGINE=${ENGINE:-kernel}
for a in $(seq 1 $N); do
    rm -rf logs
    port=$((29700 + a))
    pids=()
    for r in 0 1; do
        MPX_POOL_EXIT=$MPX_POOL_EXIT MPX_DEBUG=1 MPX_RANK=$r MPX_SIZE=2 MPX_LOCAL_RANK=$r MPX_PROCESSOR_NAMES=vm,runsc \
        MPX_BOOTSTRAP=127.0.0.1:$port MPX_BOOTSTRAP_TIMEOUT=60 MPX_HOSTNAME=localhost \
            ../../mpi-perf_amd/bin/mpx_perf -g 0,0 -t 5000 -f group1 -n 1 -p 1 -r 3 -i 3 -b 456131 -l logs \
            -e $ENGINE -c 1 > out_${a}_$r.txt 2> err_${a}_$r.txt &
        pids+=($!)
    done
    t=0
    while [ $t -lt ${WAIT_TICKS:-400} ]; do
        alive=0
        for p in "${pids[@]}"; do kill -0 $p 2>/dev/null && alive=1; done
        [ $alive -eq 0 ] && break
        sleep 0.1; t=$((t + 1))
    done
    stuck=0
    for i in 0 1; do
        p=${pids[$i]}
        if kill -0 $p 2>/dev/null; then
            stuck=1
            echo "attempt $a rank $i: still running after $((${WAIT_TICKS:-400} / 10)) s" | tee -a summary.txt
            for tk in /proc/$p/task/*; do echo "$(basename $tk) $(cat $tk/comm) wchan=$(cat $tk/wchan)"; done >> summary.txt
            kill -USR1 $p; sleep 2
        fi
    done
    for p in "${pids[@]}"; do kill -9 $p 2>/dev/null; wait $p 2>/dev/null; done
    [ $stuck -eq 1 ] && [ -z "$KEEP_GOING" ] && exit 3
    [ $stuck -eq 0 ] && echo "attempt $a: clean" | tee -a summary.txt
done
exit 0
