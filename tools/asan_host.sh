#!/bin/bash
# Host C code under AddressSanitizer + UBSan (CPU only; GPU sanitizers are not
# available): the host library behind the CPU tests, and the mpx_perf CLI on
# its GPU-free paths.  The reference's two SIGFPE crashes are reproduced on
# purpose and are deselected here (the sanitizer intercepts the signal).
set -e -o pipefail
cd "$(dirname "$0")/.."
SAN="-O1 -g -std=c11 -D_GNU_SOURCE -fsanitize=address,undefined -fno-omit-frame-pointer"
cp mpi-perf_amd/lib/libmpx_host.so /tmp/libmpx_host.so.orig
trap 'cp /tmp/libmpx_host.so.orig mpi-perf_amd/lib/libmpx_host.so' EXIT
gcc $SAN -fPIC -shared -o mpi-perf_amd/lib/libmpx_host.so mpi-perf_amd/host/mpx_host.c mpi-perf_amd/host/mpx_boot.c
LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)" ASAN_OPTIONS=detect_leaks=0 \
    python -m pytest tests/test_host.py tests/test_procs.py tests/test_windows_variant.py -q -m "not gpu" \
    -p no:cacheprovider -k "not sigfpe and not crashes and not live_reference"
gcc $SAN -o /tmp/mpx_perf_asan mpi-perf_amd/host/mpx_perf.c mpi-perf_amd/host/mpx_host.c mpi-perf_amd/host/mpx_boot.c \
    -Lmpi-perf_amd/lib -lmpx -lpthread -Wl,-rpath,$PWD/mpi-perf_amd/lib
d=$(mktemp -d); echo vm > $d/g1
for args in "-h" "-f $d/g1 -n 1 -p 1 -d 1 -r 2 -l $d/logs" "-f $d/nosuch -n 1 -p 1" "-f $d/g1 -n 1 -p 1 -S 1:x" \
            "-f $d/g1 -n 1 -p 1 -i 0 -r 0 -l $d/logs -d 1"; do
    MPX_PROCESSOR_NAMES=vm,runsc /tmp/mpx_perf_asan -w 2 $args > $d/out 2>&1 || true
    ! grep -q -E "ERROR: AddressSanitizer|\.c:[0-9]+:[0-9]+: runtime error" $d/out || { cat $d/out; exit 1; }
done
# the Windows variant's front end (deliberate SIGSEGV paths excluded)
gcc $SAN -DMPX_WINDOWS_CLI -o /tmp/mpx_perf_win_asan mpi-perf_amd/host/mpx_perf.c mpi-perf_amd/host/mpx_host.c \
    mpi-perf_amd/host/mpx_boot.c -Lmpi-perf_amd/lib -lmpx -lpthread -Wl,-rpath,$PWD/mpi-perf_amd/lib
echo 10.0.0.2 > $d/w1
for args in "$d/w1 1 1 10 100 2 $d/logs" "$d/w1 0 1 10 100 2 $d/logs" "$d/nosuch 1 1 10 100 2 $d/logs" \
            "$d/w1 1 1 10 100 2 $d/logs -w 2 -e kernel -t 100" "$d/w1 1 1 10 100 2 $d/logs -u 1"; do
    MPX_PROCESSOR_NAMES=10.0.0.1,10.0.0.2 HIP_VISIBLE_DEVICES= /tmp/mpx_perf_win_asan $args > $d/out 2>&1 || true
    ! grep -q -E "ERROR: AddressSanitizer|\.c:[0-9]+:[0-9]+: runtime error" $d/out || { cat $d/out; exit 1; }
done
echo "asan_host: clean"
