/*
 * mpxprof.h — hardware counters of a process's own GPU work, sampled from
 * inside the process (libmpxprof.so, mpi-perf_amd/csrc/mpx_counters.cpp).
 *
 * north_star asks for "rocprof counters (achieved xGMI and HBM GB/s)" beside
 * the reference's bandwidth number (mpi_perf.c:535-542).  The reference has no
 * counterpart; this is measurement infrastructure of the benchmark host
 * (bench.py), not part of the drop-in seam (include/mpx.h).
 *
 * It is a rocprofiler-sdk tool that uses the DEVICE counting service: agent-
 * wide counters read between two samples, with no per-dispatch serialisation
 * (rocprofv3 --pmc is the dispatch counting service, which serialises kernels
 * and so cannot run the two co-dependent halves of a pair).
 *
 * Use: mpxprof_register() before the process's first HIP call (the tool must
 * be configured before the HSA runtime initialises), then around any stretch
 * of GPU work, outside timed regions:
 *     mpxprof_begin(bus_id, "FETCH_SIZE");  ... work ...  mpxprof_end(v, 1, &mode);
 * One pass holds what one hardware pass can (MI355X_MICROARCH.md "PMC slots":
 * TCC 4 slots; FETCH_SIZE uses 3 and WRITE_SIZE 2, so they go in separate
 * passes).  Counters are summed over all their instances (XCC, TCC channel).
 */
#ifndef MPXPROF_H
#define MPXPROF_H

#ifdef __cplusplus
extern "C" {
#endif

/* Registers the tool with rocprofiler-sdk (rocprofiler_force_configure).
   0 = ok; -1 = rocprofiler is already configured (too late: HIP started, or
   another tool such as rocprofv3 owns the process) — mpxprof_error() says. */
int mpxprof_register(void);
/* 1 once the tool initialised and holds a device-counting context for at
   least one GPU agent (that happens when the HSA runtime starts) */
int mpxprof_ready(void);
/* text of the last failure on any call ("" if none) */
const char *mpxprof_error(void);
/* Start sampling `counters` (comma-separated rocprofiler counter names,
   derived ones included) on the GPU with PCI bus id `bus_id`
   ("DDDD:BB:DD.F", as hipDeviceGetPCIBusId writes it).  0 = ok. */
int mpxprof_begin(const char *bus_id, const char *counters);
/* Sample again and stop.  values[i] = counter i of the begin call, summed
   over its instances, accumulated between begin and end.  *reads_reset
   (may be NULL) = 1 if this SDK's samples restart from zero at every read
   (then values are the end sample), 0 if they accumulate from the context
   start (then values are end - begin).  0 = ok. */
int mpxprof_end(double *values, int n, int *reads_reset);

#ifdef __cplusplus
}
#endif
#endif /* MPXPROF_H */
