/*
 * mpx_boot.h — the out-of-band job communicator of mpx_perf's multi-process
 * mode (one process per rank, started by any launcher: mpiexec, torchrun,
 * srun).  Pure C over TCP sockets, star topology around rank 0.
 *
 * It replaces the MPI collectives the reference calls OUTSIDE its transfer
 * loops (SURVEY.md §2 call-site table); the loops themselves never touch it:
 *   mpxb_bcast0         MPI_Bcast of options / group-1 hosts   mpi_perf.c:422-431
 *   mpxb_allgather      MPI_Allgather of node_info             mpi_perf.c:223-224
 *   mpxb_barrier        MPI_Barrier                            mpi_perf.c:499,557,579
 *   mpxb_allreduce_f64  MPI_Allreduce MIN / MAX / SUM          mpi_perf.c:560-562
 * Every call is collective: all ranks make the same calls in the same order.
 * Errors return -1 with a message in mpxb_error(); callers abort the job.
 */
#ifndef MPX_BOOT_H
#define MPX_BOOT_H

#include <stddef.h>

typedef struct mpxb mpxb;

/* The launcher's view of this process (first variable set wins):
 *   rank : MPX_RANK, RANK, PMI_RANK, OMPI_COMM_WORLD_RANK, SLURM_PROCID
 *   size : MPX_SIZE, WORLD_SIZE, PMI_SIZE, OMPI_COMM_WORLD_SIZE, SLURM_NTASKS
 *   local: MPX_LOCAL_RANK, LOCAL_RANK, MPI_LOCALRANKID, OMPI_COMM_WORLD_LOCAL_RANK, SLURM_LOCALID
 * Returns 1 if a launcher was found (rank and size set), else 0 with
 * *rank = 0, *size = 1, *local = 0. */
int mpxb_launcher(int *rank, int *size, int *local);

/* Rendezvous address: MPX_BOOTSTRAP="host:port", else MASTER_ADDR and
 * MASTER_PORT + 1 (torchrun's own store owns MASTER_PORT), else
 * 127.0.0.1:29571.  Writes host into host[cap]; returns the port. */
int mpxb_address(char *host, size_t cap);

/* Connect the job: rank 0 listens on host:port, every other rank connects
 * (retrying until timeout_s).  Returns 0 or -1. */
int mpxb_init(mpxb **out, int rank, int size, const char *host, int port, double timeout_s);
void mpxb_finalize(mpxb *b);

int mpxb_rank(const mpxb *b);
int mpxb_size(const mpxb *b);

/* all[r*bytes .. (r+1)*bytes) = rank r's `mine`, on every rank */
int mpxb_allgather(mpxb *b, const void *mine, void *all, size_t bytes);
/* rank 0's buf[0:bytes) to every rank */
int mpxb_bcast0(mpxb *b, void *buf, size_t bytes);
int mpxb_barrier(mpxb *b);
/* min / max / sum of one double per rank (any output may be NULL); every
 * rank gets bit-identical results (reduced in rank order) */
int mpxb_allreduce_f64(mpxb *b, double v, double *mn, double *mx, double *sum);

/* Spin barrier for the barrier in front of every timed loop (MPI_Barrier,
 * mpi_perf.c:499): a TCP star round trip or a futex wake-up lets ranks leave
 * tens of microseconds apart, and a rank's timer starts at its own exit, so
 * that skew lands in short loops' records; MPI's intra-node barrier spins on
 * shared memory.  name = NULL: in this process (threads); else a POSIX shm
 * object (e.g. "/mpxbar-<job>") the ranks of one node share, created by one
 * of them (create = 1) before the others open it.  Every wait is bounded by
 * timeout_s.  Returns 0 or -1 (mpxb_error). */
typedef struct mpxb_spin mpxb_spin;
int mpxb_spin_open(mpxb_spin **out, const char *name, int nranks, int create);
int mpxb_spin_wait(mpxb_spin *s, double timeout_s);
/* Wait on the barrier, then call fn(ctx, mode, ..., timing) — libmpx's
   mpx_xfer_ex, passed by pointer (this library does not link libmpx) — on
   this thread with nothing in between, and store its return in *xfer_rc.
   For a host whose barrier and timed call live in an interpreted layer
   (bench.py): between leaving the barrier and an armed call's start it adds
   no interpreter round trip (several microseconds, different on every rank),
   as mpx_perf, all C, adds none.  Returns the barrier's status; fn is not
   called when the barrier fails. */
typedef int (*mpxb_xfer_fn)(void *ctx, int mode, int group, int rank, int peer, int iters, void *tx, void *rx,
                            int len, const void *opts, void *timing);
int mpxb_spin_wait_xfer(mpxb_spin *s, double timeout_s, mpxb_xfer_fn fn, void *ctx, int mode, int group, int rank,
                        int peer, int iters, void *tx, void *rx, int len, const void *opts, void *timing,
                        int *xfer_rc);
void mpxb_spin_close(mpxb_spin *s, int unlink_it);

const char *mpxb_error(void);

#endif
