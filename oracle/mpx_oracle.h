/*
 * mpx_oracle.h — CPU restatement of mpi_perf's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this code, and only as the checker /
 * the timed CPU baseline — never as the product path (libmpx has no CPU
 * fallback).  Every function cites the /root/reference/mpi_perf.c lines it
 * restates.  Parity of this restatement is pinned against the compiled
 * reference (oracle/Makefile `ref` target, tests/golden/gen_golden.py).
 */
#ifndef MPX_ORACLE_H
#define MPX_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#define ORACLE_MAX_HOST 128   /* MAX_HOST_SZ, mpi_perf.c:13 */

/* --- payload arithmetic (shared definition with libmpx) ------ */
uint64_t oracle_mix64(uint64_t z);
/* order-independent checksum: sum_k mix64(w_k + (k+1)*G) ^ mix64(n) */
uint64_t oracle_checksum(const void *buf, size_t n);
/* MPX_FILL_BYTE (0): memset; MPX_FILL_SPLITMIX (1): word k = mix64((arg^k)+G) */
void oracle_fill(void *buf, size_t n, int pattern, uint64_t arg);

/* --- group / peer rule (mpi_perf.c:34-53, :437-450, :200-238) ---------- */
/* strnicmp exactly as mpi_perf.c:34-53 */
int oracle_strnicmp(const char *s1, const char *s2, size_t n);
/* 1 if `name` (length name_len) prefix-matches any of the `group_size`
   MAX_HOST-strided lines in `lines` (mpi_perf.c:438-444) */
int oracle_in_group1(const char *name, int name_len, const char *lines, int group_size);
/* Given each world rank's group (0/1), compute group_rank (MPI_Comm_split
   keyed by world rank, :447-450) and peer (first rank of the other group with
   the same group_rank, :225-233; -1 if none). */
void oracle_pairing(int world, const int *group, int *group_rank, int *peer);

/* --- the Windows / MS-MPI variant's group rule (windows/mpi-perf.cpp) ---
   Restated from the source: that file needs MS-MPI and Winsock, so it cannot
   be compiled here and this part of the oracle is parity-unpinned. */
/* 1 if `addr` equals (case-insensitively, whole string) any of the
   `group_size` MAX_HOST-strided lines after each line's newline is cut off
   (:256-260, :283-289) */
int oracle_win_in_group1(const char *addr, const char *lines, int group_size);
/* Comm_split keyed by world rank (:292-295) and get_peer_info's loop without
   a break: the LAST other-group rank with the same group rank (:114-133) */
void oracle_win_pairing(int world, const int *group, int *group_rank, int *peer);

/* --- transfer loops (mpi_perf.c:66-145), CPU engine -------------------- */
enum { ORACLE_PINGPONG = 0, ORACLE_NONBLOCKING = 1, ORACLE_UNIDIR = 2 };
typedef struct oracle_rank_stats {
    uint64_t recv_done;      /* receives completed inside the loop           */
    uint64_t recv_bytes;     /* bytes of those receives                      */
    uint64_t recv_digest;    /* sum of oracle_checksum of each completed recv */
    uint64_t sent_bytes;
    double time_s;           /* my_time (mpi_perf.c:501,532-533)             */
} oracle_rank_stats;

/* Number of receives the reference's nonblocking loop waits on for `iters`
   iterations (mpi_perf.c:95-124: slot 255 of each full window is never
   waited on). */
long long oracle_nb_waited(long long iters);

/* Run one pair (G1 thread and G0 thread) for `iters` iterations of `mode`
   with B-byte messages; tx of group g is filled with 'a'+g... as the
   reference (mpi_perf.c:244-251).  stats[1] = group-1 rank, stats[0] = G0.
   Returns 0 on success. */
int oracle_run_pair(int mode, int iters, size_t B, oracle_rank_stats stats[2]);

/* Run `npairs` concurrent pairs (the -p ppn layout) once; fills per-rank
   stats (2*npairs entries: ranks [0,npairs) are G1, the rest G0) and returns
   the max time over ranks in *max_time (the reference's MAX allreduce). */
int oracle_run_pairs(int npairs, int mode, int iters, size_t B, oracle_rank_stats *stats, double *max_time);

/* --- records (mpi_perf.c:341-353, :494, :550-554, :538-539) ------------- */
/* CSV record, mpi_perf.c:551-554 */
int oracle_format_record(char *out, size_t cap, const char *timestamp, const char *uuid, int world_rank,
                         int world_size, int ppn, const char *local_ip, const char *remote_ip, int buff_len,
                         int iters, double my_time_s, long long run_idx);
/* log file name, mpi_perf.c:494 */
int oracle_log_name(char *out, size_t cap, const char *logfolder, const char *uuid, int world_rank,
                    const char *file_time);
/* REPORT_BANDWIDTH formula, mpi_perf.c:538-539: Gbit/s */
double oracle_gbps(int buff_len, int iters, int uni_dir, double my_time_s);

#endif
