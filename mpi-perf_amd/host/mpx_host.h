/*
 * mpx_host.h — host-side logic of mpx_perf (pure C, no HIP): command line,
 * group/peer rule, all-pairs round schedule, CSV records and log files.
 * Built into libmpx_host.so (tested on CPU against tests/golden) and linked
 * into the mpx_perf executable.
 *
 * Reference: /root/reference/mpi_perf.c — every function cites its lines.
 */
#ifndef MPX_HOST_H
#define MPX_HOST_H

#include <stddef.h>
#include <stdio.h>

#define MPXH_MAX_HOST 128          /* MAX_HOST_SZ            mpi_perf.c:13  */
#define MPXH_DEF_BUF_SZ 456131     /* DEF_BUF_SZ             mpi_perf.c:14  */
#define MPXH_DEF_ITERS 10          /* DEF_ITERS              mpi_perf.c:15  */
#define MPXH_LOG_REFRESH_SEC 900   /* LOG_REFRESH_TIME_SEC   mpi_perf.c:16  */
#define MPXH_MAX_RANKS 64

/* struct options, mpi_perf.c:257-268, plus the MI355X-only settings.  The
   first nine fields keep the reference's meaning and defaults. */
typedef struct mpxh_options {
    int use_dotnet;                 /* -d */
    int iters;                      /* -i */
    int buff_sz;                    /* -b */
    int uni_dir;                    /* -u */
    int num_runs;                   /* -r  (-1 = forever)   */
    int ppn;                        /* -p */
    int nonblocking;                /* -x */
    char uuid[64];
    char logfolder[MPXH_MAX_HOST];  /* -l */
    /* not in the reference */
    char group1_hostfile[MPXH_MAX_HOST]; /* -f (a global in mpi_perf.c:254) */
    int group_size;                 /* -n (a global in mpi_perf.c:255) */
    int world;                      /* -w  ranks (mpirun -np);  0 = 2*ppn   */
    int engine;                     /* -e  0 kernel, 1 sdma, 2 rccl          */
    int all_pairs;                  /* -a  1 = circle-method rounds           */
    int check;                      /* -c  1 = checksum every payload, 2 = and
                                           seeded-pattern payloads            */
    int sweep_min, sweep_max;       /* -S  min:max  power-of-two size sweep   */
    int timeout_ms;                 /* -t  per-wait device timeout            */
    char gpus[256];                 /* -g  rank->GPU list "0,1,..."          */
    int arm;                        /* -A  1 (default) = arm each run's kernel
                                           before the barrier (mpx_xfer_arm) */
} mpxh_options;

/* parse status */
enum {
    MPXH_PARSE_OK = 0,
    MPXH_PARSE_USAGE = 1,           /* unknown flag / -h: usage + abort      */
    MPXH_PARSE_BAD_VALUE = 2,       /* a value of a new flag is malformed    */
    MPXH_PARSE_CRASH = 3            /* the reference dereferences a missing
                                       argument (Windows variant)           */
};

/* defaults of main(), mpi_perf.c:388-392 (+ the new fields) */
void mpxh_defaults(mpxh_options *o);
/* parse_args, mpi_perf.c:273-339 (getopt ":f:n:d:p:i:b:u:h:r:l:x:" plus
   "w:e:a:c:S:t:g:A:"); fills o->uuid with a fresh v4 UUID.  Resets getopt. */
int mpxh_parse_args(mpxh_options *o, int argc, char **argv);
/* print_usage, mpi_perf.c:20-32 (the reference's text, then the new flags) */
void mpxh_print_usage(FILE *f);
/* engine name <-> id */
int mpxh_engine_from_name(const char *s);
const char *mpxh_engine_name(int e);

/* validate group_size, mpi_perf.c:399-403.  Returns:
   0 ok, 1 invalid (message printed, caller aborts), 2 the reference divides
   by zero here (ppn == 0 in bidirectional mode): the caller raises SIGFPE. */
int mpxh_validate(const mpxh_options *o, int world, FILE *err);
/* read the -f file with fgets into group_size lines of MAX_HOST bytes,
   mpi_perf.c:405-418.  Returns a calloc'd block or NULL (cannot open). */
char *mpxh_read_group1(const char *path, int group_size);

/* strnicmp, mpi_perf.c:34-53 */
int mpxh_strnicmp(const char *s1, const char *s2, size_t n);
/* membership, mpi_perf.c:437-444 */
int mpxh_in_group1(const char *name, const char *lines, int group_size);
/* Comm_split + peer, mpi_perf.c:447-450, :225-233 */
void mpxh_pairing(int world, const int *group, int *group_rank, int *group_size, int *peer);

/* Virtual processor name of rank r: "<node>-<r / ppn>" (ppn ranks per
   virtual host, as --map-by ppr:ppn:node places them); MPX_PROCESSOR_NAMES
   ("a,a,b,b") overrides.  Writes into out[MPXH_MAX_HOST]. */
void mpxh_processor_name(char *out, const char *node, int rank, int ppn, const char *override_list);

/* circle-method 1-factorisation: round r of n ranks (even
   n >= 2) -> pairs[k] = {g1, g0}, k < n/2.  Returns n/2 or -1. */
int mpxh_round_pairs(int n, int r, int (*pairs)[2]);
/* role of `rank` in round r: *group (1/0) and *peer.  Returns 0 or -1. */
int mpxh_round_role(int n, int r, int rank, int *group, int *peer);

/* parse "0,1,2" into devs[] (max n); returns count or -1 */
int mpxh_parse_gpu_list(const char *s, int *devs, int n);

/* time strings, getformatted_time mpi_perf.c:341-353 */
void mpxh_format_time(char *buf, size_t cap, int for_kusto);
/* record line, mpi_perf.c:550-554 */
int mpxh_format_record(char *out, size_t cap, const char *timestamp, const char *uuid, int world_rank,
                       int world_size, int ppn, const char *local_ip, const char *remote_ip, int buff_len,
                       int iters, double my_time_s, long long run_idx);
/* log file name, mpi_perf.c:494 */
int mpxh_log_name(char *out, size_t cap, const char *logfolder, const char *uuid, int world_rank,
                  const char *file_time);
/* REPORT_BANDWIDTH line, mpi_perf.c:535-541 */
int mpxh_format_bandwidth(char *out, size_t cap, int world_rank, long long run_idx, int buff_len, int iters,
                          int uni_dir, double my_time_s);
/* rank-0 summary, mpi_perf.c:564-568 */
int mpxh_format_summary(char *out, size_t cap, long long run_idx, double total_s, double min_s, double max_s,
                        double sum_s, int world);
/* INFO line, mpi_perf.c:460-461 */
int mpxh_format_info(char *out, size_t cap, const char *name, int rank, int world, int group, int group_size,
                     int group_rank, int peer, const char *my_ip, const char *peer_name, const char *peer_ip);
/* .NET launcher lines, mpi_perf.c:147-168 (printed, never executed) */
int mpxh_format_dotnet(char *out, size_t cap, int my_group, int my_rank, int peer_rank, const char *peer_ip,
                       const char *my_ip, int buff_len, int iters, int ppn);
/* v4 UUID (libuuid's uuid_generate + uuid_unparse, mpi_perf.c:335-337) */
void mpxh_uuid(char out[37]);
/* IPv4 of a host name: last AF_INET result like get_ipaddress,
   mpi_perf.c:171-198.  Returns 0 ok, -1 lookup failed. */
int mpxh_ipv4(const char *host, char *out, size_t cap);

/* ---- the Windows / MS-MPI variant, windows/mpi-perf.cpp ----------------- */
/* 7-character job id (generate_uuid's sizeof(char *) truncation, :175-184) */
void mpxh_uuid_windows(char out[64]);
/* positional parse_args, :187-197, over main's defaults :226-230 */
int mpxh_parse_args_windows(mpxh_options *o, int argc, char **argv);
/* group-1 address lines with the newline cut off, :249-261 */
char *mpxh_read_group1_windows(const char *path, int group_size);
/* whole-address case-insensitive membership, :283-289 */
int mpxh_in_group1_windows(const char *addr, const char *lines, int group_size);
/* Comm_split + last-match peer, :114-133, :292-295 */
void mpxh_pairing_windows(int world, const int *group, int *group_rank, int *group_size, int *peer);

#endif
