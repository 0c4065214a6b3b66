/*
 * mpx_perf.c — mpi_perf for MI355X GPUs.
 *
 * Same command line, group/peer rule, run loop, timing, CSV records and log
 * rotation as /root/reference/mpi_perf.c:367-582; the transfer loop is
 * libmpx's mpx_xfer_ex (kernel / SDMA / RCCL engines over xGMI) instead of
 * MPI point-to-point.  Two ways to start the ranks, same flags:
 *
 *   threads   mpx_perf -w N -f g1 -n 1 -p P ...
 *             one process, one host thread per rank (and GPU).
 *   processes mpiexec -n N mpx_perf -f g1 -n 1 -p P ...      (or torchrun, srun)
 *             one process per rank, exactly the reference's process model
 *             (mpirun -np N --map-by ppr:P:node mpi_perf ...).  The launcher's
 *             rank variables are read by mpx_boot_launcher(); the collectives
 *             the reference makes outside its loops (Bcast, Allgather,
 *             Barrier, Allreduce) run over mpx_boot's TCP star.  Ranks of one
 *             node map each other's rx and mailbox through IPC (kernel and
 *             SDMA engines); the RCCL engine also spans nodes.
 *             MPX_LAUNCH=threads forces the threads mode under a launcher.
 *
 * Processor names (the string matched against the -f file, mpi_perf.c:433-444):
 * MPX_PROCESSOR_NAMES="a,a,b,b" (indexed by world rank) if set; else, when the
 * ranks span several hosts, the host name, like MPI_Get_processor_name; else
 * (one host) virtual host k = "<host>-<k>" for ranks [k*P, (k+1)*P).  With
 * -a 1 every run is one round of the circle-method all-pairs schedule.
 *
 * Built with -DMPX_WINDOWS_CLI (bin/mpx_perf_win), the front end is the
 * Windows / MS-MPI variant's (/root/reference/windows/mpi-perf.cpp):
 *
 *   mpx_perf_win <group1-addresses> <group-size> <ppn> <iters> <buffer-size>
 *                <runs> <logfolder> [-w N -g ... -e ... -a ... -c ... -t ...]
 *
 * unidirectional only, ranks grouped by IPv4 address (whole-string match),
 * 7-character job id, INFO lines on stdout, no ingest hook and no
 * REPORT_BANDWIDTH.  A rank's address is its processor name when that is a
 * numeric IPv4 address, the host's address when the name is the host's own,
 * and otherwise (a virtual host of one node) the name itself.
 */
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include <dirent.h>
#include <errno.h>
#include <execinfo.h>
#include <pthread.h>
#include <sys/mman.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <arpa/inet.h>

#include "../../include/mpx.h"
#include "mpx_boot.h"
#include "mpx_host.h"

/* MPI_CHECK analogue, mpi_perf.c:55-64: print and exit(EXIT_FAILURE) */
/* A failed call ends the process at once, after flushing stdio (records and
   messages written so far reach their files, as exit() would flush them):
   _exit skips the atexit handlers and HIP's static destructors.  Other rank
   threads may still be inside libmpx calls on the same context, so neither
   finalizing the context here nor libmpx's exit handler can tear the rank
   streams down safely; the kernel driver releases the GPU state of the
   exiting process.  mpi_perf.c:55-64's MPI_CHECK exits EXIT_FAILURE too. */
#define MPX_CHECK(stmt)                                                                                  \
    do {                                                                                                 \
        int mpx_errno = (stmt);                                                                          \
        if (MPX_OK != mpx_errno) {                                                                       \
            fprintf(stderr, "[%s:%d] mpx call failed with %d (%s: %s) \n", __FILE__, __LINE__, mpx_errno, \
                    mpx_strerror(mpx_errno), mpx_last_error());                                          \
            fflush(NULL);                                                                                \
            _exit(EXIT_FAILURE);                                                                         \
        }                                                                                                \
    } while (0)

/* MPI_Abort(MPI_COMM_WORLD, -1) analogue: the launcher reported 255 */
static void mpx_abort(void)
{
    fflush(stdout);
    fflush(stderr);
    _exit(255);
}

static mpxh_options opt;
static int world;
static mpx_ctx *ctx;
static int dev_of[MPXH_MAX_RANKS];
static char name_of[MPXH_MAX_RANKS][MPXH_MAX_HOST];
static char host_of[MPXH_MAX_RANKS][MPXH_MAX_HOST]; /* real host names */
static char ip_of[MPXH_MAX_RANKS][MPXH_MAX_HOST];
static int group_of[MPXH_MAX_RANKS], grank_of[MPXH_MAX_RANKS], gsize_of[MPXH_MAX_RANKS], peer_of[MPXH_MAX_RANKS];
static void *tx_of[MPXH_MAX_RANKS], *rx_of[MPXH_MAX_RANKS];
static double time_of[MPXH_MAX_RANKS];
static uint64_t txsum_of[MPXH_MAX_RANKS], txsum1_of[MPXH_MAX_RANKS];
static pthread_barrier_t bar;
static int report_bandwidth;
static int sizes[40], nsizes;
/* LOG_REFRESH_TIME_SEC (mpi_perf.c:16); MPX_LOG_REFRESH_SEC overrides it for tests */
static double log_refresh_sec = MPXH_LOG_REFRESH_SEC;

/* processes mode */
static int procs;            /* 1: one process per rank under a launcher */
static int me;               /* this process's world rank (processes mode) */
static int local_rank;       /* its node-local rank */
static int multi_host;       /* the ranks span more than one host */
static mpxb *boot;

#ifdef MPX_WINDOWS_CLI
static const int win_cli = 1; /* windows/mpi-perf.cpp front end */
#else
static const int win_cli = 0;
#endif
static char addr_of[MPXH_MAX_RANKS][MPXH_MAX_HOST]; /* Windows variant's group key */

static double wtime(void) /* MPI_Wtime */
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int is_root(void) { return !procs || me == 0; }

static void boot_failed(void)
{
    fprintf(stderr, "mpx_perf: job communicator failed: %s\n", mpxb_error());
    mpx_abort();
}

/* MPI_Barrier, mpi_perf.c:499,557,579 */
static void barrier(void)
{
    if (procs) {
        if (mpxb_barrier(boot) != 0) boot_failed();
    } else {
        pthread_barrier_wait(&bar);
    }
}

/* The barrier right in front of every timed loop (mpi_perf.c:499): a spin
   barrier (threads: in this process; processes on one node: POSIX shared
   memory named after the job id), so the ranks leave it within about a
   microsecond as MPI's intra-node barrier lets them — a TCP round trip or a
   futex wake-up let them leave tens of microseconds apart, and each rank's
   timer starts at its own exit.  Ranks on several hosts use barrier(). */
static mpxb_spin *start_bar;

static void open_start_barrier(void)
{
    if (!procs) {
        if (mpxb_spin_open(&start_bar, NULL, world, 1) != 0) boot_failed();
        return;
    }
    if (multi_host) return;
    char name[128];
    snprintf(name, sizeof name, "/mpxbar-%s", opt.uuid);
    if (me == 0 && mpxb_spin_open(&start_bar, name, world, 1) != 0) boot_failed();
    barrier();
    if (me != 0 && mpxb_spin_open(&start_bar, name, world, 0) != 0) boot_failed();
    barrier();
    if (me == 0) shm_unlink(name);   /* every rank has it mapped: the name can go now */
}

static void start_barrier(void)
{
    if (!start_bar) {
        barrier();
        return;
    }
    if (mpxb_spin_wait(start_bar, 600.0) != 0) boot_failed();
}

/* every rank learns every rank's tx checksums (check mode's expected values) */
static void share_tx_checksums(int r, uint64_t s, uint64_t s1)
{
    if (procs) {
        uint64_t mine[2] = {s, s1}, all[MPXH_MAX_RANKS][2];
        if (mpxb_allgather(boot, mine, all, sizeof mine) != 0) boot_failed();
        for (int q = 0; q < world; ++q) {
            txsum_of[q] = all[q][0];
            txsum1_of[q] = all[q][1];
        }
        return;
    }
    barrier(); /* nobody still reads last run's values */
    txsum_of[r] = s;
    txsum1_of[r] = s1;
    barrier();
}

/* node-local rank of rank r: the ingest hook runs on node-local rank 0 only
   (OMPI_COMM_WORLD_LOCAL_RANK, mpi_perf.c:355-365, :378-384) */
static int node_local(int r)
{
    if (procs && multi_host) return local_rank;
    return r % (opt.ppn > 0 ? opt.ppn : 1);
}

/* kusto_injest, mpi_perf.c:355-365: the command is site configuration here
   (MPX_INGEST_CMD) instead of a hard-coded path */
static void ingest_hook(int rank)
{
    const char *cmd = getenv("MPX_INGEST_CMD");
    if (win_cli) return; /* the Windows variant has no ingest hook */
    if (node_local(rank) != 0 || !cmd || !*cmd) return;
    if (system(cmd) == -1) fprintf(stderr, "ingest hook failed: %s\n", strerror(errno));
}

typedef struct {
    FILE *log_fp, *gpu_fp;
    double t_last_logtime;
} rank_files;

static void open_logs(int rank, rank_files *f)
{
    if (f->log_fp) {
        fflush(f->log_fp);
        fclose(f->log_fp);
    }
    if (f->gpu_fp) fclose(f->gpu_fp);
    ingest_hook(rank);
    char ft[26] = {0};
    char name[2 * MPXH_MAX_HOST + 64];
    mpxh_format_time(ft, sizeof ft, 0);
    mpxh_log_name(name, sizeof name, opt.logfolder, opt.uuid, rank, ft);
    f->log_fp = fopen(name, "w");
    /* GPU side file: never starts with "tcp", so kusto_ingest.py (which
       picks files starting with "tcp", kusto_ingest.py:32) ignores it */
    snprintf(name, sizeof name, "%s/gpu-%s-%d-%s.csv", opt.logfolder, opt.uuid, rank, ft);
    f->gpu_fp = fopen(name, "w");
    if (f->gpu_fp)
        fprintf(f->gpu_fp, "Timestamp,JobId,Rank,Engine,Mode,Device,PeerRank,PeerDevice,BufferSize,NumOfBuffers,"
                           "WallTimems,DeviceTimems,GBps,Protocol,Workgroups,CheckedPayloads,CheckFailures,RunId,RecvDone,"
                           "RecvDigest,Launch,Rccl\n");
    f->t_last_logtime = wtime();
}

/* the RCCL this process runs, "<release>:<library path>" (engine rccl), for
   the gpu-*.csv side file: bench.py, which loads torch first, runs torch's
   bundled RCCL; mpx_perf the image's */
static char rccl_build[600];

static void note_rccl_build(void)
{
    int v = 0;
    char path[512] = {0};
    if (opt.engine != MPX_ENGINE_RCCL || mpx_rccl_version(&v, path, sizeof path) != MPX_OK) return;
    snprintf(rccl_build, sizeof rccl_build, "%d.%d.%d:%s", v / 10000, v / 100 % 100, v % 100, path);
    fprintf(stderr, "[mpx_perf] RCCL %s\n", rccl_build);
}

static int xfer_mode(void)
{
    if (opt.uni_dir) return MPX_MODE_UNIDIR;
    return opt.nonblocking ? MPX_MODE_NONBLOCKING : MPX_MODE_PINGPONG;
}

/* the run loop of one rank, mpi_perf.c:470-569 */
static void *rank_main(void *arg)
{
    const int r = (int)(intptr_t)arg;
    rank_files files = {NULL, NULL, wtime()};
    int prev_group = -1;
    for (int si = 0; si < nsizes; ++si) {
        const int B = sizes[si];
        for (long long run_idx = 0; opt.num_runs == -1 || run_idx < opt.num_runs; run_idx++) {
            int group = group_of[r], peer = peer_of[r];
            if (opt.all_pairs) {
                const int round = (int)(run_idx % (world - 1));
                if (mpxh_round_role(world, round, r, &group, &peer)) peer = -1;
            }
            if (!opt.use_dotnet) {
                /* tx content per group (mpi_perf.c:244-251) or a seeded pattern */
                if (opt.check == 2) {
                    MPX_CHECK(mpx_fill(ctx, dev_of[r], tx_of[r], (size_t)B, MPX_FILL_SPLITMIX,
                                       mpx_pattern_key(MPX_PATTERN_SEED, (unsigned)r, (unsigned)peer,
                                                       (unsigned)run_idx)));
                    prev_group = -1;
                } else if (group != prev_group) {
                    MPX_CHECK(mpx_fill(ctx, dev_of[r], tx_of[r], (size_t)B, MPX_FILL_BYTE, group ? 'b' : 'a'));
                    prev_group = group;
                }
            }
            if (group == 1 && (files.log_fp == NULL || (wtime() - files.t_last_logtime) > log_refresh_sec))
                open_logs(r, &files);

            mpx_xfer_opts xo;
            memset(&xo, 0, sizeof xo);
            xo.timeout_ms = (uint32_t)opt.timeout_ms;
            if (opt.check && !opt.use_dotnet) {
                /* expected payloads: the peer's tx, read after every fill */
                uint64_t s, s1;
                MPX_CHECK(mpx_checksum(ctx, dev_of[r], tx_of[r], (size_t)B, &s));
                MPX_CHECK(mpx_checksum(ctx, dev_of[r], tx_of[r], 1, &s1));
                share_tx_checksums(r, s, s1);
                xo.check = 1;
                xo.expect_checksum = txsum_of[peer];
                xo.expect_ack = txsum1_of[peer];
            }

            /* SDMA engine: capture this (mode, peer, B)'s graph chunks now, not
               inside the timed call (the reference's timer brackets only the
               loop, mpi_perf.c:501-533) */
            if (!opt.use_dotnet) MPX_CHECK(mpx_xfer_prepare(ctx, xfer_mode(), group, r, peer, opt.iters, B, &xo));
            /* -A 1: the run's kernel is launched now and started by the
               mpx_xfer_ex after the barrier (MPI_Start of a persistent
               request), so the launch is not inside the timed loop */
            if (!opt.use_dotnet && opt.arm)
                MPX_CHECK(mpx_xfer_arm(ctx, xfer_mode(), group, r, peer, opt.iters, tx_of[r], rx_of[r], B, &xo));
            start_barrier(); /* MPI_Barrier, mpi_perf.c:499 */
            const double t_start = wtime();
            mpx_timing tm;
            memset(&tm, 0, sizeof tm);
            if (opt.use_dotnet) {
                char line[512];
                mpxh_format_dotnet(line, sizeof line, group, r, peer, ip_of[peer], ip_of[r], B, opt.iters, opt.ppn);
                fputs(line, stderr);
            } else {
                MPX_CHECK(mpx_xfer_ex(ctx, xfer_mode(), group, r, peer, opt.iters, tx_of[r], rx_of[r], B, &xo, &tm));
            }
            const double my_time = wtime() - t_start; /* mpi_perf.c:532-533 */

            if (report_bandwidth && group == 0) {
                char line[256];
                mpxh_format_bandwidth(line, sizeof line, r, run_idx, B, opt.iters, opt.uni_dir, my_time);
                fputs(line, stderr);
            }
            if (!opt.use_dotnet && run_idx > 0 && group == 1) { /* mpi_perf.c:545-555 */
                if (opt.ppn == 0) raise(SIGFPE); /* world_size / ppn in the reference's record */
                char ts[MPXH_MAX_HOST] = {0}, line[1024];
                mpxh_format_time(ts, sizeof ts, 1);
                mpxh_format_record(line, sizeof line, ts, opt.uuid, r, world, opt.ppn, ip_of[r], ip_of[peer], B,
                                   opt.iters, my_time, run_idx);
                if (files.log_fp) fputs(line, files.log_fp);
                if (files.gpu_fp) {
                    const double gbps = my_time > 0 ? (double)tm.bytes / my_time / 1e9 : 0.0;
                    static const char *proto[] = {"ll", "bulk", "sdma", "rccl", "copy", "copy_steps", "copy_pipe", "pull",
                                                 "sdma_pull"};
                    fprintf(files.gpu_fp, "%s,%s,%d,%s,%d,%d,%d,%d,%d,%d,%.4f,%.4f,%.3f,%s,%d,%llu,%d,%lld,%llu,%llu,%s,%s\n", ts,
                            opt.uuid, r, mpxh_engine_name(opt.engine), xfer_mode(), dev_of[r], peer, dev_of[peer], B,
                            opt.iters, my_time * 1e3, tm.device_s * 1e3, gbps,
                            (tm.protocol >= 0 && tm.protocol <= 8) ? proto[tm.protocol] : "?", tm.nwg,
                            (unsigned long long)tm.check_iters, tm.check_failures, run_idx,
                            (unsigned long long)tm.recv_done, (unsigned long long)tm.recv_digest,
                            (opt.arm && opt.engine == MPX_ENGINE_KERNEL) ? "armed" : "inline", rccl_build);
                }
            }

            time_of[r] = my_time;
            barrier(); /* MPI_Barrier, mpi_perf.c:557 */
            const double t_end = wtime();
            /* Allreduce MIN/MAX/SUM, mpi_perf.c:560-562 (every run, every rank) */
            double mn = my_time, mx = my_time, sum = my_time;
            if (procs) {
                if (mpxb_allreduce_f64(boot, my_time, &mn, &mx, &sum) != 0) boot_failed();
            } else if (r == 0) {
                /* the other threads cannot overwrite time_of before rank 0
                   reaches the next run's barrier */
                sum = 0;
                for (int q = 0; q < world; ++q) {
                    if (time_of[q] < mn) mn = time_of[q];
                    if (time_of[q] > mx) mx = time_of[q];
                    sum += time_of[q];
                }
            }
            if (r == 0 && (run_idx % 1000 == 0)) { /* mpi_perf.c:564-568 */
                char line[256];
                mpxh_format_summary(line, sizeof line, run_idx, t_end - t_start, mn, mx, sum, world);
                fputs(line, stderr);
            }
        }
    }
    if (files.log_fp) fclose(files.log_fp);
    if (files.gpu_fp) fclose(files.gpu_fp);
    return NULL;
}

/* ---- processes mode: the reference's once-per-job collectives ------------ */

/* MPI_Bcast of the options (with rank 0's UUID) and of the group-1 host
   lines, mpi_perf.c:422-431.  Rank 0 has read the -f file. */
static char *share_options_and_group1(char *group1)
{
    if (mpxb_bcast0(boot, &opt, sizeof opt) != 0) boot_failed();
    int ok = group1 != NULL;
    if (mpxb_bcast0(boot, &ok, sizeof ok) != 0) boot_failed();
    if (!ok) mpx_abort(); /* rank 0 printed "cannot open group1 file" */
    if (me != 0) group1 = (char *)calloc((size_t)(opt.group_size > 0 ? opt.group_size : 1), MPXH_MAX_HOST);
    if (mpxb_bcast0(boot, group1, (size_t)opt.group_size * MPXH_MAX_HOST) != 0) boot_failed();
    return group1;
}

/* node_info Allgather (mpi_perf.c:215-224): host name, GPU, IP of every rank */
typedef struct {
    char host[MPXH_MAX_HOST];
    char ip[MPXH_MAX_HOST];
    int32_t dev;
} node_info;

static void share_node_info(const char *node, const char *ip, int dev)
{
    node_info mine, all[MPXH_MAX_RANKS];
    memset(&mine, 0, sizeof mine);
    snprintf(mine.host, sizeof mine.host, "%s", node);
    snprintf(mine.ip, sizeof mine.ip, "%s", ip);
    mine.dev = dev;
    if (mpxb_allgather(boot, &mine, all, sizeof mine) != 0) boot_failed();
    for (int q = 0; q < world; ++q) {
        memcpy(host_of[q], all[q].host, MPXH_MAX_HOST);
        memcpy(ip_of[q], all[q].ip, MPXH_MAX_HOST);
        dev_of[q] = all[q].dev;
        if (strcmp(host_of[q], host_of[0]) != 0) multi_host = 1;
    }
}

/* Peers this rank transfers with: its fixed peer, or everyone (-a 1). */
static int needs_peer(int q)
{
    if (q == me) return 0;
    return opt.all_pairs || peer_of[me] == q;
}

/* The kernel and SDMA engines write into a peer's HBM: both ranks of every
   pair this rank transfers with must be on its node.  Checked right after
   the pairing, before any GPU call, like the reference's configuration
   errors. */
static void check_pairs_share_a_node(void)
{
    if (opt.engine == MPX_ENGINE_RCCL || opt.use_dotnet) return;
    for (int q = 0; q < world; ++q) {
        if (needs_peer(q) && strcmp(host_of[q], host_of[me]) != 0) {
            fprintf(stderr,
                    "rank %d (%s) and rank %d (%s) are on different hosts: the %s engine needs both on one node "
                    "(use -e rccl)\n",
                    me, host_of[me], q, host_of[q], mpxh_engine_name(opt.engine));
            mpx_abort();
        }
    }
}

/* Map the peers' buffers (kernel / SDMA engines: IPC within one node) or
   join the RCCL communicator (rank 0's unique id, any number of nodes). */
static void connect_ranks(void)
{
    if (opt.engine == MPX_ENGINE_RCCL) {
        unsigned char id[MPX_RCCL_ID_BYTES] = {0};
        if (me == 0) MPX_CHECK(mpx_rccl_get_unique_id(id));
        if (mpxb_bcast0(boot, id, sizeof id) != 0) boot_failed();
        MPX_CHECK(mpx_rccl_init_rank(ctx, me, world, id));
        note_rccl_build();
        return;
    }
    static unsigned char all[MPXH_MAX_RANKS][MPX_RANK_DESC_BYTES];
    unsigned char mine[MPX_RANK_DESC_BYTES];
    MPX_CHECK(mpx_rank_export(ctx, me, mine));
    if (mpxb_allgather(boot, mine, all, sizeof mine) != 0) boot_failed();
    for (int q = 0; q < world; ++q)
        if (q != me && strcmp(host_of[q], host_of[me]) == 0) MPX_CHECK(mpx_rank_import(ctx, q, all[q]));
}

/* Diagnostics (MPX_DEBUG set): `kill -USR1 <pid>` prints the stack of every
   thread of the process to stderr, so a run that stalls — inside a loop, a
   teardown or the runtime's exit — says where. */
static void dump_this_thread(int sig)
{
    (void)sig;
    void *pc[48];
    char hdr[64];
    const int n = snprintf(hdr, sizeof hdr, "[mpx] thread %ld:\n", (long)syscall(SYS_gettid));
    if (write(2, hdr, (size_t)n) < 0) return;
    backtrace_symbols_fd(pc, backtrace(pc, 48), 2);
}

static void dump_all_threads(int sig)
{
    const long self = (long)syscall(SYS_gettid);
    DIR *d = opendir("/proc/self/task");
    if (d) {
        struct dirent *e;
        while ((e = readdir(d)) != NULL) {
            const long tid = atol(e->d_name);
            if (tid <= 0 || tid == self) continue;
            syscall(SYS_tgkill, (long)getpid(), tid, SIGUSR2);
            usleep(20000);   /* one stack at a time */
        }
        closedir(d);
    }
    dump_this_thread(sig);
}

static void install_stack_dump(void)
{
    void *warm[2];
    (void)backtrace(warm, 2);   /* loads the unwinder now, not inside a handler */
    signal(SIGUSR2, dump_this_thread);
    signal(SIGUSR1, dump_all_threads);
}

int main(int argc, char **argv)
{
    int lrank = 0, lsize = 1;
    if (getenv("MPX_DEBUG")) install_stack_dump();
    const char *launch = getenv("MPX_LAUNCH");
    const int found = mpxb_launcher(&lrank, &lsize, &local_rank);
    procs = found && lsize > 1 && !(launch && !strcmp(launch, "threads"));
    me = procs ? lrank : 0;

    mpxh_defaults(&opt);
    const int pst = win_cli ? mpxh_parse_args_windows(&opt, argc, argv) : mpxh_parse_args(&opt, argc, argv);
    if (pst == MPXH_PARSE_CRASH) raise(SIGSEGV); /* strncpy(..., argv[argc] == NULL), windows/mpi-perf.cpp:189 */
    if (pst == MPXH_PARSE_USAGE) {
        if (is_root()) mpxh_print_usage(stderr);
        mpx_abort();
    }
    if (pst == MPXH_PARSE_BAD_VALUE) {
        if (is_root()) {
            fprintf(stderr, "bad value for -e / -S\n");
            mpxh_print_usage(stderr);
        }
        mpx_abort();
    }
    if (is_root() && !win_cli) fprintf(stderr, "UUID: %s\n", opt.uuid); /* mpi_perf.c:338 */
#ifdef REPORT_BANDWIDTH
    report_bandwidth = 1;
#else
    report_bandwidth = getenv("MPX_REPORT_BANDWIDTH") != NULL;
#endif
    if (win_cli) report_bandwidth = 0;
    if (getenv("MPX_LOG_REFRESH_SEC")) log_refresh_sec = atof(getenv("MPX_LOG_REFRESH_SEC"));

    if (procs) {
        world = lsize;
        if (world > MPXH_MAX_RANKS || world > MPX_MAX_RANKS || lrank < 0 || lrank >= world) {
            if (is_root()) fprintf(stderr, "at most %d ranks\n", MPXH_MAX_RANKS);
            mpx_abort();
        }
        if (opt.world > 0 && opt.world != world) {
            if (is_root()) fprintf(stderr, "-w %d but the launcher started %d ranks\n", opt.world, world);
            mpx_abort();
        }
    } else {
        world = opt.world > 0 ? opt.world : (opt.ppn > 0 ? 2 * opt.ppn : 2);
        if (world > MPXH_MAX_RANKS || world > MPX_MAX_RANKS) {
            fprintf(stderr, "at most %d ranks\n", MPXH_MAX_RANKS);
            mpx_abort();
        }
    }
    /* rank 0 validates (mpi_perf.c:399-403); the others see the same values */
    FILE *quiet = is_root() ? stderr : fopen("/dev/null", "w");
    const int v = mpxh_validate(&opt, world, quiet ? quiet : stderr);
    if (v == 2) raise(SIGFPE);
    if (v) mpx_abort();
    char *group1 = NULL;
    if (is_root()) {
        group1 = win_cli ? mpxh_read_group1_windows(opt.group1_hostfile, opt.group_size)
                         : mpxh_read_group1(opt.group1_hostfile, opt.group_size);
        if (!group1) {
            fprintf(stderr, "cannot open group1 file: %s\n", opt.group1_hostfile);
            if (!procs) mpx_abort();
        }
    }
    if (opt.all_pairs && (world < 2 || (world & 1))) {
        if (is_root()) fprintf(stderr, "-a 1 needs an even number of ranks\n");
        mpx_abort();
    }

    /* this process's host, IP and (processes mode) GPU */
    char node[MPXH_MAX_HOST] = {0};
    gethostname(node, sizeof node - 1);
    /* MPX_HOSTNAME: the host name this process reports (multi-node rehearsal
       on one machine: each process names a different "node") */
    if (getenv("MPX_HOSTNAME") && *getenv("MPX_HOSTNAME")) snprintf(node, sizeof node, "%s", getenv("MPX_HOSTNAME"));
    char node_ip[MPXH_MAX_HOST] = "127.0.0.1";
    if (mpxh_ipv4(node, node_ip, sizeof node_ip) != 0) snprintf(node_ip, sizeof node_ip, "127.0.0.1");
    int ndev = world;
    int gl[MPXH_MAX_RANKS];
    const int ngl = opt.gpus[0] ? mpxh_parse_gpu_list(opt.gpus, gl, MPXH_MAX_RANKS) : 0;

    if (procs) {
        char bhost[MPXH_MAX_HOST];
        const int port = mpxb_address(bhost, sizeof bhost);
        const char *tmo = getenv("MPX_BOOTSTRAP_TIMEOUT");
        if (mpxb_init(&boot, me, world, bhost, port, tmo ? atof(tmo) : 120.0) != 0) boot_failed();
        group1 = share_options_and_group1(group1);
        /* GPU of this rank: -g indexed by node-local rank, else the node-local
           rank itself (checked against the visible GPUs after the pairing, so
           the configuration errors come first, as in the reference) */
        int dev = local_rank;
        if (opt.gpus[0]) {
            if (ngl <= local_rank) {
                fprintf(stderr, "-g lists no GPU for node-local rank %d\n", local_rank);
                mpx_abort();
            }
            dev = gl[local_rank];
        }
        /* LocalIP / RemoteIP of the records and INFO lines: the IPv4 of the
           rank's host, as get_ipaddress(processor name) gives it in the
           reference (mpi_perf.c:236-237,553); the GPU ids go to gpu-*.csv */
        share_node_info(node, node_ip, dev);
    } else {
        for (int r = 0; r < world; ++r) snprintf(host_of[r], MPXH_MAX_HOST, "%s", node);
    }

    /* processor names and the group/peer rule, mpi_perf.c:433-458 */
    const char *names_env = getenv("MPX_PROCESSOR_NAMES");
    for (int r = 0; r < world; ++r) {
        if (names_env && *names_env)
            mpxh_processor_name(name_of[r], host_of[r], r, opt.ppn, names_env);
        else if (multi_host)
            snprintf(name_of[r], MPXH_MAX_HOST, "%s", host_of[r]); /* MPI_Get_processor_name */
        else
            mpxh_processor_name(name_of[r], host_of[r], r, opt.ppn, NULL);
        if (win_cli) { /* get_ipaddress(myhostname), windows/mpi-perf.cpp:278-289 */
            unsigned char a4[4];
            if (inet_pton(AF_INET, name_of[r], a4) == 1)
                snprintf(addr_of[r], MPXH_MAX_HOST, "%s", name_of[r]);
            else if (!strcmp(name_of[r], host_of[r]))
                snprintf(addr_of[r], MPXH_MAX_HOST, "%.*s", (int)strcspn(procs ? ip_of[r] : node_ip, ":"),
                         procs ? ip_of[r] : node_ip);
            else
                snprintf(addr_of[r], MPXH_MAX_HOST, "%s", name_of[r]);
            group_of[r] = mpxh_in_group1_windows(addr_of[r], group1, opt.group_size);
        } else {
            group_of[r] = mpxh_in_group1(name_of[r], group1, opt.group_size);
        }
    }
    if (win_cli)
        mpxh_pairing_windows(world, group_of, grank_of, gsize_of, peer_of);
    else
        mpxh_pairing(world, group_of, grank_of, gsize_of, peer_of);
    free(group1);

    if (win_cli && !opt.all_pairs) {
        /* every rank prints its INFO line to stdout right after the pairing
           (windows/mpi-perf.cpp:303-306); a rank without a peer dereferences
           the NULL peer_node_info there */
        for (int r = 0; r < world; ++r) {
            if (procs && r != me) continue;
            const int p = peer_of[r];
            if (p < 0) raise(SIGSEGV);
            char line[1024];
            mpxh_format_info(line, sizeof line, name_of[r], r, world, group_of[r], gsize_of[r], grank_of[r], p,
                             addr_of[r], name_of[p], addr_of[p]);
            fputs(line, stdout);
        }
        fflush(stdout);
    }

    if (!opt.all_pairs) {
        for (int r = 0; r < world; ++r) {
            if (peer_of[r] < 0 && (!procs || r == me)) { /* get_ipaddress(NULL peer), mpi_perf.c:180-184 */
                fprintf(stderr, "getaddrinfo error: rank %d (%s) has no peer in the other group\n", r, name_of[r]);
                mpx_abort();
            }
        }
        /* a rank whose peer is missing aborts the whole job (MPI_Abort) */
        for (int r = 0; r < world; ++r)
            if (peer_of[r] < 0) mpx_abort();
    }
    if (procs) check_pairs_share_a_node();
    if (!procs) { /* threads mode: rank r on GPU -g[r], else r mod #GPUs */
        if (!opt.use_dotnet) MPX_CHECK(mpx_device_count(&ndev));
        if (opt.gpus[0]) {
            if (ngl < world) {
                fprintf(stderr, "-g lists fewer GPUs than ranks (%d)\n", world);
                mpx_abort();
            }
            for (int r = 0; r < world; ++r) dev_of[r] = gl[r];
        } else {
            for (int r = 0; r < world; ++r) dev_of[r] = r % ndev;
        }
        for (int r = 0; r < world; ++r) {
            if (dev_of[r] >= ndev) {
                fprintf(stderr, "rank %d: GPU %d not visible (%d GPUs)\n", r, dev_of[r], ndev);
                mpx_abort();
            }
            snprintf(ip_of[r], sizeof ip_of[r], "%s", node_ip); /* the host's IPv4, mpi_perf.c:236-237 */
        }
    }
    if (!opt.all_pairs && !win_cli) {
        for (int r = 0; r < world; ++r) {
            if (procs && r != me) continue; /* every rank prints its own line, mpi_perf.c:460-461 */
            char line[1024];
            const int p = peer_of[r];
            mpxh_format_info(line, sizeof line, name_of[r], r, world, group_of[r], gsize_of[r], grank_of[r], p,
                             ip_of[r], name_of[p], ip_of[p]);
            fputs(line, stderr);
        }
    } else if (opt.all_pairs && is_root()) {
        for (int rd = 0; rd < world - 1; ++rd) {
            int pairs[MPXH_MAX_RANKS / 2][2];
            const int np = mpxh_round_pairs(world, rd, pairs);
            fprintf(stderr, "ROUND %d:", rd);
            for (int k = 0; k < np; ++k) fprintf(stderr, " (%d,%d)", pairs[k][0], pairs[k][1]);
            fprintf(stderr, "\n");
        }
    }

    /* sizes: one -b, or the -S power-of-two sweep */
    if (opt.sweep_min > 0) {
        for (long long b = opt.sweep_min; b <= opt.sweep_max && nsizes < 40; b *= 2) sizes[nsizes++] = (int)b;
    } else {
        sizes[nsizes++] = opt.buff_sz;
    }
    int maxb = 1;
    for (int i = 0; i < nsizes; ++i)
        if (sizes[i] > maxb) maxb = sizes[i];

    if (procs && !opt.use_dotnet) {
        MPX_CHECK(mpx_device_count(&ndev));
        if (dev_of[me] >= ndev) {
            fprintf(stderr, "rank %d: GPU %d not visible (%d GPUs; -g maps node-local ranks to GPUs)\n", me,
                    dev_of[me], ndev);
            mpx_abort();
        }
    }
    if (opt.logfolder[0]) mkdir(opt.logfolder, 0755);
    if (!opt.use_dotnet) { /* allocate_tx_rx_buffers, mpi_perf.c:463-468 */
        MPX_CHECK(mpx_init(world, opt.engine, &ctx));
        for (int r = 0; r < world; ++r) {
            if (procs && r != me) continue;
            MPX_CHECK(mpx_alloc(ctx, dev_of[r], (size_t)maxb, &tx_of[r]));
            MPX_CHECK(mpx_alloc(ctx, dev_of[r], (size_t)maxb, &rx_of[r]));
            MPX_CHECK(mpx_fill(ctx, dev_of[r], rx_of[r], (size_t)maxb, MPX_FILL_BYTE, 0));
            MPX_CHECK(mpx_rank_attach(ctx, r, dev_of[r], tx_of[r], rx_of[r], (size_t)maxb));
        }
        if (procs)
            connect_ranks();
        else if (opt.engine == MPX_ENGINE_RCCL) {
            MPX_CHECK(mpx_rccl_init_all(ctx));
            note_rccl_build();
        }
    }

    if (procs) {
        open_start_barrier();
        barrier();
        rank_main((void *)(intptr_t)me);
        barrier(); /* MPI_Barrier, mpi_perf.c:579: no peer still maps our buffers */
        if (ctx) MPX_CHECK(mpx_finalize(ctx)); /* frees tx/rx too */
        /* the pooled rank streams go before exit, as in threads mode below.
           Round 4 left them to the runtime here: the destroy stalled 1 exit
           in 4 (profiles/r04_procs_exit_stall.txt) — HIP's completion handler
           of the stream's last host function dropped the last reference on
           the HSA events thread, whose queue destroy then waited for itself.
           mpx_shutdown's fence now waits for that handler to return first
           (event_thread_barrier, DESIGN.md §5 "Exit"). */
        if (ctx) MPX_CHECK(mpx_shutdown());
        barrier();
        mpxb_spin_close(start_bar, 0);
        mpxb_finalize(boot);
        return 0;
    }

    pthread_barrier_init(&bar, NULL, (unsigned)world);
    open_start_barrier();
    pthread_t th[MPXH_MAX_RANKS];
    for (int r = 0; r < world; ++r) pthread_create(&th[r], NULL, rank_main, (void *)(intptr_t)r);
    for (int r = 0; r < world; ++r) pthread_join(th[r], NULL);
    pthread_barrier_destroy(&bar);
    mpxb_spin_close(start_bar, 0);

    if (!opt.use_dotnet) {
        for (int r = 0; r < world; ++r) {
            MPX_CHECK(mpx_free(ctx, tx_of[r]));
            MPX_CHECK(mpx_free(ctx, rx_of[r]));
        }
    }
    if (ctx) MPX_CHECK(mpx_finalize(ctx));
    /* one process, threads: the pooled rank streams go before exit — left
       to the HIP runtime's exit teardown, a profiler tool's exit-time
       finalizer (rocprofiler-sdk, as under rocprofv3 --pmc) faulted on them
       in libhsa-runtime64 (profiles/r04_exit_segv_stack.txt) */
    if (ctx) MPX_CHECK(mpx_shutdown());
    return 0;
}
