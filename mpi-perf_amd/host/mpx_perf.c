/*
 * mpx_perf.c — mpi_perf for the GPUs of one MI355X node.
 *
 * Same command line, group/peer rule, run loop, timing, CSV records and log
 * rotation as /root/reference/mpi_perf.c:367-582, but the ranks are host
 * threads of one process, one per GPU, and the transfer loop is libmpx's
 * mpx_xfer_ex (kernel / SDMA / RCCL engines over xGMI) instead of MPI p2p.
 *
 *   mpirun -np N --map-by ppr:P:node mpi_perf -f g1 -n 1 -p P ...   (reference)
 *   mpx_perf -w N -f g1 -n 1 -p P ...                                 (here)
 *
 * Ranks [k*P, (k+1)*P) form virtual host k, named "<node>-<k>" (the
 * processor name each rank matches against the -f file, mpi_perf.c:433-444;
 * MPX_PROCESSOR_NAMES="a,a,b,b" overrides).  With -a 1 every run is one round
 * of the circle-method all-pairs schedule instead of the fixed pairing.
 */
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include <errno.h>
#include <pthread.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "../../include/mpx.h"
#include "mpx_host.h"

/* MPI_CHECK analogue, mpi_perf.c:55-64: print and exit(EXIT_FAILURE) */
#define MPX_CHECK(stmt)                                                                                  \
    do {                                                                                                 \
        int mpx_errno = (stmt);                                                                          \
        if (MPX_OK != mpx_errno) {                                                                       \
            fprintf(stderr, "[%s:%d] mpx call failed with %d (%s: %s) \n", __FILE__, __LINE__, mpx_errno, \
                    mpx_strerror(mpx_errno), mpx_last_error());                                          \
            exit(EXIT_FAILURE);                                                                          \
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

static double wtime(void) /* MPI_Wtime */
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void barrier(void) { pthread_barrier_wait(&bar); }

/* kusto_injest, mpi_perf.c:355-365: only node-local rank 0; the command is
   site configuration here (MPX_INGEST_CMD) instead of a hard-coded path */
static void ingest_hook(int rank)
{
    const char *cmd = getenv("MPX_INGEST_CMD");
    if (rank % (opt.ppn > 0 ? opt.ppn : 1) != 0 || !cmd || !*cmd) return;
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
                           "WallTimems,DeviceTimems,GBps,Protocol,Workgroups,CheckedPayloads,CheckFailures,RunId\n");
    f->t_last_logtime = wtime();
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
                barrier();
                MPX_CHECK(mpx_checksum(ctx, dev_of[r], tx_of[r], (size_t)B, &txsum_of[r]));
                MPX_CHECK(mpx_checksum(ctx, dev_of[r], tx_of[r], 1, &txsum1_of[r]));
                barrier();
                xo.check = 1;
                xo.expect_checksum = txsum_of[peer];
                xo.expect_ack = txsum1_of[peer];
            }

            barrier(); /* MPI_Barrier, mpi_perf.c:499 */
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
                    static const char *proto[] = {"ll", "bulk", "sdma", "rccl", "copy"};
                    fprintf(files.gpu_fp, "%s,%s,%d,%s,%d,%d,%d,%d,%d,%d,%.4f,%.4f,%.3f,%s,%d,%llu,%d,%lld\n", ts,
                            opt.uuid, r, mpxh_engine_name(opt.engine), xfer_mode(), dev_of[r], peer, dev_of[peer], B,
                            opt.iters, my_time * 1e3, tm.device_s * 1e3, gbps,
                            (tm.protocol >= 0 && tm.protocol <= 4) ? proto[tm.protocol] : "?", tm.nwg,
                            (unsigned long long)tm.check_iters, tm.check_failures, run_idx);
                }
            }

            time_of[r] = my_time;
            barrier(); /* MPI_Barrier, mpi_perf.c:557 */
            const double t_end = wtime();
            if (r == 0 && (run_idx % 1000 == 0)) { /* Allreduce MIN/MAX/SUM + print, :560-568 */
                double mn = time_of[0], mx = time_of[0], sum = 0;
                for (int q = 0; q < world; ++q) {
                    if (time_of[q] < mn) mn = time_of[q];
                    if (time_of[q] > mx) mx = time_of[q];
                    sum += time_of[q];
                }
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

int main(int argc, char **argv)
{
    mpxh_defaults(&opt);
    const int pst = mpxh_parse_args(&opt, argc, argv);
    if (pst == MPXH_PARSE_USAGE) {
        mpxh_print_usage(stderr);
        mpx_abort();
    }
    if (pst == MPXH_PARSE_BAD_VALUE) {
        fprintf(stderr, "bad value for -e / -S\n");
        mpxh_print_usage(stderr);
        mpx_abort();
    }
    fprintf(stderr, "UUID: %s\n", opt.uuid); /* mpi_perf.c:338 */
#ifdef REPORT_BANDWIDTH
    report_bandwidth = 1;
#else
    report_bandwidth = getenv("MPX_REPORT_BANDWIDTH") != NULL;
#endif

    if (getenv("MPX_LOG_REFRESH_SEC")) log_refresh_sec = atof(getenv("MPX_LOG_REFRESH_SEC"));
    world = opt.world > 0 ? opt.world : (opt.ppn > 0 ? 2 * opt.ppn : 2);
    if (world > MPXH_MAX_RANKS || world > MPX_MAX_RANKS) {
        fprintf(stderr, "at most %d ranks\n", MPXH_MAX_RANKS);
        mpx_abort();
    }
    const int v = mpxh_validate(&opt, world, stderr); /* mpi_perf.c:399-403 */
    if (v == 2) raise(SIGFPE);
    if (v) mpx_abort();
    char *group1 = mpxh_read_group1(opt.group1_hostfile, opt.group_size);
    if (!group1) {
        fprintf(stderr, "cannot open group1 file: %s\n", opt.group1_hostfile);
        mpx_abort();
    }
    if (opt.all_pairs && (world < 2 || (world & 1))) {
        fprintf(stderr, "-a 1 needs an even number of ranks (-w)\n");
        mpx_abort();
    }

    /* processor names and the group/peer rule, mpi_perf.c:433-458 */
    char node[MPXH_MAX_HOST] = {0};
    gethostname(node, sizeof node - 1);
    char node_ip[MPXH_MAX_HOST] = "127.0.0.1";
    if (mpxh_ipv4(node, node_ip, sizeof node_ip) != 0) snprintf(node_ip, sizeof node_ip, "127.0.0.1");
    const char *names_env = getenv("MPX_PROCESSOR_NAMES");
    for (int r = 0; r < world; ++r) {
        mpxh_processor_name(name_of[r], node, r, opt.ppn, names_env);
        group_of[r] = mpxh_in_group1(name_of[r], group1, opt.group_size);
    }
    mpxh_pairing(world, group_of, grank_of, gsize_of, peer_of);
    free(group1);

    if (!opt.all_pairs) {
        for (int r = 0; r < world; ++r) {
            if (peer_of[r] < 0) { /* get_ipaddress(NULL peer host) aborts, mpi_perf.c:180-184 */
                fprintf(stderr, "getaddrinfo error: rank %d (%s) has no peer in the other group\n", r, name_of[r]);
                mpx_abort();
            }
        }
    }

    /* the .NET mode only prints launcher lines (mpi_perf.c:147-168) and, like
       the reference, allocates nothing: it needs no GPU */
    int ndev = world;
    if (!opt.use_dotnet) MPX_CHECK(mpx_device_count(&ndev));
    if (opt.gpus[0]) {
        if (mpxh_parse_gpu_list(opt.gpus, dev_of, MPXH_MAX_RANKS) < world) {
            fprintf(stderr, "-g lists fewer GPUs than ranks (%d)\n", world);
            mpx_abort();
        }
    } else {
        for (int r = 0; r < world; ++r) dev_of[r] = r % ndev;
    }
    for (int r = 0; r < world; ++r) {
        if (dev_of[r] >= ndev) {
            fprintf(stderr, "rank %d: GPU %d not visible (%d GPUs)\n", r, dev_of[r], ndev);
            mpx_abort();
        }
        snprintf(ip_of[r], sizeof ip_of[r], "%s:gpu%d", node_ip, dev_of[r]);
    }
    if (!opt.all_pairs) {
        for (int r = 0; r < world; ++r) {
            char line[1024];
            const int p = peer_of[r];
            mpxh_format_info(line, sizeof line, name_of[r], r, world, group_of[r], gsize_of[r], grank_of[r], p,
                             ip_of[r], name_of[p], ip_of[p]);
            fputs(line, stderr);
        }
    } else {
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

    if (opt.logfolder[0]) mkdir(opt.logfolder, 0755);
    if (!opt.use_dotnet) MPX_CHECK(mpx_init(world, opt.engine, &ctx));
    if (!opt.use_dotnet) { /* allocate_tx_rx_buffers, mpi_perf.c:463-468 */
        for (int r = 0; r < world; ++r) {
            MPX_CHECK(mpx_alloc(ctx, dev_of[r], (size_t)maxb, &tx_of[r]));
            MPX_CHECK(mpx_alloc(ctx, dev_of[r], (size_t)maxb, &rx_of[r]));
            MPX_CHECK(mpx_fill(ctx, dev_of[r], rx_of[r], (size_t)maxb, MPX_FILL_BYTE, 0));
            MPX_CHECK(mpx_rank_attach(ctx, r, dev_of[r], tx_of[r], rx_of[r], (size_t)maxb));
        }
        if (opt.engine == MPX_ENGINE_RCCL) MPX_CHECK(mpx_rccl_init_all(ctx));
    }

    pthread_barrier_init(&bar, NULL, (unsigned)world);
    pthread_t th[MPXH_MAX_RANKS];
    for (int r = 0; r < world; ++r) pthread_create(&th[r], NULL, rank_main, (void *)(intptr_t)r);
    for (int r = 0; r < world; ++r) pthread_join(th[r], NULL);
    pthread_barrier_destroy(&bar);

    if (!opt.use_dotnet) {
        for (int r = 0; r < world; ++r) {
            MPX_CHECK(mpx_free(ctx, tx_of[r]));
            MPX_CHECK(mpx_free(ctx, rx_of[r]));
        }
    }
    if (ctx) MPX_CHECK(mpx_finalize(ctx));
    return 0;
}
