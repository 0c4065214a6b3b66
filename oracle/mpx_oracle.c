/*
 * mpx_oracle.c — CPU restatement of mpi_perf's hot path (see mpx_oracle.h).
 *
 * TEST INFRASTRUCTURE ONLY: the checker for libmpx and the timed CPU
 * baseline ("kind": "port") of bench.py.  Never linked into the product.
 * Restates /root/reference/mpi_perf.c; each function cites the lines.
 * Pinned against the compiled reference by tests/golden (gen_golden.py).
 */
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include "mpx_oracle.h"

#include <ctype.h>
#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define GOLDEN 0x9E3779B97F4A7C15ULL

uint64_t oracle_mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

uint64_t oracle_checksum(const void *buf, size_t n)
{
    const unsigned char *p = (const unsigned char *)buf;
    uint64_t s = 0;
    size_t k = 0;
    for (; 8 * k + 8 <= n; ++k) {
        uint64_t w;
        memcpy(&w, p + 8 * k, 8); /* little-endian host, like the GPU */
        s += oracle_mix64(w + (k + 1) * GOLDEN);
    }
    if (8 * k < n) {
        uint64_t w = 0;
        for (size_t b = 0; 8 * k + b < n; ++b) w |= (uint64_t)p[8 * k + b] << (8 * b);
        s += oracle_mix64(w + (k + 1) * GOLDEN);
    }
    return s ^ oracle_mix64((uint64_t)n);
}

void oracle_fill(void *buf, size_t n, int pattern, uint64_t arg)
{
    unsigned char *p = (unsigned char *)buf;
    if (pattern == 0) { /* memset, mpi_perf.c:246,250 */
        memset(p, (int)(arg & 0xff), n);
        return;
    }
    for (size_t k = 0; 8 * k < n; ++k) {
        const uint64_t w = oracle_mix64((arg ^ k) + GOLDEN);
        for (size_t b = 0; b < 8 && 8 * k + b < n; ++b) p[8 * k + b] = (unsigned char)(w >> (8 * b));
    }
}

/* mpi_perf.c:34-53 */
int oracle_strnicmp(const char *s1, const char *s2, size_t n)
{
    for (size_t i = 0; i < n; i++) {
        const int c1 = tolower((unsigned char)s1[i]);
        const int c2 = tolower((unsigned char)s2[i]);
        if (c1 != c2) return c1 - c2;
        if (c1 == '\0') break;
    }
    return 0;
}

/* mpi_perf.c:438-444: compare name_len chars of my name against each line */
int oracle_in_group1(const char *name, int name_len, const char *lines, int group_size)
{
    int g = 0;
    for (int i = 0; i < group_size; i++)
        if (oracle_strnicmp(name, lines + (size_t)i * ORACLE_MAX_HOST, (size_t)name_len) == 0) g = 1;
    return g;
}

/* mpi_perf.c:447-450 (Comm_split keyed by world rank) and :225-233 */
void oracle_pairing(int world, const int *group, int *group_rank, int *peer)
{
    for (int r = 0; r < world; ++r) {
        int gr = 0;
        for (int q = 0; q < r; ++q) gr += group[q] == group[r];
        group_rank[r] = gr;
    }
    for (int r = 0; r < world; ++r) {
        peer[r] = -1;
        for (int i = 0; i < world; ++i)
            if (group[i] != group[r] && group_rank[i] == group_rank[r]) {
                peer[r] = i;
                break;
            }
    }
}

/* windows/mpi-perf.cpp:28-46 (my_strnicmp, same as mpi_perf.c's), :256-260
   (newline cut), :283-289 (n = MAX_HOST_SZ: the whole string) */
int oracle_win_in_group1(const char *addr, const char *lines, int group_size)
{
    int g = 0;
    char line[ORACLE_MAX_HOST];
    for (int i = 0; i < group_size; i++) {
        memcpy(line, lines + (size_t)i * ORACLE_MAX_HOST, ORACLE_MAX_HOST);
        line[ORACLE_MAX_HOST - 1] = '\0';
        line[strcspn(line, "\n")] = '\0';
        if (oracle_strnicmp(addr, line, ORACLE_MAX_HOST) == 0) g = 1;
    }
    return g;
}

/* windows/mpi-perf.cpp:292-295 and :125-132 (no break: the last match) */
void oracle_win_pairing(int world, const int *group, int *group_rank, int *peer)
{
    for (int r = 0; r < world; ++r) {
        int gr = 0;
        for (int q = 0; q < r; ++q) gr += group[q] == group[r];
        group_rank[r] = gr;
    }
    for (int r = 0; r < world; ++r) {
        peer[r] = -1;
        for (int i = 0; i < world; ++i)
            if (group[i] != group[r] && group_rank[i] == group_rank[r]) peer[r] = i;
    }
}

/* mpi_perf.c:95-124 */
long long oracle_nb_waited(long long iters)
{
    long long waited = 0;
    int inflight = 0;
    for (long long i = 0; i < iters; i++) {
        if (inflight == 255) {
            waited += inflight;
            inflight = 0;
        } else {
            inflight++;
        }
    }
    return waited + inflight;
}

/* ------------------------------------------------------------------------ */
/* CPU engine: ranks are threads, a message is a memcpy into the peer's rx  */
/* followed by a release increment of the peer's arrival counter.           */
/* ------------------------------------------------------------------------ */
typedef struct {
    unsigned char *tx, *rx;
    _Atomic uint64_t arrived; /* messages delivered into rx */
} oracle_ep;

typedef struct {
    oracle_ep *ep;            /* [2*npairs] */
    int npairs, mode, iters;
    size_t B;
    int digest;
    pthread_barrier_t bar;
    oracle_rank_stats *st;
} oracle_job;

typedef struct {
    oracle_job *job;
    int rank;
} oracle_arg;

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void o_send(oracle_ep *me, oracle_ep *peer, size_t n, oracle_rank_stats *st)
{
    memcpy(peer->rx, me->tx, n);
    atomic_fetch_add_explicit(&peer->arrived, 1, memory_order_release);
    st->sent_bytes += n;
}

static void o_wait(oracle_ep *me, uint64_t count)
{
    unsigned spins = 0;
    while (atomic_load_explicit(&me->arrived, memory_order_acquire) < count)
        if (++spins % 64 == 0) sched_yield();
}

static void o_recv_done(oracle_job *j, oracle_ep *me, size_t n, uint64_t k, oracle_rank_stats *st)
{
    st->recv_done += k;
    st->recv_bytes += k * n;
    if (j->digest) st->recv_digest += k * oracle_checksum(me->rx, n);
}

static void *oracle_thread(void *argp)
{
    oracle_arg *a = (oracle_arg *)argp;
    oracle_job *j = a->job;
    const int r = a->rank;
    const int group = r < j->npairs ? 1 : 0; /* ranks [0,ppn) are group 1 */
    const int peer = group ? r + j->npairs : r - j->npairs;
    oracle_ep *me = &j->ep[r], *pe = &j->ep[peer];
    oracle_rank_stats *st = &j->st[r];
    const size_t B = j->B;
    uint64_t got = 0;

    pthread_barrier_wait(&j->bar); /* MPI_Barrier, mpi_perf.c:499 */
    const double t0 = now_s();
    if (j->mode == ORACLE_PINGPONG) { /* mpi_perf.c:70-82 */
        for (int i = 0; i < j->iters; i++) {
            if (group == 1) {
                o_send(me, pe, B, st);
                o_wait(me, ++got);
                o_recv_done(j, me, B, 1, st);
            } else {
                o_wait(me, ++got);
                o_recv_done(j, me, B, 1, st);
                o_send(me, pe, B, st);
            }
        }
    } else if (j->mode == ORACLE_UNIDIR) { /* mpi_perf.c:132-144 */
        for (int i = 0; i < j->iters; i++) {
            if (group == 1) {
                o_send(me, pe, B, st);
                o_wait(me, ++got);
                o_recv_done(j, me, 1, 1, st); /* Recv(rx, 1) */
            } else {
                o_wait(me, ++got);
                o_recv_done(j, me, B, 1, st);
                memcpy(pe->rx, me->tx, 1); /* Send(tx, 1) */
                atomic_fetch_add_explicit(&pe->arrived, 1, memory_order_release);
                st->sent_bytes += 1;
            }
        }
    } else { /* mpi_perf.c:95-124 */
        int inflight = 0;
        for (int i = 0; i < j->iters; i++) {
            o_send(me, pe, B, st); /* Isend (buffered: completes at once) */
            if (inflight == 255) {
                o_wait(me, (uint64_t)i); /* Waitall(255): receives 0..i-1 */
                o_recv_done(j, me, B, (uint64_t)inflight, st);
                inflight = 0;
            } else {
                inflight++;
            }
        }
        if (inflight > 0) {
            o_wait(me, (uint64_t)j->iters);
            o_recv_done(j, me, B, (uint64_t)inflight, st);
        }
    }
    st->time_s = now_s() - t0; /* mpi_perf.c:532-533 */
    /* the peer may still be writing our rx after our loop returned (nb
       mode's leaked slot): drain before the buffers go away */
    pthread_barrier_wait(&j->bar);
    return NULL;
}

int oracle_run_pairs(int npairs, int mode, int iters, size_t B, oracle_rank_stats *stats, double *max_time)
{
    const int world = 2 * npairs;
    oracle_job j;
    memset(&j, 0, sizeof j);
    j.npairs = npairs;
    j.mode = mode;
    j.iters = iters;
    j.B = B;
    j.digest = getenv("ORACLE_NO_DIGEST") == NULL;
    j.st = stats;
    j.ep = (oracle_ep *)calloc((size_t)world, sizeof(oracle_ep));
    if (!j.ep) return -1;
    for (int r = 0; r < world; ++r) {
        const size_t cap = B ? B : 1;
        if (posix_memalign((void **)&j.ep[r].tx, 4096, cap) || posix_memalign((void **)&j.ep[r].rx, 4096, cap))
            return -1;
        /* allocate_tx_rx_buffers, mpi_perf.c:244-251: group 0 'a', group 1 'b'.
           At B = 0 the memset writes nothing, yet the unidir ack still sends
           tx[0] (:142): a fresh glibc chunk's 0 (golden zero_bytes_unidir) */
        memset(j.ep[r].tx, B ? (r < npairs ? 'b' : 'a') : 0, cap);
        memset(j.ep[r].rx, 0, cap);
        atomic_init(&j.ep[r].arrived, 0);
        memset(&stats[r], 0, sizeof stats[r]);
    }
    pthread_barrier_init(&j.bar, NULL, (unsigned)world);
    pthread_t *th = (pthread_t *)calloc((size_t)world, sizeof(pthread_t));
    oracle_arg *args = (oracle_arg *)calloc((size_t)world, sizeof(oracle_arg));
    for (int r = 0; r < world; ++r) {
        args[r].job = &j;
        args[r].rank = r;
        pthread_create(&th[r], NULL, oracle_thread, &args[r]);
    }
    double mx = 0;
    for (int r = 0; r < world; ++r) {
        pthread_join(th[r], NULL);
        if (stats[r].time_s > mx) mx = stats[r].time_s;
    }
    if (max_time) *max_time = mx;
    pthread_barrier_destroy(&j.bar);
    for (int r = 0; r < world; ++r) {
        free(j.ep[r].tx);
        free(j.ep[r].rx);
    }
    free(j.ep);
    free(th);
    free(args);
    return 0;
}

int oracle_run_pair(int mode, int iters, size_t B, oracle_rank_stats stats[2])
{
    oracle_rank_stats s[2];
    const int rc = oracle_run_pairs(1, mode, iters, B, s, NULL);
    stats[1] = s[0]; /* world rank 0 is group 1 */
    stats[0] = s[1];
    return rc;
}

/* mpi_perf.c:551-554 */
int oracle_format_record(char *out, size_t cap, const char *timestamp, const char *uuid, int world_rank,
                         int world_size, int ppn, const char *local_ip, const char *remote_ip, int buff_len,
                         int iters, double my_time_s, long long run_idx)
{
    return snprintf(out, cap, "%s,%s,%d,%d,%s,%s,%d,%d,%d,%.2lf,%lld\n", timestamp, uuid, world_rank,
                    world_size / ppn, local_ip, remote_ip, ppn, buff_len, iters, my_time_s * 1000.0, run_idx);
}

/* mpi_perf.c:494 */
int oracle_log_name(char *out, size_t cap, const char *logfolder, const char *uuid, int world_rank,
                    const char *file_time)
{
    return snprintf(out, cap, "%s/tcp-%s-%d-%s.log", logfolder, uuid, world_rank, file_time);
}

/* mpi_perf.c:538-539 */
double oracle_gbps(int buff_len, int iters, int uni_dir, double my_time_s)
{
    const long double gbits = 8.0 * buff_len * iters * ((uni_dir == 1) ? 1.0 : 2.0) * 1e-9;
    return (double)(gbits / my_time_s);
}
