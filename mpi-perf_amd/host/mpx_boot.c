/*
 * mpx_boot.c — TCP job communicator for mpx_perf's multi-process mode (see
 * mpx_boot.h).  Rank 0 is the hub: every collective is "leaves send to the
 * hub, the hub answers every leaf", so one collective costs two message
 * latencies whatever the job size (a job is one node's GPUs or a few nodes).
 * Nothing here is on the timed path.
 */
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include "mpx_boot.h"

#include <arpa/inet.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#define MPXB_MAGIC 0x6d70786230303031ULL /* "mpxb0001" */
#define MPXB_MAX 64

struct mpxb {
    int rank, size;
    int fd[MPXB_MAX]; /* hub: fd[r] = leaf r; leaf: fd[0] = hub */
};

static __thread char g_err[256];

static int err(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return -1;
}

const char *mpxb_error(void) { return g_err; }

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static const char *first_env(const char *const *names)
{
    for (; *names; ++names) {
        const char *v = getenv(*names);
        if (v && *v) return v;
    }
    return NULL;
}

int mpxb_launcher(int *rank, int *size, int *local)
{
    static const char *const R[] = {"MPX_RANK", "RANK", "PMI_RANK", "OMPI_COMM_WORLD_RANK", "SLURM_PROCID", NULL};
    static const char *const S[] = {"MPX_SIZE", "WORLD_SIZE", "PMI_SIZE", "OMPI_COMM_WORLD_SIZE", "SLURM_NTASKS", NULL};
    static const char *const L[] = {"MPX_LOCAL_RANK", "LOCAL_RANK", "MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK",
                                    "SLURM_LOCALID", NULL};
    const char *r = first_env(R), *s = first_env(S), *l = first_env(L);
    *rank = 0;
    *size = 1;
    *local = 0;
    if (!r || !s) return 0;
    *rank = atoi(r);
    *size = atoi(s);
    *local = l ? atoi(l) : *rank;
    return 1;
}

int mpxb_address(char *host, size_t cap)
{
    const char *b = getenv("MPX_BOOTSTRAP");
    if (b && *b) {
        const char *colon = strrchr(b, ':');
        if (colon) {
            size_t n = (size_t)(colon - b);
            if (n >= cap) n = cap - 1;
            memcpy(host, b, n);
            host[n] = 0;
            return atoi(colon + 1);
        }
    }
    const char *ma = getenv("MASTER_ADDR"), *mp = getenv("MASTER_PORT");
    if (ma && *ma && mp && *mp) {
        snprintf(host, cap, "%s", ma);
        return atoi(mp) + 1;
    }
    snprintf(host, cap, "127.0.0.1");
    return 29571;
}

static int send_all(int fd, const void *p, size_t n)
{
    const unsigned char *c = (const unsigned char *)p;
    while (n) {
        const ssize_t k = send(fd, c, n, MSG_NOSIGNAL);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return err("send: %s", k < 0 ? strerror(errno) : "connection closed");
        c += k;
        n -= (size_t)k;
    }
    return 0;
}

static int recv_all(int fd, void *p, size_t n)
{
    unsigned char *c = (unsigned char *)p;
    while (n) {
        const ssize_t k = recv(fd, c, n, 0);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return err("recv: %s", k < 0 ? strerror(errno) : "connection closed (a rank exited)");
        c += k;
        n -= (size_t)k;
    }
    return 0;
}

static void tune(int fd)
{
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
}

static int resolve(const char *host, int port, struct sockaddr_in *sa)
{
    memset(sa, 0, sizeof *sa);
    sa->sin_family = AF_INET;
    sa->sin_port = htons((uint16_t)port);
    if (inet_pton(AF_INET, host, &sa->sin_addr) == 1) return 0;
    struct addrinfo hints, *res;
    memset(&hints, 0, sizeof hints);
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host, NULL, &hints, &res) != 0) return err("cannot resolve bootstrap host %s", host);
    sa->sin_addr = ((struct sockaddr_in *)res->ai_addr)->sin_addr;
    freeaddrinfo(res);
    return 0;
}

typedef struct {
    uint64_t magic;
    int32_t rank, size;
} hello;

static int hub_accept(mpxb *b, const struct sockaddr_in *sa, double timeout_s)
{
    const int ls = socket(AF_INET, SOCK_STREAM, 0);
    if (ls < 0) return err("socket: %s", strerror(errno));
    int one = 1;
    setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    struct sockaddr_in any = *sa;
    any.sin_addr.s_addr = htonl(INADDR_ANY);
    if (bind(ls, (const struct sockaddr *)&any, sizeof any) != 0 || listen(ls, MPXB_MAX) != 0) {
        const int e = errno;
        close(ls);
        return err("bootstrap: cannot listen on port %d: %s", ntohs(sa->sin_port), strerror(e));
    }
    const double deadline = now_s() + timeout_s;
    int joined = 1;
    while (joined < b->size) {
        struct pollfd pf = {ls, POLLIN, 0};
        const int left_ms = (int)((deadline - now_s()) * 1e3);
        if (left_ms <= 0 || poll(&pf, 1, left_ms) <= 0) {
            close(ls);
            return err("bootstrap: only %d of %d ranks joined", joined, b->size);
        }
        const int fd = accept(ls, NULL, NULL);
        if (fd < 0) continue;
        tune(fd);
        hello h;
        if (recv_all(fd, &h, sizeof h) != 0 || h.magic != MPXB_MAGIC || h.size != b->size || h.rank <= 0 ||
            h.rank >= b->size || b->fd[h.rank] >= 0) {
            close(fd); /* a stray or duplicate connection */
            continue;
        }
        b->fd[h.rank] = fd;
        ++joined;
    }
    close(ls);
    return 0;
}

static int leaf_connect(mpxb *b, const struct sockaddr_in *sa, double timeout_s)
{
    const double deadline = now_s() + timeout_s;
    for (;;) {
        const int fd = socket(AF_INET, SOCK_STREAM, 0);
        if (fd < 0) return err("socket: %s", strerror(errno));
        if (connect(fd, (const struct sockaddr *)sa, sizeof *sa) == 0) {
            tune(fd);
            hello h = {MPXB_MAGIC, b->rank, b->size};
            if (send_all(fd, &h, sizeof h) != 0) {
                close(fd);
                return -1;
            }
            b->fd[0] = fd;
            return 0;
        }
        const int e = errno;
        close(fd);
        if (now_s() > deadline) return err("bootstrap: cannot reach rank 0 (%s)", strerror(e));
        usleep(20000);
    }
}

int mpxb_init(mpxb **out, int rank, int size, const char *host, int port, double timeout_s)
{
    *out = NULL;
    if (size < 1 || size > MPXB_MAX || rank < 0 || rank >= size) return err("bad rank %d / size %d", rank, size);
    mpxb *b = (mpxb *)calloc(1, sizeof *b);
    if (!b) return err("out of memory");
    b->rank = rank;
    b->size = size;
    for (int i = 0; i < MPXB_MAX; ++i) b->fd[i] = -1;
    int rc = 0;
    if (size > 1) {
        struct sockaddr_in sa;
        rc = resolve(host, port, &sa);
        if (rc == 0) rc = rank == 0 ? hub_accept(b, &sa, timeout_s) : leaf_connect(b, &sa, timeout_s);
    }
    if (rc == 0) rc = mpxb_barrier(b);
    if (rc != 0) {
        mpxb_finalize(b);
        return -1;
    }
    *out = b;
    return 0;
}

void mpxb_finalize(mpxb *b)
{
    if (!b) return;
    for (int i = 0; i < MPXB_MAX; ++i)
        if (b->fd[i] >= 0) close(b->fd[i]);
    free(b);
}

int mpxb_rank(const mpxb *b) { return b->rank; }
int mpxb_size(const mpxb *b) { return b->size; }

int mpxb_allgather(mpxb *b, const void *mine, void *all, size_t bytes)
{
    unsigned char *a = (unsigned char *)all;
    if (b->rank != 0) {
        if (send_all(b->fd[0], mine, bytes) != 0) return -1;
        return recv_all(b->fd[0], a, bytes * (size_t)b->size);
    }
    memmove(a, mine, bytes);
    for (int r = 1; r < b->size; ++r)
        if (recv_all(b->fd[r], a + (size_t)r * bytes, bytes) != 0) return -1;
    for (int r = 1; r < b->size; ++r)
        if (send_all(b->fd[r], a, bytes * (size_t)b->size) != 0) return -1;
    return 0;
}

int mpxb_bcast0(mpxb *b, void *buf, size_t bytes)
{
    if (b->rank != 0) return recv_all(b->fd[0], buf, bytes);
    for (int r = 1; r < b->size; ++r)
        if (send_all(b->fd[r], buf, bytes) != 0) return -1;
    return 0;
}

int mpxb_barrier(mpxb *b)
{
    unsigned char one = 1, all[MPXB_MAX];
    return mpxb_allgather(b, &one, all, 1);
}

int mpxb_allreduce_f64(mpxb *b, double v, double *mn, double *mx, double *sum)
{
    double all[MPXB_MAX];
    if (mpxb_allgather(b, &v, all, sizeof v) != 0) return -1;
    double lo = all[0], hi = all[0], s = 0;
    for (int r = 0; r < b->size; ++r) {
        if (all[r] < lo) lo = all[r];
        if (all[r] > hi) hi = all[r];
        s += all[r];
    }
    if (mn) *mn = lo;
    if (mx) *mx = hi;
    if (sum) *sum = s;
    return 0;
}

/* ---- spin barrier ---------------------------------------------------------
 * A central counter + generation word (each on its own cache line); the
 * last arriver resets the counter and bumps the generation, everyone else
 * spins on the generation.  In a process (threads mode) or in a POSIX shm
 * object shared by the ranks of one node. */
struct spin_words {
    _Alignas(64) uint64_t count;
    _Alignas(64) uint64_t gen;
    _Alignas(64) int32_t n;
};

struct mpxb_spin {
    struct spin_words *w;
    int n;
    int shared;
    char name[128];
};

static double spin_now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int mpxb_spin_open(mpxb_spin **out, const char *name, int nranks, int create)
{
    *out = NULL;
    if (nranks < 1) return err("spin barrier of %d ranks", nranks);
    mpxb_spin *s = calloc(1, sizeof *s);
    if (!s) return err("out of memory");
    s->n = nranks;
    if (!name) {
        s->w = aligned_alloc(64, sizeof *s->w);
        if (!s->w) {
            free(s);
            return err("out of memory");
        }
        memset(s->w, 0, sizeof *s->w);
        s->w->n = nranks;
        *out = s;
        return 0;
    }
    snprintf(s->name, sizeof s->name, "%s", name);
    const int fd = shm_open(name, create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
    if (fd < 0) {
        free(s);
        return err("shm_open(%s): %s", name, strerror(errno));
    }
    if (create && ftruncate(fd, (off_t)sizeof(struct spin_words)) != 0) {
        close(fd);
        shm_unlink(name);
        free(s);
        return err("ftruncate(%s): %s", name, strerror(errno));
    }
    void *p = mmap(NULL, sizeof(struct spin_words), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
        if (create) shm_unlink(name);
        free(s);
        return err("mmap(%s): %s", name, strerror(errno));
    }
    s->w = p;
    s->shared = 1;
    if (create) __atomic_store_n(&s->w->n, nranks, __ATOMIC_RELEASE);   /* (ftruncate zeroed the words) */
    else {
        const int made = __atomic_load_n(&s->w->n, __ATOMIC_ACQUIRE);
        if (made != nranks) {
            mpxb_spin_close(s, 0);
            return err("spin barrier %s: made for %d ranks, not %d", name, made, nranks);
        }
    }
    *out = s;
    return 0;
}

int mpxb_spin_wait(mpxb_spin *s, double timeout_s)
{
    struct spin_words *w = s->w;
    const uint64_t g = __atomic_load_n(&w->gen, __ATOMIC_ACQUIRE);
    if (__atomic_add_fetch(&w->count, 1, __ATOMIC_ACQ_REL) == (uint64_t)s->n) {
        __atomic_store_n(&w->count, 0, __ATOMIC_RELAXED);
        __atomic_store_n(&w->gen, g + 1, __ATOMIC_RELEASE);
        return 0;
    }
    const double deadline = spin_now() + timeout_s;
    for (unsigned long k = 1; __atomic_load_n(&w->gen, __ATOMIC_ACQUIRE) == g; ++k) {
        __builtin_ia32_pause();
        if ((k & 4095) == 0) {
            if (spin_now() > deadline) return err("spin barrier: timed out after %.0f s", timeout_s);
            if (k > (1ul << 20)) sched_yield();   /* a long wait (a slow rank): give the core back now and then */
        }
    }
    return 0;
}

int mpxb_spin_wait_xfer(mpxb_spin *s, double timeout_s, mpxb_xfer_fn fn, void *ctx, int mode, int group, int rank,
                        int peer, int iters, void *tx, void *rx, int len, const void *opts, void *timing,
                        int *xfer_rc)
{
    if (!fn || !xfer_rc) return err("spin barrier: no transfer to start");
    const int st = mpxb_spin_wait(s, timeout_s);
    if (st != 0) return st;
    *xfer_rc = fn(ctx, mode, group, rank, peer, iters, tx, rx, len, opts, timing);
    return 0;
}

void mpxb_spin_close(mpxb_spin *s, int unlink_it)
{
    if (!s) return;
    if (s->shared) {
        munmap(s->w, sizeof(struct spin_words));
        if (unlink_it) shm_unlink(s->name);
    } else {
        free(s->w);
    }
    free(s);
}
