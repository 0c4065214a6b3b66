/*
 * mpx.h — C-ABI of libmpx, the MI355X transfer engine behind mpx_perf.
 *
 * This is the drop-in boundary for mpi_perf's hot path.  In the reference the
 * seam is the transfer-loop signature shared by the three loops
 *
 *   void do_mpi_benchmark*(int my_group, int my_rank, int peer_rank,
 *                          char *peer_host, char *my_host, int iters,
 *                          void *buffer_tx, void *buffer_rx, int buff_len)
 *
 *   (/root/reference/mpi_perf.c:66-67, :85-86, :127-128), called from main
 *   between t_start and t_end_local (mpi_perf.c:501-532) on buffers made by
 *   allocate_tx_rx_buffers (mpi_perf.c:240-252) and freed by main (:574-578).
 *
 * mpx_xfer() keeps that argument order (minus the two host strings, plus the
 * loop mode and an out-parameter for the elapsed time).  Every other entry
 * point replaces one MPI/libc call the reference makes around the loop; each
 * declaration cites the call it replaces.
 *
 * Conventions
 *  - Every function returns an int status: MPX_OK (0) or an MPX_ERR_* code;
 *    mpx_strerror() turns it into text.  The host wraps calls in MPX_CHECK,
 *    which mirrors the reference's MPI_CHECK print-and-exit (mpi_perf.c:55-64).
 *  - Plain pointers and sizes only; no HIP, RCCL or torch types cross the ABI.
 *  - Ownership: the caller allocates (mpx_alloc) and frees (mpx_free) tx/rx;
 *    transfer calls borrow them, exactly like the reference's loops.
 *  - Threading: one context may be shared by several host threads, one per
 *    rank; calls for different ranks may run concurrently.  Calls for the same
 *    rank must not.
 *  - A "rank" is a logical endpoint (the reference's MPI rank).  A rank lives
 *    on one GPU.  Ranks of the same context are "local" (attached with
 *    mpx_rank_attach); ranks living in another process are "imported" from
 *    the descriptor that process exported (mpx_rank_export/mpx_rank_import).
 */
#ifndef MPX_H
#define MPX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPX_ABI_VERSION 7
#define MPX_MAX_RANKS 64          /* ranks one context can address           */
#define MPX_RANK_DESC_BYTES 512   /* size of the opaque exported descriptor  */
#define MPX_RCCL_ID_BYTES 128     /* size of an RCCL unique id               */

/* ---- status codes ------------------------------------------------------ */
enum mpx_status {
    MPX_OK = 0,
    MPX_ERR_INVALID = 1,      /* bad argument (null, range, unknown rank)   */
    MPX_ERR_HIP = 2,          /* a HIP runtime call failed                  */
    MPX_ERR_NOMEM = 3,        /* device allocation failed                   */
    MPX_ERR_TIMEOUT = 4,      /* a device-side wait exceeded its deadline   */
    MPX_ERR_RCCL = 5,         /* an RCCL call failed                        */
    MPX_ERR_UNSUPPORTED = 6,  /* engine/mode combination not available      */
    MPX_ERR_STATE = 7,        /* call out of order (not attached, no comm)  */
    MPX_ERR_CHECK = 8         /* a received payload failed its checksum     */
};

/* ---- transfer engines (north_star (a)/(b)/(c)) ------------------------- */
enum mpx_engine {
    MPX_ENGINE_KERNEL = 0,    /* hand-written CDNA4 push kernels + device flags */
    MPX_ENGINE_SDMA = 1,      /* copy-engine hipMemcpyAsync (NoCU across GPUs)
                                 + one-lane signal / bounded-wait kernels       */
    MPX_ENGINE_RCCL = 2,      /* ncclSend/ncclRecv                              */
    MPX_ENGINE_HOST = 3       /* SURVEY §8b's CPU engine: not built; mpx_init
                                 returns MPX_ERR_UNSUPPORTED (the
                                 CPU side is the compiled reference itself, and
                                 libmpx has no CPU transfer path to fall into) */
};

/* ---- loop modes: the three reference loops ----------------------------- */
enum mpx_mode {
    MPX_MODE_PINGPONG = 0,    /* do_mpi_benchmark             mpi_perf.c:66-83   */
    MPX_MODE_NONBLOCKING = 1, /* do_mpi_benchmark_nonblocking mpi_perf.c:85-125  */
    MPX_MODE_UNIDIR = 2       /* do_mpi_benchmark_unidir      mpi_perf.c:127-145 */
};

/* ---- fill patterns ----------------------------------------------------- */
enum mpx_fill {
    MPX_FILL_BYTE = 0,        /* memset(ptr, arg & 0xff, n): the reference's
                                 'a'/'b' tx fill, mpi_perf.c:244-251           */
    MPX_FILL_SPLITMIX = 1     /* 64-bit word k = splitmix64(arg ^ k), tail
                                 bytes little-endian from the same word        */
};

/* key for MPX_FILL_SPLITMIX: seed ^ src<<56 ^ dst<<48 ^ iter<<24 */
#define MPX_PATTERN_SEED 0x6d70695f70657266ULL
static inline uint64_t mpx_pattern_key(uint64_t seed, unsigned src, unsigned dst,
                                       unsigned iter)
{
    return seed ^ ((uint64_t)src << 56) ^ ((uint64_t)dst << 48) ^ ((uint64_t)iter << 24);
}

/* ---- timing / statistics of one transfer call ---------------------------- */
typedef struct mpx_timing {
    double wall_s;            /* host wall clock around the loop (MPI_Wtime
                                 analogue, mpi_perf.c:501,532-533)             */
    double device_s;          /* hipEvent time of the loop on the rank's stream */
    uint64_t bytes;           /* algorithmic bytes of the loop (a9 formula:
                                 B*iters*(unidir?1:2), mpi_perf.c:538)         */
    int32_t launches;         /* kernels / copies issued for the loop          */
    int32_t nwg;              /* workgroups of the data push (kernel engine)   */
    int32_t protocol;         /* 0 = LL granules, 1 = bulk+flags, 2 = SDMA,
                                 3 = RCCL, 4 = local copy kernel (a launch per
                                 copy), 5 = local copy, all iterations in one
                                 launch (k_copy_steps), 6 = the same with the
                                 next copy's loads in flight (k_copy_pipe),
                                 7 = bulk payloads pulled by the receiver
                                 (MPX_XFER_PULL), 8 = the SDMA engine's
                                 pulled form                                    */
    int32_t check_failures;   /* iterations whose payload checksum mismatched  */
    uint64_t check_iters;     /* iterations whose payload was checksummed      */
    /* receive accounting, as the reference's loop completes receives: every
       Recv of ping-pong / unidir (mpi_perf.c:75,79,137,141), and the requests
       each MPI_Waitall of the non-blocking loop waits for (:110-111,122-123;
       slot 255 of each full window is never waited for).  Counted on the
       device (kernel engine always; SDMA / RCCL engines in check mode). */
    uint64_t recv_done;       /* receives completed                             */
    uint64_t recv_digest;     /* check mode: sum of mpx_checksum() of each of
                                 those received payloads (the golden fixtures'
                                 recv_digest); 0 otherwise                      */
} mpx_timing;

/* options of mpx_xfer_ex beyond the reference seam */
typedef struct mpx_xfer_opts {
    int32_t check;            /* 1: checksum + poison every received payload   */
    int32_t flags;            /* MPX_XFER_* bits below; 0 = defaults            */
    uint64_t expect_checksum; /* mpx_checksum() of the peer's tx[0:len) (B-byte
                                 receives) — required when check = 1           */
    uint64_t expect_ack;      /* mpx_checksum() of the peer's tx[0:1) (unidir
                                 G1's 1-byte acks)                             */
    uint32_t timeout_ms;      /* per-wait device deadline; 0 = default (10 s)  */
    int32_t nwg;              /* override push workgroups; 0 = automatic        */
} mpx_xfer_opts;

/* mpx_xfer_opts.flags: bulk payload stores carry the streaming (nontemporal)
   hint on top of their system-scope write-through policy (sc0 sc1 nt instead
   of sc0 sc1).  Visibility is unchanged, so the two sides need not agree. */
#define MPX_XFER_STREAM 1
/* mpx_xfer_opts.flags: every B-byte payload is PULLED: the sender publishes
   "tx holds message k" (one store into the receiver's mailbox) and the
   receiver loads the bytes from the sender's peer-mapped tx into its own rx —
   the kernel engine with its receiving kernel's loads, the SDMA engine with a
   copy on the receiver's stream — instead of the sender storing them into the
   receiver's rx.  Kernel engine: LL messages (<= the link's LL threshold)
   stay pushes; both engines push the unidir 1-byte ack.  Both sides of a
   link must set it alike (as nwg); the RCCL engine refuses it
   (MPX_ERR_UNSUPPORTED).  The environment variable MPX_XFER_PULL=1 makes it
   the kernel and SDMA engines' default. */
#define MPX_XFER_PULL 2
/* mpx_xfer_opts.flags: kernel engine, bulk pushes read tx from HBM at every
   push instead of from the LDS copy each pushing workgroup takes once per
   call (the default whenever a workgroup's chunk fits in LDS, <= 60 KiB: tx
   is read-only while the loop runs, and the reference re-sends the same
   buffer every iteration, mpi_perf.c:72,80,136).  The link bytes are the
   same either way; this flag shows that the staged figure is not an LDS
   artefact (bench.py extras.unidir_4MiB_unstaged_GBps). */
#define MPX_XFER_NOSTAGE 4

/* opaque context */
typedef struct mpx_ctx mpx_ctx;

/* ---- library ------------------------------------------------------------ */
int mpx_version(void);
const char *mpx_strerror(int status);
/* detail of the last failing call on this thread ("" if none) */
const char *mpx_last_error(void);
/* number of visible GPUs (replaces MPI_Comm_size's role of sizing the job,
   mpi_perf.c:375, for the one-process/many-GPU launch) */
int mpx_device_count(int *count);
/* interconnect between two visible GPUs (no reference call does this; the
   nearest is the peer-host lookup of mpi_perf.c:171-198, which names the
   path a pair's bytes take): link_type is the HSA link type
   (MPX_LINK_XGMI, MPX_LINK_PCIE, ...), hops the hop count */
#define MPX_LINK_PCIE 2
#define MPX_LINK_XGMI 4
int mpx_link_info(int dev_a, int dev_b, int *link_type, int *hops);
/* PCI bus id of a visible GPU ("DDDD:BB:DD.F", hipDeviceGetPCIBusId) — how
   hosts name a GPU to tools that address devices by bus (the counters of
   include/mpxprof.h); len >= 16 */
int mpx_device_bus_id(int dev, char *buf, int len);

/* MPI_Init analogue (mpi_perf.c:372): a context able to address `nranks`
   ranks (<= MPX_MAX_RANKS) with the given engine. */
int mpx_init(int nranks, int engine, mpx_ctx **ctx);
/* MPI_Finalize analogue (mpi_perf.c:581) */
int mpx_finalize(mpx_ctx *ctx);
/* After the last mpx_finalize: destroy the process-lifetime rank streams
   (mpx_finalize returns them to a per-device pool) while the process is
   fully alive, instead of leaving them to the HIP runtime's exit teardown.
   MPX_ERR_STATE while a context is alive; MPX_ERR_TIMEOUT (streams left to
   the runtime) if the stream fence did not complete in 10 s.  May be called
   mid-process: a later context creates new rank streams. */
int mpx_shutdown(void);
/* Diagnostic: HIP events this library holds right now, across every context
   (each is owned by an RAII holder and destroyed on every return path:
   the tests' leak check around a failing mpx_copy, MPX_TEST=fail_copy). */
int mpx_live_events(int *count);

/* ---- buffers (allocate_tx_rx_buffers, mpi_perf.c:240-252) ---------------- */
/* posix_memalign(4096) analogue: device memory on `dev`, 4 KiB aligned.  The
   allocation is exportable to other processes (IPC) and peer-mappable.
   bytes == 0 yields a zeroed 16-byte block: the unidir ack still reads
   tx[0] at -b 0 (mpi_perf.c:142), which is 0 in the reference. */
int mpx_alloc(mpx_ctx *ctx, int dev, size_t bytes, void **ptr);
/* free() analogue (mpi_perf.c:576-577) */
int mpx_free(mpx_ctx *ctx, void *ptr);
/* memset analogue (mpi_perf.c:246,250); see enum mpx_fill */
int mpx_fill(mpx_ctx *ctx, int dev, void *ptr, size_t n, int pattern, uint64_t arg);
/* order-independent 64-bit checksum of n bytes (definition in DESIGN.md and
   oracle/mpx_oracle.c: oracle_checksum) */
int mpx_checksum(mpx_ctx *ctx, int dev, const void *ptr, size_t n, uint64_t *out);
/* device -> host copy, for tests */
int mpx_read(mpx_ctx *ctx, int dev, void *host_dst, const void *dev_src, size_t n);

/* ---- local device-to-device copy (BASELINE config 2) --------------------- */
/* `iters` back-to-back launches of the HBM copy kernel dst[0:n) = src[0:n) on
   `dev`; the 1-GPU degenerate case of the loop (tx -> rx, no peer). */
int mpx_copy(mpx_ctx *ctx, int dev, void *dst, const void *src, size_t n, int iters,
             mpx_timing *t);

/* ---- ranks: pairing/registration (get_peer_rank, mpi_perf.c:200-238) ----- */
/* Register a rank of this process: its GPU, tx/rx (from mpx_alloc on `dev`)
   and the largest message it will move.  Allocates the rank's mailbox (flag
   words + LL landing zone) and stream. */
int mpx_rank_attach(mpx_ctx *ctx, int rank, int dev, void *tx, void *rx, size_t len);
/* Serialise a local rank into MPX_RANK_DESC_BYTES bytes for another process
   (replaces the node_info Allgather, mpi_perf.c:223-224). */
int mpx_rank_export(mpx_ctx *ctx, int rank, void *desc);
/* Map a rank exported by another process (IPC) into this context. */
int mpx_rank_import(mpx_ctx *ctx, int rank, const void *desc);

/* ---- the hot loop -------------------------------------------------------- */
/* do_mpi_benchmark* replacement.  Runs `iters` iterations of `mode` between
   local rank `my_rank` (group `my_group`, 1 = sender side) and `peer_rank`,
   returning when this rank's side of the loop is complete, like the MPI loop.
   tx/rx must be the buffers attached for my_rank; buff_len <= attached len.
   *sec (may be NULL) receives the wall time of the loop.
   peer_rank == my_rank is accepted for MPX_MODE_NONBLOCKING only (MPI's
   self-send: Isend + Irecv to itself), a one-launch loopback of the path.
   Check mode (mpx_xfer_opts.check) checksums every received payload in every
   mode; in the non-blocking loop each in-flight receive lands in a slot of
   its own (the reference posts all of them into one rx, mpi_perf.c:100,104). */
int mpx_xfer(mpx_ctx *ctx, int mode, int my_group, int my_rank, int peer_rank, int iters,
             void *tx, void *rx, int buff_len, double *sec);
/* same, with options (checksum mode, timeouts) and full timing */
int mpx_xfer_ex(mpx_ctx *ctx, int mode, int my_group, int my_rank, int peer_rank, int iters,
                void *tx, void *rx, int buff_len, const mpx_xfer_opts *opts, mpx_timing *t);

/* Arm the next transfer of my_rank (kernel engine): its kernel is launched
   now and waits on the device; the next mpx_xfer_ex with the SAME arguments
   starts it with one store into host-mapped memory and times only that
   start and the loop.  MPI's persistent requests split a transfer the same
   way (MPI_Send_init / MPI_Recv_init before, MPI_Start inside the timed
   region); hosts arm before their barrier (mpi_perf.c:499), so the kernel
   launch (~14 us on MI355X, profiles/r04_phases_query.jsonl) is no longer
   part of every short loop's recorded time.  The armed call's device_s is
   the kernel's own clock from start to end.  mpx_xfer_arm returns once the
   kernel's whole grid runs and waits (at most 5 ms later), so the start does
   not also pay the rest of the dispatch.  A rank holds one armed call;
   mpx_xfer_ex with other arguments fails (MPX_ERR_STATE) and leaves it
   armed.  An armed kernel waits for its start at most max(the call's
   timeout, 60 s) — the host's barrier lies between arm and start — and
   then ends the call with MPX_ERR_TIMEOUT; a host whose start will not
   come (a failed barrier) cancels it with mpx_xfer_disarm at once.  A
   failed arm leaves the link as it was (no call number taken).  The SDMA
   and RCCL engines accept the call and do nothing. */
int mpx_xfer_arm(mpx_ctx *ctx, int mode, int my_group, int my_rank, int peer_rank, int iters,
                 void *tx, void *rx, int buff_len, const mpx_xfer_opts *opts);
/* Cancel an armed call that will not be started (no transfer happens);
   mpx_finalize does it for every armed rank. */
int mpx_xfer_disarm(mpx_ctx *ctx, int my_rank);

/* Build, outside any timed region, what a later mpx_xfer_ex with the same
   (mode, group, ranks, iters, buff_len, opts) would otherwise build on its
   first call: the SDMA engine's graph-captured loop chunks, or the RCCL
   engine's p2p channel to peer_rank (a one-byte exchange, once per pair; both
   ranks of the pair must call it, as they call the transfer).  The
   reference's timer brackets only the loop (mpi_perf.c:501-533), so hosts
   call this before their barrier (mpi_perf.c:499).  A no-op for the kernel
   engine. */
int mpx_xfer_prepare(mpx_ctx *ctx, int mode, int my_group, int my_rank, int peer_rank, int iters,
                     int buff_len, const mpx_xfer_opts *opts);

/* Where the last kernel-engine call of a local rank spent its wall time.
   The reference times the loop with MPI_Wtime around it (mpi_perf.c:501,
   532-533); a GPU loop adds a launch before the kernel runs and a
   completion after, which short loops (run-hbv3.sh: -i 10) pay per call.
   Kernel-side times come from the kernel's own clock (s_memrealtime), host-
   side ones from CLOCK_MONOTONIC; launch_to_start_s and done_to_return_s
   are 0 when the call waited with MPX_SYNC=event. */
typedef struct mpx_phases {
    double wall_s;            /* the call's mpx_timing.wall_s                   */
    double host_prep_s;       /* call entry -> launch (argument set-up)         */
    double launch_to_start_s; /* launch -> the kernel's first workgroup runs
                                 (completion word seen - launch - kernel_s)     */
    double posted_wait_s;     /* kernel start -> the peer's receives are posted
                                 (sides that push first; includes the peer's
                                 own late start)                                */
    double kernel_s;          /* first workgroup start -> last workgroup end    */
    double done_to_return_s;  /* completion word seen -> the kernel retired and
                                 the call returned                              */
    int32_t armed;            /* 1: the call was armed (mpx_xfer_arm): its
                                 launch happened before the call, and
                                 launch_to_start_s is go store -> running       */
    int32_t resident;         /* armed: 1 if every workgroup of the kernel was
                                 running and waiting for the start when
                                 mpx_xfer_arm returned (it waits up to 5 ms)   */
    double first_iter_s;      /* the loop's first iteration, from the kernel's
                                 start (or the peer's post, sides that push
                                 first) to its end (workgroup 0; ping-pong and
                                 unidir loops, else 0)                          */
    double tail_s;            /* workgroup 0 left the loop -> the last
                                 workgroup's end (accounting, resets)           */
} mpx_phases;
int mpx_last_phases(mpx_ctx *ctx, int rank, mpx_phases *out);

/* MPI_Barrier analogue (mpi_perf.c:499,557,579) for the threads of ONE
   process: blocks until `nthreads` callers have entered with the same ctx.
   Multi-process hosts use their own barrier. */
int mpx_barrier(mpx_ctx *ctx, int nthreads);

/* ---- RCCL engine setup ---------------------------------------------------- */
/* The RCCL this process actually runs (ncclGetVersion, e.g. 22707 = 2.27.7)
   and the file it was loaded from: libmpx links the image's ROCm RCCL, but a
   process that loaded another librccl.so.1 first (torch bundles its own)
   resolves libmpx's calls to that one.  len >= 64. */
int mpx_rccl_version(int *version, char *path, int len);
int mpx_rccl_get_unique_id(void *id /* MPX_RCCL_ID_BYTES */);
/* one rank per process (multi-process hosts) */
int mpx_rccl_init_rank(mpx_ctx *ctx, int rank, int nranks, const void *id);
/* every attached local rank of this process, in one call (threads host) */
int mpx_rccl_init_all(mpx_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif /* MPX_H */
