// mpx_runtime.hip — host side of libmpx: contexts, buffers, rank registration
// (same-process peer access or cross-process IPC), and the three transfer
// engines behind mpx_xfer_ex (kernel, SDMA, RCCL).
//
// Reference mapping (all /root/reference/mpi_perf.c):
//   mpx_init/finalize        MPI_Init / MPI_Finalize              :372, :581
//   mpx_alloc/fill/free      allocate_tx_rx_buffers, free         :240-252, :574-578
//   mpx_rank_attach/export/import   get_peer_rank's node_info Allgather :200-238
//   mpx_xfer(_ex)            do_mpi_benchmark{,_nonblocking,_unidir} :66-145
//   mpx_barrier              MPI_Barrier                          :499, :557, :579
#include "mpx_internal.h"

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <rccl/rccl.h>   // types only: the functions are bound at run time (rccl_api)

#include <atomic>
#include <condition_variable>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <type_traits>
#include <vector>

#include <dlfcn.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

using namespace mpx;

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIPCK(expr)                                                                                 \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess)                                                                       \
            return fail(MPX_ERR_HIP, "%s:%d %s: %s", __FILE__, __LINE__, #expr, hipGetErrorString(e_)); \
    } while (0)

// RCCL is bound at run time from ONE file, the image's /opt/rocm/lib/librccl.so.1
// (MPX_RCCL_LIB overrides), opened RTLD_LOCAL | RTLD_DEEPBIND: no symbol of it
// enters the process's global scope, and its own references resolve inside
// it.  A process that already holds another librccl.so.1 (torch's bundled
// 2.26.6 in bench.py) therefore cannot shadow it, and bench.py and mpx_perf
// run the same RCCL.  Linking -lrccl bound libmpx to
// whichever librccl.so.1 the process had loaded first.
struct RcclApi {
    void* h = nullptr;
    char path[512] = {0};
    char error[512] = {0};
    ncclResult_t (*GetVersion)(int*) = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
};

const RcclApi& rccl_api() {
    static const RcclApi* api = [] {
        RcclApi* a = new RcclApi;   // never destroyed, never dlclosed (exit-time ordering)
        const char* want = getenv("MPX_RCCL_LIB");
        if (!want || !*want) want = "/opt/rocm/lib/librccl.so.1";
        a->h = dlopen(want, RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND);
        if (!a->h) {
            snprintf(a->error, sizeof a->error, "cannot load %s: %s", want, dlerror());
            return a;
        }
        bool ok = true;
        auto bind = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(a->h, name));
            if (!fn && ok) {
                snprintf(a->error, sizeof a->error, "%s has no %s", want, name);
                ok = false;
            }
        };
        bind(a->GetVersion, "ncclGetVersion");
        bind(a->GetErrorString, "ncclGetErrorString");
        bind(a->GetUniqueId, "ncclGetUniqueId");
        bind(a->CommInitRank, "ncclCommInitRank");
        bind(a->CommInitAll, "ncclCommInitAll");
        bind(a->CommDestroy, "ncclCommDestroy");
        bind(a->GroupStart, "ncclGroupStart");
        bind(a->GroupEnd, "ncclGroupEnd");
        bind(a->Send, "ncclSend");
        bind(a->Recv, "ncclRecv");
        if (!ok) {
            a->h = nullptr;   // unusable: every RCCL entry point fails with the error
            return a;
        }
        Dl_info info{};
        snprintf(a->path, sizeof a->path, "%s",
                 dladdr(reinterpret_cast<void*>(a->GetVersion), &info) && info.dli_fname ? info.dli_fname : want);
        return a;
    }();
    return *api;
}

#define RCCL_LOADED()                                                      \
    do {                                                                   \
        if (!rccl_api().h) return fail(MPX_ERR_RCCL, "%s", rccl_api().error); \
    } while (0)

#define NCCLCK(expr)                                                                                \
    do {                                                                                            \
        ncclResult_t r_ = (expr);                                                                   \
        if (r_ != ncclSuccess)                                                                      \
            return fail(MPX_ERR_RCCL, "%s:%d %s: %s", __FILE__, __LINE__, #expr, rccl_api().GetErrorString(r_)); \
    } while (0)

#define TRY(expr)                     \
    do {                              \
        int s_ = (expr);              \
        if (s_ != MPX_OK) return s_;  \
    } while (0)

double now_s() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

u64 mix64_host(u64 z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// Restores the calling thread's current device on scope exit.
struct DeviceGuard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        err = hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// Owns one HIP event: destroyed when its holder goes (scope exit on any
// path, an early HIPCK return included, or the owning Rank's reset), so no
// error path can leak it.  live_events() counts the events alive in the
// process (mpx_live_events: the tests' leak check).
std::atomic<int>& live_events() {
    static std::atomic<int> n{0};
    return n;
}

class Event {
  public:
    Event() = default;
    Event(const Event&) = delete;
    Event& operator=(const Event&) = delete;
    Event(Event&& o) noexcept : e_(o.e_) { o.e_ = nullptr; }
    Event& operator=(Event&& o) noexcept {
        if (this != &o) {
            reset();
            e_ = o.e_;
            o.e_ = nullptr;
        }
        return *this;
    }
    ~Event() { reset(); }
    hipError_t create() {
        reset();
        const hipError_t e = hipEventCreate(&e_);
        if (e == hipSuccess) live_events().fetch_add(1);
        else e_ = nullptr;
        return e;
    }
    void reset() {
        if (!e_) return;
        (void)hipEventDestroy(e_);
        e_ = nullptr;
        live_events().fetch_sub(1);
    }
    operator hipEvent_t() const { return e_; }

  private:
    hipEvent_t e_ = nullptr;
};

enum MailboxKind { kMbUncached = 0, kMbFine = 1, kMbCoarse = 2 };

// (mode, group, peer rank, bytes, timeout ticks, iterations) of a captured
// SDMA chunk
typedef std::tuple<int, int, int, long long, u64, int> SdmaKey;

struct Rank {
    bool local = false;
    bool imported = false;
    bool broken = false;           // a transfer timed out: link state unknown
    int dev = -1;
    char bus_id[32] = {0};
    unsigned char* tx = nullptr;   // local tx, or the imported rank's tx mapped here (pull mode:
                                   // on the first pull call, ensure_peer_tx)
    hipIpcMemHandle_t tx_handle{}; // imported rank: its tx, until mapped
    bool tx_handle_valid = false;
    unsigned char* rx = nullptr;   // local rx, or the imported rank's rx mapped here
    size_t len = 0;
    Mailbox* mb = nullptr;         // usable from this process
    int mb_kind = kMbUncached;
    hipStream_t stream = nullptr;
    Event ev0, ev1;                // start / end of the rank's last call (RAII)
    u64 token = 0;                 // kernel-engine calls made: Status.done of the last one
    mpx_phases phases{};           // the last kernel-engine call (mpx_last_phases)
    struct KernelCall* armed = nullptr;   // the call mpx_xfer_arm launched, not started yet
    Status* status = nullptr;      // host-mapped (local ranks)
    u64* scratch = nullptr;        // kScratchWords device words (local ranks)
    u64* csum = nullptr;           // per-iteration checksums (device), csum_cap words,
    u64* cnt = nullptr;            //   then cnt: checked chunks per receive (csum + csum_cap)
    size_t csum_cap = 0;
    unsigned char* ring = nullptr; // non-blocking check mode's receive slots 1..S-1
    uint64_t ring_bytes = 0;       //   (allocated on first use, or at export: ensure_ring)
    std::vector<void*> retired;    // outgrown csum arrays (freed at finalize)
    u64 tx_seq[MPX_MAX_RANKS] = {};
    u64 rx_seq[MPX_MAX_RANKS] = {};
    u64 calls[MPX_MAX_RANKS] = {};   // transfer calls on the link to that rank (Mailbox.posted)
    ncclComm_t comm = nullptr;
    int comm_rank = -1;
    bool rccl_linked[MPX_MAX_RANKS] = {};          // RCCL p2p channel to that rank set up (mpx_xfer_prepare)
    std::map<SdmaKey, hipGraphExec_t> sdma_graphs;   // run_sdma's captured chunks
};

struct RankDesc {
    char magic[8];
    int32_t abi, rank, dev, mb_kind;
    int64_t pid;
    uint64_t len;
    char bus_id[32];
    char host[64];
    hipIpcMemHandle_t rx_handle;
    hipIpcMemHandle_t mb_handle;
    uint64_t ring_bytes;
    hipIpcMemHandle_t ring_handle;   // valid when ring_bytes > 0
    hipIpcMemHandle_t tx_handle;     // the rank's tx: pull mode loads from it
};
static_assert(sizeof(RankDesc) <= MPX_RANK_DESC_BYTES, "rank descriptor too large");

struct AllocRec {
    int dev;
    size_t bytes;
};

}  // namespace

struct mpx_ctx {
    int nranks = 0;
    int engine = 0;
    std::mutex mu;
    Rank r[MPX_MAX_RANKS];
    std::map<uintptr_t, AllocRec> allocs;
    std::map<int, hipStream_t> dev_stream;     // utility stream per device
    std::map<int, u64*> dev_tmp;               // 8-byte device scratch per device
    std::vector<void*> ipc_opened;             // to close on finalize
    std::mutex util_mu;                        // fill / checksum / copy share dev_stream + dev_tmp
    int import_dev = -1;
    // barrier (mpx_barrier)
    std::mutex bmu;
    std::condition_variable bcv;
    int bcount = 0;
    u64 bgen = 0;
};

namespace {

int util_stream(mpx_ctx* ctx, int dev, hipStream_t* s) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    auto it = ctx->dev_stream.find(dev);
    if (it != ctx->dev_stream.end()) {
        *s = it->second;
        return MPX_OK;
    }
    DeviceGuard g(dev);
    HIPCK(g.err);
    hipStream_t st;
    HIPCK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    u64* tmp;
    // [0] checksum sum; [16 ..) the one-launch copies' barrier: 17 words
    // 128 B apart (top counter, 8 group counters, 8 release words)
    HIPCK(hipMalloc(&tmp, 16 * 19 * sizeof(u64)));
    ctx->dev_stream[dev] = st;
    ctx->dev_tmp[dev] = tmp;
    *s = st;
    return MPX_OK;
}

int check_dev(int dev) {
    int n = 0;
    HIPCK(hipGetDeviceCount(&n));
    if (dev < 0 || dev >= n) return fail(MPX_ERR_INVALID, "device %d out of range [0,%d)", dev, n);
    return MPX_OK;
}

// Allocate the rank's mailbox; prefer uncached device memory (every access
// goes to memory, so polls see xGMI stores), then fine-grained, then coarse.
// The kind must also be IPC-exportable for multi-process use.
int alloc_mailbox(Rank& rk) {
    const unsigned flags[2] = {hipDeviceMallocUncached, hipDeviceMallocFinegrained};
    for (int k = 0; k <= 1; ++k) {
        void* p = nullptr;
        if (hipExtMallocWithFlags(&p, sizeof(Mailbox), flags[k]) != hipSuccess) {
            (void)hipGetLastError();
            continue;
        }
        hipIpcMemHandle_t h;
        const hipError_t e = hipIpcGetMemHandle(&h, p);
        if (getenv("MPX_DEBUG"))
            fprintf(stderr, "[mpx] mailbox kind %d alloc ok, ipc handle: %s\n", k, hipGetErrorString(e));
        (void)hipGetLastError();
        if (e != hipSuccess) {
            (void)hipFree(p);
            continue;
        }
        rk.mb = static_cast<Mailbox*>(p);
        rk.mb_kind = k;
        return MPX_OK;
    }
    void* p = nullptr;
    HIPCK(hipMalloc(&p, sizeof(Mailbox)));
    if (getenv("MPX_DEBUG")) fprintf(stderr, "[mpx] mailbox kind 2 (coarse hipMalloc)\n");
    rk.mb = static_cast<Mailbox*>(p);
    rk.mb_kind = kMbCoarse;
    return MPX_OK;
}

// Grows the checksum array without hipFree: hipFree waits for the whole
// device, i.e. for other ranks' spinning transfer kernels on the same GPU,
// which may be waiting for this rank.  Retired arrays are freed at finalize.
int ensure_csum(Rank& rk, int iters) {
    if ((size_t)iters <= rk.csum_cap) return MPX_OK;
    if (rk.csum) rk.retired.push_back(rk.csum);
    rk.csum = rk.cnt = nullptr;
    size_t cap = 1024;
    while (cap < (size_t)iters) cap *= 2;
    HIPCK(hipMalloc(&rk.csum, 2 * cap * sizeof(u64)));
    rk.cnt = rk.csum + cap;
    rk.csum_cap = cap;
    return MPX_OK;
}

// Bytes of a rank's check-mode receive ring: up to 255 further slots of the
// attached length, capped at MPX_CHECK_RING_BYTES (default 64 MiB; 0 = rx
// only, one slot per link).
uint64_t ring_bytes_for(size_t len) {
    static const uint64_t cap = [] {
        const char* v = getenv("MPX_CHECK_RING_BYTES");
        return v ? (uint64_t)strtoull(v, nullptr, 0) : (uint64_t)64 << 20;
    }();
    if (len == 0) return 0;
    const uint64_t want = (uint64_t)(kNbWindow - 1) * len;
    const uint64_t slots = (want < cap ? want : cap) / len;
    return slots * len;
}

// The check-mode receive ring of a local rank, allocated on its first use
// (a non-blocking call in check mode, by either rank of the link) or when the
// rank is exported: a peer process may push into it, and the descriptor
// carries its IPC handle.  A job that never checks non-blocking payloads
// never pays for it (up to 64 MiB per rank).  Caller holds ctx->mu.
int ensure_ring(Rank& rk) {
    if (!rk.local || rk.ring) return MPX_OK;
    const uint64_t bytes = ring_bytes_for(rk.len);
    if (!bytes) return MPX_OK;
    DeviceGuard g(rk.dev);
    HIPCK(g.err);
    void* p = nullptr;
    const hipError_t e = hipMalloc(&p, bytes);
    if (e == hipErrorOutOfMemory)
        return fail(MPX_ERR_NOMEM, "check ring of %llu B on device %d", (unsigned long long)bytes, rk.dev);
    HIPCK(e);
    rk.ring = static_cast<unsigned char*>(p);
    rk.ring_bytes = bytes;
    return MPX_OK;
}

// receive slots of the link between two ranks: the same on both sides
int link_slots(const Rank& a, const Rank& b, long long len) {
    const int sa = ring_slots(a.ring_bytes, len), sb = ring_slots(b.ring_bytes, len);
    return sa < sb ? sa : sb;
}

unsigned char* slot_ptr(const Rank& rk, int j, int iters, int slots, long long len) {
    const int s = ring_slot(j, iters, slots);
    return s == 0 ? rk.rx : rk.ring + (long long)(s - 1) * len;
}

// mpx_copy's form.  Default: all copies of a call in one launch where a
// launch per copy is dispatch-bound — k_copy_steps up to 512 KiB, k_copy_pipe
// above it to 16 MiB — and a k_copy launch per copy above.
// MPX_COPY (read per call; the tests drive every form and shape with it):
//   "launch"                      a k_copy launch per copy, any size
//   "steps[:cap:xcd:drain:upl:threads:one_xcd]"   k_copy_steps at any size
//   "pipe[:upl[:hier]]"           k_copy_pipe at any size it can hold
// Round 3's six copy knobs (MPX_COPY_VARIANT, _STEPS, _STEPS_MAX,
// _PIPE_MIN, _PIPE_MAX, _PIPE_UPL, _PIPE_HIER) are this one.
enum CopyForm { kCopyAuto = 0, kCopyLaunch, kCopySteps, kCopyPipe };
struct CopyChoice {
    int form = kCopyAuto;
    bool shaped = false;
    int shape[6] = {0, 0, 0, 0, 0, 0};   // k_copy_steps: cap, xcd, drain, upl, threads, one_xcd
    int upl = 0, hier = -1;              // k_copy_pipe
};
CopyChoice copy_choice() {
    CopyChoice c;
    const char* v = getenv("MPX_COPY");
    if (!v || !*v) return c;
    if (!strncmp(v, "launch", 6)) {
        c.form = kCopyLaunch;
    } else if (!strncmp(v, "steps", 5)) {
        c.form = kCopySteps;
        int* x = c.shape;
        const int k = sscanf(v + 5, ":%d:%d:%d:%d:%d:%d", &x[0], &x[1], &x[2], &x[3], &x[4], &x[5]);
        c.shaped = k >= 5;   // one_xcd may be omitted (0)
    } else if (!strncmp(v, "pipe", 4)) {
        c.form = kCopyPipe;
        (void)sscanf(v + 4, ":%d:%d", &c.upl, &c.hier);
    }
    return c;
}

// the receives the reference's non-blocking loop completes (Waitall) for
// `iters` iterations: slot 255 of each full window is never waited for
// (mpi_perf.c:95-124)
u64 nb_waited(int iters) {
    return (u64)iters - (u64)(iters / kNbWindow);
}

// Fault injection for the tests' negative controls, all in ONE variable:
//   MPX_TEST="skip_push=k,lag_wg=rank:wg:us,no_posted,no_pull_wait"
//   skip_push=k     the k-th push of every call (1-based) moves no payload
//                   bytes but is still signalled: a correct receiver's check
//                   must fail
//   lag_wg=r:w:us   in non-blocking check mode, workgroup w of rank r (w < 0
//                   counts from the last) stalls `us` before it checks the
//                   call's last receive (pull mode: before it loads the call's
//                   last payload), so that rank's call ends long after its peer's
//   no_posted       no receive-posted handshake (round 2's behaviour): the
//                   negative control of tests/test_gpu_ordering.py
//   no_pull_wait    pull mode: a sending side returns without waiting for the
//                   peer's loads of its tx (the buffer-reuse negative control)
//   fail_launch=r   rank r's kernel-engine calls fail before their kernel is
//                   enqueued (after prepare_call took their numbers): the
//                   rollback test of unprepare_call
//   fail_copy       mpx_copy fails after its events are created and the start
//                   one is recorded: the event-leak test (mpx_live_events)
// Whether the variable exists is read ONCE per process: a process that
// starts without it (bench.py, mpx_perf) never looks again, and none of the
// knobs can reach it.  The tests set it (empty) before their first call
// (tests/conftest.py) and change its value between calls.
struct TestKnobs {
    int skip_push = 0;
    int lag_rank = -1, lag_wg = 0;
    long long lag_us = 0;
    bool no_posted = false, no_pull_wait = false;
    int fail_launch = -1;
    bool fail_copy = false;
};
TestKnobs test_knobs() {
    static const bool gate = getenv("MPX_TEST") != nullptr;
    TestKnobs k;
    if (!gate) return k;
    const char* v = getenv("MPX_TEST");
    if (!v) return k;
    std::string all(v);
    size_t pos = 0;
    while (pos <= all.size()) {
        size_t end = all.find(',', pos);
        if (end == std::string::npos) end = all.size();
        const std::string item = all.substr(pos, end - pos);
        if (!item.compare(0, 10, "skip_push=")) k.skip_push = atoi(item.c_str() + 10);
        else if (!item.compare(0, 7, "lag_wg=")) {
            if (sscanf(item.c_str() + 7, "%d:%d:%lld", &k.lag_rank, &k.lag_wg, &k.lag_us) != 3) k.lag_rank = -1;
        } else if (item == "no_posted") k.no_posted = true;
        else if (item == "no_pull_wait") k.no_pull_wait = true;
        else if (!item.compare(0, 12, "fail_launch=")) k.fail_launch = atoi(item.c_str() + 12);
        else if (item == "fail_copy") k.fail_copy = true;
        pos = end + 1;
    }
    return k;
}

// A rank's stream must own its hardware queue.  The two halves of a pair
// are co-dependent persistent kernels; when both ranks live on one GPU and
// HIP multiplexes their streams onto one of its GPU_MAX_HW_QUEUES shared
// queues, the second kernel waits behind the first and both time out.  A
// stream created with a CU mask is never placed on a shared queue, so every
// rank stream is created with a mask that enables all CUs.
//
// Teardown rule (gfx950 / ROCm 7.2, isolated with tools/stream_teardown.hip,
// profiles/r02_stream_teardown.txt): a CU-masked stream owns a dedicated HSA
// queue that hipStreamDestroy frees.  hipFree of memory whose last use was a
// kernel on such a destroyed stream leaves the runtime waiting on that queue:
// the next queue creation, stream destruction or the process exit hangs
// ("a0 m0 k0.0 d0 f0" hangs at exit; "a0 m0 k0.0 f0 d0" is fine; freeing a
// buffer no kernel touched is fine either way).  The other stalls of rounds
// 2-4 — in a later context of the -m gpu suite when each finalize destroyed
// its streams (profiles/r02_stream_destroy_suite_hang.txt,
// r03_pytest_nopool.log) and at exit in processes mode
// (r04_procs_exit_stall.txt) — were one race, root-caused in round 5 from
// the stacks (profiles/r05_exit_stall_symbolized.txt): the destroy dropped
// its reference before HIP's completion handler of the stream's last
// command did, and the queue was then destroyed on the HSA events thread,
// which deadlocked on itself.  callback_fence now closes it
// (event_thread_barrier).  Rank streams stay process-lifetime objects all
// the same — a CU-masked queue costs a KFD queue creation — : mpx_finalize
// drains them (callback_fence), frees every allocation of the context, and
// returns them to a per-device pool that later contexts reuse; the host
// destroys them with mpx_shutdown once no context is alive (mpx_perf in
// both modes, bench.py).  A host that never calls it leaves them to the
// runtime's exit teardown (every allocation their kernels touched is freed by
// then: the safe order).
struct StreamPool {
    std::mutex mu;
    std::map<int, std::vector<hipStream_t>> idle;    // per device
    std::vector<std::pair<int, hipStream_t>> all;    // every stream ever created
    int live_contexts = 0;
};
StreamPool& pool() {
    static StreamPool* p = new StreamPool;   // never destroyed: no static-destructor ordering
    return *p;
}

void fence_cb(void* p) { static_cast<std::atomic<int>*>(p)->fetch_add(1, std::memory_order_release); }

// Hands off twice through the HSA async-events thread, the one thread that
// runs every hsa_amd_signal_async_handler callback, serially (hsa_ext_amd.h)
// — HIP's command-completion handlers, which run host functions, among them.
// When the second hand-off has run, every handler whose signal was satisfied
// before the first was registered has returned (one pass of the events loop
// fires every satisfied signal, in an arbitrary order: hence two).  One
// signal serves the process (value 0, condition EQ 0: satisfied at once;
// each registration returns false and is dropped).  Bounded at 10 s like the
// fence; false if the thread never came round.
bool on_events_thread(hsa_signal_value_t, void* arg) {
    static_cast<std::atomic<int>*>(arg)->store(1, std::memory_order_release);
    return false;
}

bool event_thread_barrier() {
    static hsa_signal_t sig = [] {
        hsa_signal_t s{0};
        if (hsa_signal_create(0, 0, nullptr, &s) != HSA_STATUS_SUCCESS) s.handle = 0;
        return s;
    }();
    if (!sig.handle) return false;
    const double t_end = now_s() + 10.0;
    for (int k = 0; k < 2; ++k) {
        // heap-held: leaked if the bound expires, so a late handler never
        // writes a dead stack frame
        std::atomic<int>* done = new std::atomic<int>(0);
        if (hsa_amd_signal_async_handler(sig, HSA_SIGNAL_CONDITION_EQ, 0, on_events_thread, done) != HSA_STATUS_SUCCESS) {
            delete done;
            return false;
        }
        while (!done->load(std::memory_order_acquire) && now_s() < t_end) usleep(20);
        if (!done->load(std::memory_order_acquire)) return false;
        delete done;
    }
    return true;
}

// Before streams are destroyed (and before the memory their commands used is
// freed).  Why (round 5, symbolized from profiles/r04_procs_exit_stall.txt;
// DESIGN.md §5 "Exit"): HIP's completion handler of a stream's command runs
// on the HSA async-events thread and holds a reference to the stream's
// virtual device until it returns — after the host function it ran.  When
// hipStreamDestroy drops the stream's own reference first, the handler's
// release is the last one: ~VirtualGPU runs ON the events thread, takes the
// device's virtual-GPU lock, and for a CU-masked stream (never pooled)
// hsa_queue_destroy's AqlQueue destructor waits, with no timeout, in the KFD
// event wait (AMDKFD_IOC_WAIT_EVENTS) for the queue's inactive-signal
// handler — which only that same thread can run.  The thread never returns;
// the next runtime call that needs the lock (a later stream teardown, or the
// fat-binary unregistration at exit) waits forever.  hipStreamSynchronize
// and the host functions below cannot close that window: they return when the
// command completed or the host function ran, both BEFORE the handler's
// release.  So: two host functions go onto each stream as its last commands
// (every callback before the second has returned once it runs), the streams
// are drained, and then event_thread_barrier() waits until the events
// thread has come round twice, i.e. has left the handler that ran the second
// host function and dropped its reference.  After that the caller's
// hipStreamDestroy drops the last reference on its own thread.
// Repro without libmpx: tools/exit_stall_repro cycle_fence|cycle_barrier
// (profiles/r05_stream_teardown_cycles.jsonl).  The waits are bounded (10 s)
// only so that a runtime that never runs the callbacks cannot hang the
// caller; the order, not the time, is what the fence relies on.  Returns
// false when a bound expired (the caller then must not destroy the streams).
bool callback_fence(const std::vector<std::pair<int, hipStream_t>>& ss) {
    // heap-held counters: leaked if the bound expires, so a late callback
    // never writes freed memory
    std::atomic<int>* cnt = new std::atomic<int>[ss.size() ? ss.size() : 1];
    std::vector<bool> armed(ss.size(), false);
    int prev = -1;
    (void)hipGetDevice(&prev);
    for (size_t i = 0; i < ss.size(); ++i) {
        cnt[i].store(0);
        (void)hipSetDevice(ss[i].first);
        armed[i] = hipLaunchHostFunc(ss[i].second, fence_cb, &cnt[i]) == hipSuccess &&
                   hipLaunchHostFunc(ss[i].second, fence_cb, &cnt[i]) == hipSuccess;
        (void)hipGetLastError();
    }
    const double t_end = now_s() + 10.0;
    bool done = true;
    for (size_t i = 0; i < ss.size(); ++i) {
        while (armed[i] && cnt[i].load(std::memory_order_acquire) < 2 && now_s() < t_end) usleep(50);
        done &= !armed[i] || cnt[i].load(std::memory_order_acquire) >= 2;
        (void)hipSetDevice(ss[i].first);
        (void)hipStreamSynchronize(ss[i].second);
    }
    if (prev >= 0) (void)hipSetDevice(prev);
    if (done) delete[] cnt;
    else if (getenv("MPX_DEBUG")) fprintf(stderr, "[mpx] callback fence: host functions did not run in 10 s\n");
    const bool handed_off = event_thread_barrier();
    if (!handed_off && getenv("MPX_DEBUG")) fprintf(stderr, "[mpx] callback fence: events-thread barrier did not complete\n");
    return done && handed_off;
}

// A rank stream goes back to the pool at finalize; later contexts reuse it
// (a CU-masked queue costs a KFD queue creation).  Pooled streams are
// destroyed only by mpx_shutdown, once no context is alive — which may be
// mid-process (mpx.h; tests/test_gpu_teardown.py): callback_fence and its
// event_thread_barrier order that destroy after every completion handler's
// release (round 5's root cause of the stalls rounds 2-4 saw, when each
// finalize destroyed its streams, profiles/r03_pytest_nopool.log).
void release_rank_stream(int dev, hipStream_t s) {
    std::lock_guard<std::mutex> lk(pool().mu);
    pool().idle[dev].push_back(s);
}

int create_rank_stream(int dev, hipStream_t* s) {
    {
        std::lock_guard<std::mutex> lk(pool().mu);
        auto& v = pool().idle[dev];
        if (!v.empty()) {
            *s = v.back();
            v.pop_back();
            return MPX_OK;
        }
    }
    hipDeviceProp_t prop;
    HIPCK(hipGetDeviceProperties(&prop, dev));
    const int words = (prop.multiProcessorCount + 31) / 32;
    std::vector<uint32_t> mask((size_t)words, 0xffffffffu);
    HIPCK(hipExtStreamCreateWithCUMask(s, (uint32_t)words, mask.data()));
    std::lock_guard<std::mutex> lk(pool().mu);
    pool().all.emplace_back(dev, *s);
    return MPX_OK;
}

bool same_device(const Rank& a, const Rank& b) {
    if (a.local && b.local) return a.dev == b.dev;
    return a.bus_id[0] && strcmp(a.bus_id, b.bus_id) == 0;
}

// Non-blocking mode: a push is published (kernel engine: drained + flag;
// SDMA engine: flag kernel) every nb_publish() pushes and at the last one —
// receivers wait only at window flushes and at the end.
// MPX_NB_PUBLISH=k (a divisor of 256; 1 = every push).
int nb_publish() {
    static const int k = [] {
        const char* v = getenv("MPX_NB_PUBLISH");
        const int x = v ? atoi(v) : 16;
        return (x >= 1 && x <= kNbWindow && (kNbWindow % x) == 0) ? x : 16;
    }();
    return k;
}

// Pull mode (MPX_XFER_PULL): the call's flag, else MPX_XFER_PULL=1 in the
// environment (every rank of a job inherits it, so both sides agree).  Kernel
// engine only.
bool pull_requested(const mpx_xfer_opts* o) {
    static const bool env_pull = [] {
        const char* v = getenv("MPX_XFER_PULL");
        return v && atoi(v) != 0;
    }();
    return (o && (o->flags & MPX_XFER_PULL)) || env_pull;
}

u64 timeout_ticks(const mpx_xfer_opts* o) {
    const u64 ms = (o && o->timeout_ms) ? o->timeout_ms : 10000;
    return ms * 100000ull;   // s_memrealtime runs at 100 MHz
}

// ---------------------------------------------------------------------------
// engine: kernel
// ---------------------------------------------------------------------------
int ensure_peer_tx_locked(mpx_ctx* ctx, Rank& peer, int peer_rank);
// Pull mode loads from the peer's tx: an imported rank's tx is mapped here on
// first use (under the context lock: both halves of a pair, or several local
// ranks, may get here at once), on the device imports are opened on.
int ensure_peer_tx(mpx_ctx* ctx, Rank& peer, int peer_rank) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    return ensure_peer_tx_locked(ctx, peer, peer_rank);
}
int ensure_peer_tx_locked(mpx_ctx* ctx, Rank& peer, int peer_rank) {
    if (peer.tx) return MPX_OK;
    if (!peer.imported || !peer.tx_handle_valid)
        return fail(MPX_ERR_STATE, "pull mode: rank %d's tx is not known here", peer_rank);
    DeviceGuard g(ctx->import_dev);
    HIPCK(g.err);
    void* p = nullptr;
    const hipError_t e = hipIpcOpenMemHandle(&p, peer.tx_handle, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(MPX_ERR_HIP, "pull mode: mapping rank %d's tx: %s", peer_rank, hipGetErrorString(e));
    }
    ctx->ipc_opened.push_back(p);
    peer.tx = static_cast<unsigned char*>(p);
    return MPX_OK;
}

// How a kernel-engine call waits for its kernel (MPX_SYNC, read once):
//   query (default) — spin on the host-mapped completion word the kernel's
//           last workgroup stores (Status.done), then on hipEventQuery of the
//           end event: the call returns once the kernel has retired (its
//           writes visible to every later command), with no interrupt on
//           the way;
//   event — hipEventSynchronize (round 3's form: the runtime's blocking
//           wait, woken by an interrupt once its short active spin expires).
// run-hbv3's 456131 B x 10 calls carried ~21 us of fixed
// cost each; mpx_last_phases reports where a call's time goes.
enum SyncMode { kSyncQuery = 0, kSyncEvent = 1 };
int sync_mode() {
    static const int m = [] {
        const char* v = getenv("MPX_SYNC");
        return (v && !strcmp(v, "event")) ? kSyncEvent : kSyncQuery;
    }();
    return m;
}

inline void cpu_relax() { __builtin_ia32_pause(); }

// One kernel-engine call: its arguments and launch shape, built by
// prepare_call; launched at once (run_kernel) or armed ahead of the host's
// barrier (mpx_xfer_arm) and started later (mpx_xfer_ex).
struct KernelCall {
    XferArgs a{};
    int grid = 0;
    bool ll = false;
    int my_rank = 0, peer_rank = 0, mode = 0, group = 0, iters = 0;
    long long len = 0;
    // what an armed call was armed with: mpx_xfer_ex must match it
    int check = 0, flags = 0, nwg_opt = 0;
    uint32_t timeout_ms = 0;
    uint64_t expect = 0, expect_ack = 0;
    double t_launch = 0;
    bool resident = false;   // armed: every workgroup was waiting when arm returned
    bool took_call = false;  // prepare_call took a call number on the link (iters > 0)
    bool launched = false;   // the kernel was enqueued: the call number is spent
};

// A call that failed before its kernel was enqueued gives back what
// prepare_call took (its token and the link's call number): the peer never
// sees that number, and a later call must post the one the peer waits for
// (ADVICE r04).  Once the kernel is enqueued the numbers stay taken — the
// kernel posts them — whatever fails after it.
void unprepare_call(Rank& me, const KernelCall& kc) {
    if (kc.launched) return;
    if (kc.took_call) --me.calls[kc.peer_rank];
    --me.token;
}

// Wait for the call's completion.  Unarmed: the end event ev1 (see
// sync_mode); *t_done = when the completion word was first seen (0 in event
// mode).  Armed: the completion word only — every byte the kernel leaves for
// the host or another stream (rx included: LL unpacks are write-through) is
// in memory before it is stored; the stream is polled every 50 us so that a
// kernel that ended without storing it (it cannot, but a fault could) ends
// the wait with an error instead of a hang.
// The call's end line (Status.fin) is complete and sealed for `token`: its
// word carries the token and the seal of the other seven words as read now
// (a line seen half-written does not match; the caller reads it again).
bool fin_sealed(const Rank& me, u64 token, Fin* out) {
    const volatile Fin* f = &me.status->fin;
    const u64 w = __atomic_load_n(&me.status->fin.word, __ATOMIC_ACQUIRE);
    if ((w & 0xffffffffull) != (token & 0xffffffffull)) return false;
    Fin v;
    v.recv_done = f->recv_done;
    v.recv_digest = f->recv_digest;
    v.t_entry = f->t_entry;
    v.t_posted = f->t_posted;
    v.t_first = f->t_first;
    v.t_loop = f->t_loop;
    v.t_exit = f->t_exit;
    v.word = w;
    if (fin_word(token, v.recv_done, v.recv_digest, v.t_entry, v.t_posted, v.t_first, v.t_loop, v.t_exit) != w)
        return false;
    if (out) *out = v;
    return true;
}

int wait_kernel(Rank& me, u64 token, bool armed, double* t_done) {
    *t_done = 0;
    if (!armed && sync_mode() == kSyncEvent) {
        HIPCK(hipEventSynchronize(me.ev1));
        return MPX_OK;
    }
    // Before the word arrives the end event / stream is polled only every
    // 50 us (a kernel that could not launch never stores it); after, back to
    // back (unarmed) or not at all (armed).
    double next_query = now_s() + 50e-6;
    for (;;) {
        if (*t_done == 0 && fin_sealed(me, token, nullptr)) {
            *t_done = now_s();
            if (armed) return MPX_OK;
        }
        if (*t_done != 0 || now_s() >= next_query) {
            const hipError_t q = armed ? hipStreamQuery(me.stream) : hipEventQuery(me.ev1);
            if (q == hipSuccess) {
                if (armed && !fin_sealed(me, token, nullptr))
                    return fail(MPX_ERR_HIP, "armed transfer kernel ended without its completion line");
                if (*t_done == 0) *t_done = now_s();
                return MPX_OK;
            }
            if (q != hipErrorNotReady) HIPCK(q);
            next_query = now_s() + 50e-6;
        }
        cpu_relax();
    }
}

int prepare_call(mpx_ctx* ctx, Rank& me, Rank& peer, int my_rank, int peer_rank, int mode, int group, int iters,
                 long long len, const mpx_xfer_opts* o, KernelCall* kc) {
    XferArgs& a = kc->a;
    a = XferArgs{};
    a.tx = me.tx;
    a.rx = me.rx;
    a.peer_rx = peer.rx;
    a.my_mb = me.mb;
    a.peer_mb = peer.mb;
    a.status = me.status;
    a.csum = me.csum;
    a.gbar = me.scratch;
    a.tx_seq0 = me.tx_seq[peer_rank];
    a.rx_seq0 = me.rx_seq[peer_rank];
    a.timeout_ticks = timeout_ticks(o);
    a.len = len;
    a.iters = iters;
    a.mode = mode;
    a.group = group;
    a.my_slot = my_rank;
    a.peer_slot = peer_rank;
    // push workgroups: the call's option, else MPX_PUSH_WG (every rank of a
    // job inherits the same environment, so both sides agree), else the
    // size rule bulk_nwg()
    static const int env_nwg = [] {
        const char* v = getenv("MPX_PUSH_WG");
        return v ? atoi(v) : 0;
    }();
    a.nwg = (o && o->nwg > 0) ? o->nwg : env_nwg > 0 ? env_nwg : bulk_nwg(len, same_device(me, peer));
    if (a.nwg > kMaxPushWG) return fail(MPX_ERR_INVALID, "nwg %d > %d", a.nwg, kMaxPushWG);
    // a width chosen for large pushes (the call's option, MPX_PUSH_WG) is not
    // applied to small ones: at least kMinPushChunk bytes per workgroup (the
    // size rule's chunks are 16-32 KiB, so it never narrows them).  Both
    // sides compute it from the same width and length, so they agree.
    a.nwg = (int)std::max<long long>(1, std::min<long long>(a.nwg, (len + kMinPushChunk - 1) / kMinPushChunk));
    a.check = (o && o->check) ? 1 : 0;
    static const bool env_stream = [] {
        const char* v = getenv("MPX_PUSH_STREAM");
        return v && atoi(v) != 0;
    }();
    a.stream = ((o && (o->flags & MPX_XFER_STREAM)) || env_stream) ? 1 : 0;
    a.nb_publish = nb_publish();
    a.ll_max = ll_max_bytes(same_device(me, peer));
    if (const char* v = getenv("MPX_LL_MAX")) a.ll_max = atoi(v) < kLLMaxBytes ? atoi(v) : kLLMaxBytes;
    a.cnt = me.cnt;
    const TestKnobs knobs = test_knobs();
    a.skip_push = knobs.skip_push;
    a.no_pull_wait = knobs.no_pull_wait ? 1 : 0;
    if (knobs.lag_rank == my_rank && knobs.lag_us > 0) {
        a.lag_wg = knobs.lag_wg;
        a.lag_ticks = (u64)knobs.lag_us * 100ull;   // s_memrealtime: 100 MHz
    }
    if (a.lag_wg < 0) a.lag_wg += a.nwg;   // -1: the last pushing workgroup

    const bool ll = mode != MPX_MODE_NONBLOCKING && len <= a.ll_max;
    const bool pushes_len = mode != MPX_MODE_UNIDIR || group == 1;
    const bool recvs_len = mode != MPX_MODE_UNIDIR || group == 0;
    // pull mode: B-byte payloads are loaded by their receiver (k_xfer_pull);
    // LL messages stay pushes.  A receiving side runs nwg workgroups (one
    // chunk each), unidir group 1 one (it only publishes and takes acks).
    a.pull = (!ll && pull_requested(o)) ? 1 : 0;
    {
        // fields another rank's thread may set at the same time (a lazily
        // mapped tx, a lazily allocated ring) are read under the context lock
        std::lock_guard<std::mutex> lk(ctx->mu);
        if (a.pull) TRY(ensure_peer_tx_locked(ctx, peer, peer_rank));
        a.peer_tx = peer.tx;
        a.ring = me.ring;
        a.peer_ring = peer.ring;
        a.slots = link_slots(me, peer, len);
    }
    if (!a.pull && a.check && mode == MPX_MODE_NONBLOCKING && len > 0 && a.slots > 1 && (!a.ring || !a.peer_ring))
        return fail(MPX_ERR_STATE, "rank %d/%d: check-mode receive ring missing", my_rank, peer_rank);
    kc->grid = a.pull ? (recvs_len ? a.nwg : 1) : (!ll && (pushes_len || (a.check && recvs_len))) ? a.nwg : 1;
    // bulk pushes read tx from LDS when one workgroup's chunk fits
    // (kStageMaxBytes); the call's MPX_XFER_NOSTAGE flag reads it from HBM
    if (!(o && (o->flags & MPX_XFER_NOSTAGE)) && !ll && !a.pull && pushes_len && len > 0) {
        static const long long lds_cap = [] {
            int dev = 0, per_block = 0;
            (void)hipGetDevice(&dev);
            if (hipDeviceGetAttribute(&per_block, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess)
                per_block = 0;
            return (long long)per_block - 1024;   // room for k_xfer's static LDS
        }();
        const long long chunk = (((len + a.nwg - 1) / a.nwg) + 15) & ~15ll;
        if (chunk <= kStageMaxBytes && chunk <= lds_cap) a.stage = (int)chunk;
    }
    a.done_token = ++me.token;
    // a call that moves nothing (iters = 0) posts nothing new: the count
    // stays equal on both sides even if only one side makes such a call
    kc->took_call = iters > 0;
    a.call = kc->took_call ? ++me.calls[peer_rank] : me.calls[peer_rank];
    if (knobs.no_posted) a.call = 0;   // every wait for posted >= 0 holds at once
    kc->ll = ll;
    kc->my_rank = my_rank;
    kc->peer_rank = peer_rank;
    kc->mode = mode;
    kc->group = group;
    kc->iters = iters;
    kc->len = len;
    kc->check = a.check;
    kc->flags = o ? o->flags : 0;
    kc->nwg_opt = o ? o->nwg : 0;
    kc->timeout_ms = o ? o->timeout_ms : 0;
    kc->expect = o ? o->expect_checksum : 0;
    kc->expect_ack = o ? o->expect_ack : 0;
    return MPX_OK;
}

// Enqueue the call's kernel on the rank's stream (scratch words [0..3] and
// [8] are zero: the previous call's last workgroup reset them — no memset
// ahead of the kernel).  Armed: go_token set, no events (the kernel's span
// comes from its own clock).
int launch_call(Rank& me, KernelCall& kc, bool armed) {
    XferArgs& a = kc.a;
    if (test_knobs().fail_launch == kc.my_rank)
        return fail(MPX_ERR_HIP, "rank %d: launch failed (MPX_TEST fail_launch)", kc.my_rank);
    if (a.check) {
        HIPCK(hipMemsetAsync(me.csum, 0, (size_t)kc.iters * sizeof(u64), me.stream));
        if (kc.mode == MPX_MODE_NONBLOCKING)
            HIPCK(hipMemsetAsync(me.cnt, 0, (size_t)kc.iters * sizeof(u64), me.stream));
    }
    me.status->err = 0;
    me.status->where = 0;
    memset(&me.status->fin, 0, sizeof(Fin));
    if (armed) {
        __atomic_store_n(&me.status->ready, 0ull, __ATOMIC_RELAXED);
        a.go_token = a.done_token;
        // the host's barrier sits between arm and start: bounded generously
        a.go_timeout_ticks = std::max<u64>(a.timeout_ticks, 60ull * 100000000ull);
        kc.t_launch = now_s();
        HIPCK(launch_xfer(a, kc.grid, me.stream));
        kc.launched = true;
        return MPX_OK;
    }
    kc.t_launch = now_s();
    HIPCK(hipEventRecord(me.ev0, me.stream));
    HIPCK(launch_xfer(a, kc.grid, me.stream));
    kc.launched = true;
    HIPCK(hipEventRecord(me.ev1, me.stream));
    return MPX_OK;
}

// Wait for the call, then its timing, phases and receive accounting.  t0 =
// the start of the timed call: the launch (unarmed) or the go store (armed).
int complete_call(Rank& me, KernelCall& kc, bool armed, double t_call, double t0, mpx_timing* t) {
    XferArgs& a = kc.a;
    double t_done = 0;
    TRY(wait_kernel(me, a.done_token, armed, &t_done));
    const double t_end = now_s();
    t->wall_s = t_end - t0;
    // the end line: sealed once wait_kernel returns (a retired kernel wrote
    // it whole); a line that does not match here is a kernel that never
    // wrote it (a fault) and fails the call
    Fin fin{};
    if (!fin_sealed(me, a.done_token, &fin))
        return fail(MPX_ERR_HIP, "rank %d: the transfer kernel left no completion line", kc.my_rank);
    const u64 te = fin.t_entry, tp = fin.t_posted, tx = fin.t_exit;
    const double kernel_s = (te && tx >= te) ? (double)(tx - te) * 1e-8 : 0;
    if (armed) {
        t->device_s = kernel_s;   // from go seen to the last workgroup's end (s_memrealtime)
    } else {
        float ms = 0;
        HIPCK(hipEventElapsedTime(&ms, me.ev0, me.ev1));
        t->device_s = ms * 1e-3;
    }
    t->launches = 1;
    t->nwg = kc.ll ? 1 : a.nwg;
    t->protocol = kc.ll ? kProtoLL : a.pull ? kProtoPull : kProtoBulk;
    t->recv_done = fin.recv_done;
    t->recv_digest = fin.recv_digest;
    // phases (mpx_last_phases): the kernel's own clock splits its span; the
    // host's clock brackets it (launch or go before, completion after)
    mpx_phases& ph = me.phases;
    ph = mpx_phases{};
    ph.wall_s = t->wall_s;
    ph.host_prep_s = armed ? 0 : t0 - t_call;
    ph.kernel_s = kernel_s;
    ph.posted_wait_s = (te && tp >= te) ? (double)(tp - te) * 1e-8 : 0;
    if (t_done > 0 && kernel_s > 0) {
        ph.launch_to_start_s = (t_done - t0) - kernel_s;
        ph.done_to_return_s = t_end - t_done;
    }
    ph.armed = armed ? 1 : 0;
    ph.resident = (armed && kc.resident) ? 1 : 0;
    // inside the kernel (k_xfer): the first iteration from the moment this
    // side could start it, and the end after the loop
    const u64 tf = fin.t_first, tl = fin.t_loop;
    const u64 t_go = tp >= te ? tp : te;
    ph.first_iter_s = (te && tf >= t_go) ? (double)(tf - t_go) * 1e-8 : 0;
    ph.tail_s = (tl && tx >= tl) ? (double)(tx - tl) * 1e-8 : 0;
    const unsigned err = __atomic_load_n(&me.status->err, __ATOMIC_ACQUIRE);
    if (err == 2) {
        me.broken = true;
        return fail(MPX_ERR_TIMEOUT, "rank %d: the armed transfer was not started within its deadline", kc.my_rank);
    }
    if (err) {
        me.broken = true;
        return fail(MPX_ERR_TIMEOUT, "rank %d <- rank %d: device wait timed out at iteration %u (mode %d, %lld B)",
                    kc.my_rank, kc.peer_rank, me.status->where - 1, kc.mode, kc.len);
    }
    me.tx_seq[kc.peer_rank] += (u64)kc.iters;
    me.rx_seq[kc.peer_rank] += (u64)kc.iters;
    return MPX_OK;
}

int run_kernel(mpx_ctx* ctx, Rank& me, Rank& peer, int my_rank, int peer_rank, int mode, int group, int iters,
               long long len, const mpx_xfer_opts* o, mpx_timing* t) {
    const double t_call = now_s();
    KernelCall kc;
    TRY(prepare_call(ctx, me, peer, my_rank, peer_rank, mode, group, iters, len, o, &kc));
    const int st = launch_call(me, kc, false);
    if (st != MPX_OK) {
        unprepare_call(me, kc);
        return st;
    }
    return complete_call(me, kc, false, t_call, kc.t_launch, t);
}

// An armed call ends without a transfer: go = token | kGoCancel, wait for
// the kernel, and the call number it took back (the peer never saw it: the
// kernel exits before posting its receives).
int disarm(Rank& me) {
    if (!me.armed) return MPX_OK;
    KernelCall& kc = *me.armed;
    __atomic_store_n(&me.status->go, kc.a.go_token | kGoCancel, __ATOMIC_RELEASE);
    double t_done = 0;
    const int st = wait_kernel(me, kc.a.done_token, true, &t_done);
    if (kc.took_call) --me.calls[kc.peer_rank];   // the same condition prepare_call took it on
    delete me.armed;
    me.armed = nullptr;
    return st;
}

// ---------------------------------------------------------------------------
// engine: SDMA — hipMemcpyAsync into the peer's rx, then a one-lane flag
// store; the receiver's stream waits on its mailbox flag with a one-lane poll.
// ---------------------------------------------------------------------------
// check mode for the stream engines: checksum the received bytes into
// csum[i], then poison them — stream-ordered before the next push.
int stream_check(Rank& me, long long n, int i, int iters, unsigned char* buf = nullptr) {
    if (n <= 0) return MPX_OK;
    if (!buf) buf = me.rx;
    HIPCK(launch_checksum(buf, (size_t)n, me.csum + i, me.stream));
    if (i + 1 < iters)   // the last payload stays in rx, as in the reference
        HIPCK(launch_fill(buf, (size_t)n, MPX_FILL_BYTE, (0x5a ^ i) & 0xff, me.stream));
    return MPX_OK;
}

// The SDMA engine's payload copy kind.  Between two GPUs it is
// hipMemcpyDeviceToDeviceNoCU: the runtime must use a copy engine (SDMA), the
// engine north_star (b) names.  Within one GPU (loopback pairs) it is the
// plain device-to-device kind, which the runtime runs as its blit kernel on
// the CUs (profiles/r02_sdma_engine_loopback_kernel_stats.csv): two ranks of
// one GPU share its SDMA queues, and a copy waiting at the head of a shared
// queue for its own rank's poll blocks the other rank's copy behind it — the
// loopback ping-pong timed out that way with NoCU copies
// (profiles/r02_sdma_kind_ab.jsonl), which also moved 40 GB/s against the
// blit kernel's 570 on one GPU.  A rank paired with itself has one stream and
// cannot deadlock so.  MPX_SDMA_KIND=nocu|blit forces one kind (A/B).
hipMemcpyKind sdma_kind(bool same_gpu) {
    static const int forced = [] {
        const char* v = getenv("MPX_SDMA_KIND");
        return !v ? 0 : !strcmp(v, "nocu") ? 1 : !strcmp(v, "blit") ? 2 : 0;
    }();
    const bool nocu = forced == 1 || (forced == 0 && !same_gpu);
    return nocu ? hipMemcpyDeviceToDeviceNoCU : hipMemcpyDeviceToDevice;
}

// non-blocking publish schedule shared by the kernel and SDMA engines: every
// nb_publish() pushes, at window slot 254 (the last receive a Waitall(255)
// waits for, so no flush waits for the slot-255 push the reference leaves
// pending) and at the last push
bool nb_publishes(int i, int iters) {
    return (i + 1) % nb_publish() == 0 || i % kNbWindow == kNbWindow - 2 || i + 1 == iters;
}

struct SdmaOps {
    Rank& me;
    Rank& peer;
    int my_slot, peer_slot;
    u64 tmo;
    const u64* txb = nullptr;   // graph capture: seqs relative to these device words
    const u64* rxb = nullptr;
    int launches = 0;
    int skip = 0;               // test knob: 1 + iteration whose copy is skipped
    bool pull = false;          // MPX_XFER_PULL: B-byte payloads copied by the receiver's stream
    // The flag store is a one-lane kernel ordered after the copy on this
    // stream (hipStreamWriteValue64 measured slower, 10.9 vs 8.6 us per
    // iteration, profiles/r01_sdma_signal_ab.jsonl).  Waits are bounded
    // one-lane kernels: a stream-level wait (hipStreamWaitValue64) cannot
    // time out.
    int push(long long n, u64 seq, bool publish = true, bool skip_copy = false) {
        if (n > 0 && !skip_copy) {
            HIPCK(hipMemcpyAsync(peer.rx, me.tx, (size_t)n, sdma_kind(&me != &peer && same_device(me, peer)),
                                 me.stream));
            ++launches;
        }
        if (!publish) return MPX_OK;
        HIPCK(launch_signal(&peer.mb->flag[my_slot][0], txb, seq, me.stream));
        ++launches;
        return MPX_OK;
    }
    int wait(u64 seq) {
        HIPCK(launch_wait(&me.mb->flag[peer_slot][0], rxb, seq, me.status, tmo, me.stream));
        ++launches;
        return MPX_OK;
    }
    // Pull mode (the kernel engine's k_xfer_pull in stream form).  A send
    // publishes "tx holds push seq" in the peer's ready word (tx is read-only
    // while the loop runs, and the reference re-sends the same buffer).
    int pull_send(u64 seq) {
        HIPCK(launch_signal(&peer.mb->ready[my_slot], txb, seq, me.stream));
        ++launches;
        return MPX_OK;
    }
    // A receive waits for the peer's ready word, copies the peer's tx into rx
    // on this rank's stream (a copy engine reading the peer's HBM across
    // GPUs), then, when `publish`, hands the peer's tx back (credit = seq,
    // for every push up to seq).
    int pull_recv(long long n, u64 seq, bool publish, bool skip_copy) {
        HIPCK(launch_wait(&me.mb->ready[peer_slot], rxb, seq, me.status, tmo, me.stream));
        ++launches;
        if (n > 0 && !skip_copy) {
            HIPCK(hipMemcpyAsync(me.rx, peer.tx, (size_t)n, sdma_kind(&me != &peer && same_device(me, peer)),
                                 me.stream));
            ++launches;
        }
        if (!publish) return MPX_OK;
        HIPCK(launch_signal(&peer.mb->credit[my_slot][0], rxb, seq, me.stream));
        ++launches;
        return MPX_OK;
    }
    // every one of this side's sends up to `seq` copied by the peer
    int wait_pulled(u64 seq) {
        HIPCK(launch_wait(&me.mb->credit[peer_slot][0], txb, seq, me.status, tmo, me.stream));
        ++launches;
        return MPX_OK;
    }
    // one iteration of the pulled loop (see step)
    int pull_step(int mode, int group, long long len, int i, int iters, u64 tx0, u64 rx0, bool check, int* inflight) {
        const bool sk = skip == i + 1;
        if (mode == MPX_MODE_PINGPONG) {
            if (group == 1) {
                TRY(pull_send(tx0 + i + 1));
                TRY(pull_recv(len, rx0 + i + 1, true, sk));
                if (check) TRY(stream_check(me, len, i, iters));
            } else {
                TRY(pull_recv(len, rx0 + i + 1, true, sk));
                if (check) TRY(stream_check(me, len, i, iters));
                TRY(pull_send(tx0 + i + 1));
            }
        } else if (mode == MPX_MODE_UNIDIR) {
            if (group == 1) {
                TRY(pull_send(tx0 + i + 1));
                TRY(wait(rx0 + i + 1));                      // the 1-byte ack, pushed
                if (check) TRY(stream_check(me, 1, i, iters));
            } else {
                TRY(pull_recv(len, rx0 + i + 1, true, sk));
                if (check) TRY(stream_check(me, len, i, iters));
                TRY(push(1, tx0 + i + 1, true, false));      // Send(tx, 1): always one byte, pushed
            }
        } else {
            // Isend + Irecv; the receive is complete on this stream once its
            // copy ran; credits go back on the push's publish schedule
            TRY(pull_send(tx0 + i + 1));
            TRY(pull_recv(len, rx0 + i + 1, nb_publishes(i, iters), sk));
            if (check) TRY(stream_check(me, len, i, iters));
            if (*inflight == kNbWindow - 1) {
                // Waitall(255): the peer's copies of sends 0..254; the
                // receives of slots 0..254 are done (stream order) — count them
                TRY(wait_pulled(tx0 + i));
                if (check) HIPCK(launch_account(me.status, me.csum, i - *inflight, *inflight, len, me.stream));
                *inflight = 0;
            } else {
                ++*inflight;
            }
        }
        return MPX_OK;
    }
    // one iteration i of the loop (mpi_perf.c:70-82, 95-124, 132-144), seqs
    // relative to tx0 / rx0; check mode checksums + poisons each received
    // payload where the reference's Recv returns (before the reply / ack);
    // *inflight is the non-blocking window fill
    int step(int mode, int group, long long len, int i, int iters, u64 tx0, u64 rx0, bool check, int* inflight) {
        if (pull) return pull_step(mode, group, len, i, iters, tx0, rx0, check, inflight);
        const bool sk = skip == i + 1;
        if (mode == MPX_MODE_PINGPONG) {
            if (group == 1) {
                TRY(push(len, tx0 + i + 1, true, sk));
                TRY(wait(rx0 + i + 1));
                if (check) TRY(stream_check(me, len, i, iters));
            } else {
                TRY(wait(rx0 + i + 1));
                if (check) TRY(stream_check(me, len, i, iters));
                TRY(push(len, tx0 + i + 1, true, sk));
            }
        } else if (mode == MPX_MODE_UNIDIR) {
            if (group == 1) {
                TRY(push(len, tx0 + i + 1, true, sk));
                TRY(wait(rx0 + i + 1));
                if (check) TRY(stream_check(me, 1, i, iters));
            } else {
                TRY(wait(rx0 + i + 1));
                if (check) TRY(stream_check(me, len, i, iters));
                TRY(push(1, tx0 + i + 1, true, sk));        // Send(tx, 1): always one byte
            }
        } else {
            TRY(push(len, tx0 + i + 1, nb_publishes(i, iters), sk));
            if (*inflight == kNbWindow - 1) {
                TRY(wait(rx0 + i));                          // Waitall(255): not slot 255's receive
                *inflight = 0;
            } else {
                ++*inflight;
            }
        }
        return MPX_OK;
    }

    // The non-blocking loop in check mode, stream-ordered (the kernel
    // engine's k_xfer_nbcheck in host-enqueued form): receive i lands in slot
    // ring_slot(i) of the receiver; before a push reuses a slot the sender's
    // stream waits for the receiver's credit; each receive is waited for,
    // checksummed and poisoned right after this side's push i (so the two
    // streams never wait on each other in a cycle), and the device counts
    // the reference's Waitall receives (k_account at each flush).
    // The call's receives were posted (Mailbox.posted) before it starts, so
    // the first `slots` pushes need no credit.
    int nb_checked(int iters, long long len, u64 tx0, u64 rx0, int slots) {
        u64* credit_out = &peer.mb->credit[my_slot][0];
        const u64* credit_in = &me.mb->credit[peer_slot][0];
        int inflight = 0;
        for (int i = 0; i < iters; ++i) {
            if (i >= slots) TRY(wait_abs(credit_in, tx0 + (u64)(i - slots + 1)));
            if (len > 0 && skip != i + 1) {
                HIPCK(hipMemcpyAsync(slot_ptr(peer, i, iters, slots, len), me.tx, (size_t)len,
                                     sdma_kind(same_device(me, peer) && &me != &peer), me.stream));
                ++launches;
            }
            TRY(signal_abs(&peer.mb->flag[my_slot][0], tx0 + i + 1));
            TRY(wait_abs(&me.mb->flag[peer_slot][0], rx0 + i + 1));
            TRY(stream_check(me, len, i, iters, slot_ptr(me, i, iters, slots, len)));
            TRY(signal_abs(credit_out, rx0 + i + 1));
            if (inflight == kNbWindow - 1) {          // Waitall(255): iterations i-255 .. i-1
                HIPCK(launch_account(me.status, me.csum, i - inflight, inflight, len, me.stream));
                inflight = 0;
            } else {
                ++inflight;
            }
        }
        if (inflight > 0) HIPCK(launch_account(me.status, me.csum, iters - inflight, inflight, len, me.stream));
        return MPX_OK;
    }
    int signal_abs(u64* flag, u64 v) {
        HIPCK(launch_signal(flag, nullptr, v, me.stream));
        ++launches;
        return MPX_OK;
    }
    int wait_abs(const u64* flag, u64 v) {
        HIPCK(launch_wait(flag, nullptr, v, me.status, tmo, me.stream));
        ++launches;
        return MPX_OK;
    }
};

// Graph-captured chunks of the SDMA loop (no check mode): the host enqueues
// ~3 operations per iteration at ~3.5 us each, so the plain loop is
// host-bound (9.4-10.4 us per ping-pong iteration on a loopback pair, 6.0 us
// replayed, profiles/r01_sdma_graph_ab.jsonl); capture and instantiation
// happen before the timed region.  Sequence numbers in a chunk are relative to
// me.scratch[2..3], which k_seqbase sets before the first replay and each
// chunk's last node advances by its iteration count.  Full chunks have
// kSdmaChunk = 256 iterations, which keeps the non-blocking window (a flush
// every 256 iterations) aligned with them; the remainder (< 256, no flush
// inside) is one more captured chunk of its own length.
constexpr int kSdmaChunk = kNbWindow;
constexpr int kSdmaGraphMin = 16;   // fewer iterations: plain enqueue

bool sdma_graphs_enabled() {
    static const bool on = [] {
        const char* v = getenv("MPX_SDMA_GRAPH");
        return !(v && atoi(v) == 0);
    }();
    return on;
}

int sdma_chunk_graph(Rank& me, Rank& peer, int my_rank, int peer_rank, int mode, int group, long long len,
                     u64 tmo, int count, hipGraphExec_t* out, bool pull = false) {
    const SdmaKey key{mode + (pull ? 8 : 0), group, peer_rank, len, tmo, count};
    auto it = me.sdma_graphs.find(key);
    if (it != me.sdma_graphs.end()) {
        *out = it->second;
        return MPX_OK;
    }
    SdmaOps cap{me, peer, my_rank, peer_rank, tmo, me.scratch + kScrSeqBase, me.scratch + kScrSeqBase + 1};
    cap.pull = pull;
    HIPCK(hipStreamBeginCapture(me.stream, hipStreamCaptureModeThreadLocal));
    int inflight = 0, st = MPX_OK;
    for (int j = 0; j < count && st == MPX_OK; ++j) st = cap.step(mode, group, len, j, count, 0, 0, false, &inflight);
    if (st == MPX_OK) st = launch_seqbase(me.scratch + kScrSeqBase, count, count, 1, me.stream) == hipSuccess
                               ? MPX_OK : fail(MPX_ERR_HIP, "k_seqbase launch in capture");
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(me.stream, &g);
    if (st != MPX_OK) {
        if (g) (void)hipGraphDestroy(g);
        return st;
    }
    HIPCK(e);
    hipGraphExec_t x = nullptr;
    const hipError_t ei = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    HIPCK(ei);
    me.sdma_graphs[key] = x;
    *out = x;
    return MPX_OK;
}


int run_sdma(Rank& me, Rank& peer, int my_rank, int peer_rank, int mode, int group, int iters, long long len,
             const mpx_xfer_opts* o, mpx_timing* t, bool pull) {
    SdmaOps op{me, peer, my_rank, peer_rank, timeout_ticks(o)};
    op.skip = test_knobs().skip_push;
    op.pull = pull;
    const int check = (o && o->check) ? 1 : 0;
    const int slots = link_slots(me, peer, len);
    if (!pull && check && mode == MPX_MODE_NONBLOCKING && len > 0 && slots > 1 && (!me.ring || !peer.ring))
        return fail(MPX_ERR_STATE, "rank %d/%d: check-mode receive ring missing", my_rank, peer_rank);
    if (check) HIPCK(hipMemsetAsync(me.csum, 0, (size_t)iters * sizeof(u64), me.stream));
    me.status->err = 0;
    me.status->where = 0;
    me.status->recv_done = 0;
    me.status->recv_digest = 0;
    const u64 txs0 = me.tx_seq[peer_rank], rxs0 = me.rx_seq[peer_rank];
    // graph-replayed chunks for the bulk of the loop (not in check mode,
    // whose per-iteration checksum slots would move with every chunk)
    const bool graphs = !check && sdma_graphs_enabled() && iters >= kSdmaGraphMin;
    const int chunks = graphs ? iters / kSdmaChunk : 0;
    const int rest = graphs && iters % kSdmaChunk >= kSdmaGraphMin ? iters % kSdmaChunk : 0;
    hipGraphExec_t full = nullptr, tail = nullptr;
    if (chunks > 0)
        TRY(sdma_chunk_graph(me, peer, my_rank, peer_rank, mode, group, len, op.tmo, kSdmaChunk, &full, pull));
    if (rest > 0) TRY(sdma_chunk_graph(me, peer, my_rank, peer_rank, mode, group, len, op.tmo, rest, &tail, pull));
    if (full || tail) HIPCK(launch_seqbase(me.scratch + kScrSeqBase, txs0, rxs0, 0, me.stream));
    const double t0 = now_s();
    HIPCK(hipEventRecord(me.ev0, me.stream));
    // matched-receive order (Mailbox.posted), stream-ordered: post this
    // call's receives, and a side that pushes first waits for the peer's
    // post before its first copy into the peer's rx
    if (iters > 0 && !test_knobs().no_posted) {
        const u64 call = ++me.calls[peer_rank];
        TRY(op.signal_abs(&peer.mb->posted[my_rank], call));
        if (mode == MPX_MODE_NONBLOCKING || group == 1) TRY(op.wait_abs(&me.mb->posted[peer_rank], call));
    }
    if (check && mode == MPX_MODE_NONBLOCKING && !pull) {
        TRY(op.nb_checked(iters, len, txs0, rxs0, slots));
    } else {
        for (int c = 0; c < chunks; ++c) HIPCK(hipGraphLaunch(full, me.stream));
        if (tail) HIPCK(hipGraphLaunch(tail, me.stream));
        int inflight = 0;
        const int replayed = chunks * kSdmaChunk + rest;
        for (int i = replayed; i < iters; ++i) TRY(op.step(mode, group, len, i, iters, txs0, rxs0, check, &inflight));
        if (pull) {
            // pulled: every receive is complete on this stream; the final
            // Waitall's receives are counted (check mode), and a side that
            // sent B-byte payloads waits for the peer's copies of its tx
            if (mode == MPX_MODE_NONBLOCKING && check && inflight > 0)
                HIPCK(launch_account(me.status, me.csum, iters - inflight, inflight, len, me.stream));
            if (iters > 0 && (mode != MPX_MODE_UNIDIR || group == 1)) TRY(op.wait_pulled(txs0 + iters));
        } else if (mode == MPX_MODE_NONBLOCKING && iters > 0 && (iters % kNbWindow) != 0) {
            TRY(op.wait(rxs0 + iters));
        }
        // every receive of ping-pong / unidir is complete here; the device
        // counts them and digests their checksums
        if (check && iters > 0 && mode != MPX_MODE_NONBLOCKING)
            HIPCK(launch_account(me.status, me.csum, 0, iters,
                                 (mode == MPX_MODE_UNIDIR && group == 1) ? 1 : len, me.stream));
    }
    HIPCK(hipEventRecord(me.ev1, me.stream));
    HIPCK(hipEventSynchronize(me.ev1));
    t->wall_s = now_s() - t0;
    float ms = 0;
    HIPCK(hipEventElapsedTime(&ms, me.ev0, me.ev1));
    t->device_s = ms * 1e-3;
    t->launches = op.launches + (chunks + (tail ? 1 : 0));   // graph replays count once each
    t->nwg = 0;
    t->protocol = pull ? kProtoSdmaPull : kProtoSdma;
    // check mode: counted on the device (k_account); otherwise the loop's
    // structure fixes the count
    t->recv_done = check ? __atomic_load_n(&me.status->recv_done, __ATOMIC_ACQUIRE)
                         : (mode == MPX_MODE_NONBLOCKING ? nb_waited(iters) : (u64)iters);
    t->recv_digest = __atomic_load_n(&me.status->recv_digest, __ATOMIC_ACQUIRE);
    if (__atomic_load_n(&me.status->err, __ATOMIC_ACQUIRE)) {
        me.broken = true;
        return fail(MPX_ERR_TIMEOUT, "rank %d <- rank %d: SDMA-engine wait timed out (flag %llu, awaited %llu; "
                    "sequence bases tx %llu rx %llu, mode %d, %lld B, %d iterations)", my_rank, peer_rank,
                    me.status->seen, me.status->want, txs0, rxs0, mode, len, iters);
    }
    me.tx_seq[peer_rank] += (u64)iters;
    me.rx_seq[peer_rank] += (u64)iters;
    return MPX_OK;
}

// ---------------------------------------------------------------------------
// engine: RCCL — ncclSend/ncclRecv on the rank's stream
// ---------------------------------------------------------------------------
int run_rccl(Rank& me, Rank& peer, int my_rank, int peer_rank, int mode, int group, int iters, long long len,
             const mpx_xfer_opts* o, mpx_timing* t) {
    (void)peer;
    (void)my_rank;
    if (!me.comm) return fail(MPX_ERR_STATE, "rank %d has no RCCL communicator (mpx_rccl_init_*)", my_rank);
    const int check = (o && o->check) ? 1 : 0;
    if (check) HIPCK(hipMemsetAsync(me.csum, 0, (size_t)iters * sizeof(u64), me.stream));
    me.status->recv_done = 0;
    me.status->recv_digest = 0;
    const size_t n = (size_t)len;
    const int skip = test_knobs().skip_push;
    const double t0 = now_s();
    HIPCK(hipEventRecord(me.ev0, me.stream));
    int launches = 0, inflight = 0;
    for (int i = 0; i < iters; ++i) {
        // test knob: the "lost" send carries rx (poison or stale bytes), not tx
        const void* src = skip == i + 1 ? (const void*)me.rx : (const void*)me.tx;
        if (mode == MPX_MODE_PINGPONG) {
            if (group == 1) {
                NCCLCK(rccl_api().Send(src, n, ncclChar, peer_rank, me.comm, me.stream));
                NCCLCK(rccl_api().Recv(me.rx, n, ncclChar, peer_rank, me.comm, me.stream));
                if (check) TRY(stream_check(me, len, i, iters));
            } else {
                NCCLCK(rccl_api().Recv(me.rx, n, ncclChar, peer_rank, me.comm, me.stream));
                if (check) TRY(stream_check(me, len, i, iters));
                NCCLCK(rccl_api().Send(src, n, ncclChar, peer_rank, me.comm, me.stream));
            }
            launches += 2;
        } else if (mode == MPX_MODE_UNIDIR) {
            if (group == 1) {
                NCCLCK(rccl_api().Send(src, n, ncclChar, peer_rank, me.comm, me.stream));
                NCCLCK(rccl_api().Recv(me.rx, 1, ncclChar, peer_rank, me.comm, me.stream));
                if (check) TRY(stream_check(me, 1, i, iters));
            } else {
                NCCLCK(rccl_api().Recv(me.rx, n, ncclChar, peer_rank, me.comm, me.stream));
                if (check) TRY(stream_check(me, len, i, iters));
                NCCLCK(rccl_api().Send(src, 1, ncclChar, peer_rank, me.comm, me.stream));
            }
            launches += 2;
        } else {
            // Isend + Irecv of one iteration: one fused group (full duplex).
            // Check mode: the receive lands in rx and is checksummed (and
            // poisoned) on this stream before the next group's receive can
            // land — RCCL writes only this rank's own buffer, so no slots or
            // credits are needed; the device counts the Waitall receives.
            NCCLCK(rccl_api().GroupStart());
            NCCLCK(rccl_api().Send(src, n, ncclChar, peer_rank, me.comm, me.stream));
            NCCLCK(rccl_api().Recv(me.rx, n, ncclChar, peer_rank, me.comm, me.stream));
            NCCLCK(rccl_api().GroupEnd());
            launches += 1;
            if (check) {
                TRY(stream_check(me, len, i, iters));
                if (inflight == kNbWindow - 1) {       // Waitall(255): iterations i-255 .. i-1
                    HIPCK(launch_account(me.status, me.csum, i - inflight, inflight, len, me.stream));
                    inflight = 0;
                } else {
                    ++inflight;
                }
            }
        }
    }
    if (check && mode == MPX_MODE_NONBLOCKING && inflight > 0)
        HIPCK(launch_account(me.status, me.csum, iters - inflight, inflight, len, me.stream));
    if (check && mode != MPX_MODE_NONBLOCKING && iters > 0)
        HIPCK(launch_account(me.status, me.csum, 0, iters, (mode == MPX_MODE_UNIDIR && group == 1) ? 1 : len,
                             me.stream));
    HIPCK(hipEventRecord(me.ev1, me.stream));
    HIPCK(hipEventSynchronize(me.ev1));
    t->wall_s = now_s() - t0;
    float ms = 0;
    HIPCK(hipEventElapsedTime(&ms, me.ev0, me.ev1));
    t->device_s = ms * 1e-3;
    t->launches = launches;
    t->nwg = 0;
    t->protocol = kProtoRccl;
    t->recv_done = check ? __atomic_load_n(&me.status->recv_done, __ATOMIC_ACQUIRE)
                         : (mode == MPX_MODE_NONBLOCKING ? nb_waited(iters) : (u64)iters);
    t->recv_digest = __atomic_load_n(&me.status->recv_digest, __ATOMIC_ACQUIRE);
    return MPX_OK;
}

}  // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

int mpx_version(void) { return MPX_ABI_VERSION; }

const char* mpx_strerror(int s) {
    switch (s) {
        case MPX_OK: return "success";
        case MPX_ERR_INVALID: return "invalid argument";
        case MPX_ERR_HIP: return "HIP runtime error";
        case MPX_ERR_NOMEM: return "out of device memory";
        case MPX_ERR_TIMEOUT: return "device-side wait timed out";
        case MPX_ERR_RCCL: return "RCCL error";
        case MPX_ERR_UNSUPPORTED: return "unsupported engine/mode";
        case MPX_ERR_STATE: return "call out of order";
        case MPX_ERR_CHECK: return "payload checksum mismatch";
        default: return "unknown mpx status";
    }
}

const char* mpx_last_error(void) { return g_last_error.c_str(); }

int mpx_device_count(int* count) {
    if (!count) return fail(MPX_ERR_INVALID, "count is NULL");
    HIPCK(hipGetDeviceCount(count));
    return MPX_OK;
}

int mpx_link_info(int dev_a, int dev_b, int* link_type, int* hops) {
    if (!link_type || !hops) return fail(MPX_ERR_INVALID, "NULL argument");
    TRY(check_dev(dev_a));
    TRY(check_dev(dev_b));
    if (dev_a == dev_b) return fail(MPX_ERR_INVALID, "device %d is both ends of the link", dev_a);
    uint32_t t = 0, h = 0;
    HIPCK(hipExtGetLinkTypeAndHopCount(dev_a, dev_b, &t, &h));
    *link_type = (int)t;
    *hops = (int)h;
    return MPX_OK;
}

int mpx_device_bus_id(int dev, char* buf, int len) {
    if (!buf || len < 16) return fail(MPX_ERR_INVALID, "bus id buffer too small");
    TRY(check_dev(dev));
    HIPCK(hipDeviceGetPCIBusId(buf, len, dev));
    return MPX_OK;
}

int mpx_init(int nranks, int engine, mpx_ctx** out) {
    if (!out) return fail(MPX_ERR_INVALID, "ctx out-pointer is NULL");
    *out = nullptr;
    if (nranks < 1 || nranks > MPX_MAX_RANKS) return fail(MPX_ERR_INVALID, "nranks %d not in [1,%d]", nranks, MPX_MAX_RANKS);
    if (engine == MPX_ENGINE_HOST)
        return fail(MPX_ERR_UNSUPPORTED, "engine HOST is not built: the CPU baseline is the compiled reference "
                    "(DESIGN.md section 8)");
    if (engine < MPX_ENGINE_KERNEL || engine > MPX_ENGINE_RCCL) return fail(MPX_ERR_INVALID, "engine %d", engine);
    int ndev = 0;
    HIPCK(hipGetDeviceCount(&ndev));
    if (ndev < 1) return fail(MPX_ERR_HIP, "no GPU visible");
    mpx_ctx* c = new mpx_ctx;
    c->nranks = nranks;
    c->engine = engine;
    {
        std::lock_guard<std::mutex> lk(pool().mu);
        ++pool().live_contexts;
    }
    *out = c;
    return MPX_OK;
}

#define DBG(...) \
    do { if (getenv("MPX_DEBUG")) { fprintf(stderr, "[mpx] " __VA_ARGS__); fflush(stderr); } } while (0)

int mpx_finalize(mpx_ctx* ctx) {
    if (!ctx) return fail(MPX_ERR_INVALID, "ctx is NULL");
    // Teardown order matters: every stream is drained and every allocation
    // freed, then the rank streams go back to the process pool (the teardown
    // rule above create_rank_stream).
    // Every stream of the context, rank and utility streams alike, is
    // drained through callback_fence: no completion callback of any of them
    // is still running when their memory is freed and the utility streams
    // are destroyed (a utility stream destroyed right after its drain stalled
    // mpx_perf at exit once the rank streams were fenced: r03_exit_hang).
    std::vector<std::pair<int, hipStream_t>> ss;
    for (int i = 0; i < MPX_MAX_RANKS; ++i) {
        Rank& rk = ctx->r[i];
        if (rk.armed) {                 // an armed call never started: cancel it
            DeviceGuard g(rk.dev);
            (void)disarm(rk);
        }
        if (rk.comm) (void)rccl_api().CommDestroy(rk.comm);
        rk.comm = nullptr;
        if (rk.local && rk.stream) ss.emplace_back(rk.dev, rk.stream);
    }
    for (auto& kv : ctx->dev_stream) ss.emplace_back(kv.first, kv.second);
    const bool fenced = callback_fence(ss);
    DBG("finalize: streams drained\n");
    for (int i = 0; i < MPX_MAX_RANKS; ++i) {
        for (auto& kv : ctx->r[i].sdma_graphs) (void)hipGraphExecDestroy(kv.second);
        ctx->r[i].sdma_graphs.clear();
    }
    for (void* p : ctx->ipc_opened) {
        const hipError_t e = hipIpcCloseMemHandle(p);
        if (e != hipSuccess) DBG("finalize: hipIpcCloseMemHandle(%p): %s\n", p, hipGetErrorString(e));
    }
    (void)hipGetLastError();
    for (int i = 0; i < MPX_MAX_RANKS; ++i) {
        Rank& rk = ctx->r[i];
        if (!rk.local) continue;
        DeviceGuard g(rk.dev);
        if (rk.mb) (void)hipFree(rk.mb);
        if (rk.ring) (void)hipFree(rk.ring);
        if (rk.scratch) (void)hipFree(rk.scratch);
        if (rk.csum) (void)hipFree(rk.csum);
        for (void* q : rk.retired) (void)hipFree(q);
        if (rk.status) (void)hipHostFree(rk.status);
    }
    for (auto& kv : ctx->allocs) {
        DeviceGuard g(kv.second.dev);
        (void)hipFree(reinterpret_cast<void*>(kv.first));
    }
    for (auto& kv : ctx->dev_tmp) {
        DeviceGuard g(kv.first);
        (void)hipFree(kv.second);
    }
    DBG("finalize: memory freed\n");
    for (int i = 0; i < MPX_MAX_RANKS; ++i) {
        Rank& rk = ctx->r[i];
        if (!rk.local) continue;
        DeviceGuard g(rk.dev);
        rk.ev0.reset();
        rk.ev1.reset();
        if (rk.stream) release_rank_stream(rk.dev, rk.stream);
    }
    if (fenced) {   // else left to the runtime: a destroy could be the events thread's last release
        for (auto& kv : ctx->dev_stream) {
            DeviceGuard g(kv.first);
            (void)hipStreamDestroy(kv.second);
        }
    }
    DBG("finalize: done\n");
    delete ctx;
    {
        std::lock_guard<std::mutex> lk(pool().mu);
        --pool().live_contexts;
    }
    return MPX_OK;
}

int mpx_alloc(mpx_ctx* ctx, int dev, size_t bytes, void** ptr) {
    if (!ctx || !ptr) return fail(MPX_ERR_INVALID, "NULL argument");
    *ptr = nullptr;
    TRY(check_dev(dev));
    DeviceGuard g(dev);
    HIPCK(g.err);
    void* p = nullptr;
    // hipMalloc returns >= 4 KiB-aligned blocks (posix_memalign(4096), mpi_perf.c:242-243)
    const hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
    if (e == hipErrorOutOfMemory) return fail(MPX_ERR_NOMEM, "hipMalloc(%zu) on device %d", bytes, dev);
    HIPCK(e);
    if (reinterpret_cast<uintptr_t>(p) & 4095) {
        (void)hipFree(p);
        return fail(MPX_ERR_HIP, "hipMalloc returned a pointer that is not 4 KiB aligned");
    }
    // -b 0: the unidir ack still sends tx[0] (mpi_perf.c:142) out of a 0-byte
    // posix_memalign block — glibc hands back a fresh zeroed chunk, so the
    // reference's ack byte is 0 (its PMPI digest, tests/test_integration.py);
    // the 16-byte pad is zeroed to match, on the utility stream (the null
    // stream would wait for other ranks' persistent kernels)
    if (!bytes) {
        hipStream_t us = nullptr;
        const int st = util_stream(ctx, dev, &us);
        hipError_t z = hipSuccess;
        if (st == MPX_OK) {
            std::lock_guard<std::mutex> ul(ctx->util_mu);
            z = hipMemsetAsync(p, 0, 16, us);
            if (z == hipSuccess) z = hipStreamSynchronize(us);
        }
        if (st != MPX_OK || z != hipSuccess) {
            (void)hipFree(p);
            if (st != MPX_OK) return st;
            HIPCK(z);
        }
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->allocs[reinterpret_cast<uintptr_t>(p)] = AllocRec{dev, bytes};
    *ptr = p;
    return MPX_OK;
}

int mpx_free(mpx_ctx* ctx, void* ptr) {
    if (!ctx) return fail(MPX_ERR_INVALID, "ctx is NULL");
    if (!ptr) return MPX_OK;
    AllocRec rec;
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        auto it = ctx->allocs.find(reinterpret_cast<uintptr_t>(ptr));
        if (it == ctx->allocs.end()) return fail(MPX_ERR_INVALID, "%p was not allocated by mpx_alloc", ptr);
        rec = it->second;
        ctx->allocs.erase(it);
    }
    DeviceGuard g(rec.dev);
    HIPCK(hipFree(ptr));
    return MPX_OK;
}

int mpx_fill(mpx_ctx* ctx, int dev, void* ptr, size_t n, int pattern, uint64_t arg) {
    if (!ctx || (!ptr && n)) return fail(MPX_ERR_INVALID, "NULL argument");
    if (pattern != MPX_FILL_BYTE && pattern != MPX_FILL_SPLITMIX) return fail(MPX_ERR_INVALID, "pattern %d", pattern);
    TRY(check_dev(dev));
    if (!n) return MPX_OK;
    hipStream_t s;
    TRY(util_stream(ctx, dev, &s));
    std::lock_guard<std::mutex> ul(ctx->util_mu);
    DeviceGuard g(dev);
    HIPCK(launch_fill(ptr, n, pattern, arg, s));
    HIPCK(hipStreamSynchronize(s));
    return MPX_OK;
}

int mpx_checksum(mpx_ctx* ctx, int dev, const void* ptr, size_t n, uint64_t* out) {
    if (!ctx || !out || (!ptr && n)) return fail(MPX_ERR_INVALID, "NULL argument");
    TRY(check_dev(dev));
    hipStream_t s;
    TRY(util_stream(ctx, dev, &s));
    std::lock_guard<std::mutex> ul(ctx->util_mu);
    u64* tmp = ctx->dev_tmp[dev];
    DeviceGuard g(dev);
    u64 raw = 0;
    if (n) {
        HIPCK(hipMemsetAsync(tmp, 0, sizeof(u64), s));
        HIPCK(launch_checksum(ptr, n, tmp, s));
        HIPCK(hipMemcpyAsync(&raw, tmp, sizeof(u64), hipMemcpyDeviceToHost, s));
        HIPCK(hipStreamSynchronize(s));
    }
    *out = raw ^ mix64_host((u64)n);
    return MPX_OK;
}

int mpx_read(mpx_ctx* ctx, int dev, void* host_dst, const void* dev_src, size_t n) {
    if (!ctx || ((!host_dst || !dev_src) && n)) return fail(MPX_ERR_INVALID, "NULL argument");
    TRY(check_dev(dev));
    if (!n) return MPX_OK;
    hipStream_t s;
    TRY(util_stream(ctx, dev, &s));
    std::lock_guard<std::mutex> ul(ctx->util_mu);
    DeviceGuard g(dev);
    HIPCK(hipMemcpyAsync(host_dst, dev_src, n, hipMemcpyDeviceToHost, s));
    HIPCK(hipStreamSynchronize(s));
    return MPX_OK;
}

int mpx_copy(mpx_ctx* ctx, int dev, void* dst, const void* src, size_t n, int iters, mpx_timing* t) {
    if (!ctx || !t || ((!dst || !src) && n) || iters < 0) return fail(MPX_ERR_INVALID, "bad argument");
    if ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15)
        return fail(MPX_ERR_INVALID, "copy buffers must be 16-byte aligned");
    TRY(check_dev(dev));
    memset(t, 0, sizeof *t);
    hipStream_t s;
    TRY(util_stream(ctx, dev, &s));
    std::lock_guard<std::mutex> ul(ctx->util_mu);
    DeviceGuard g(dev);
    Event e0, e1;   // destroyed on every return below
    HIPCK(e0.create());
    HIPCK(e1.create());
    int grid = 0;
    // All iterations in one launch where a launch per copy is dispatch-bound:
    // k_copy_pipe above 512 KiB to 16 MiB, k_copy_steps up to 512 KiB; one
    // k_copy launch per copy above (profiles/r03_copy_pipe_ab.jsonl, DESIGN.md
    // §5) — or the form MPX_COPY forces (copy_choice)
    const CopyChoice cc = copy_choice();
    const bool multi = n && iters > 1;
    bool pipe = multi && (cc.form == kCopyPipe ||
                          (cc.form == kCopyAuto && n > kCopyPipeDefaultMin && n <= kCopyPipeDefaultMax));
    const bool steps = multi && !pipe && (cc.form == kCopySteps || (cc.form == kCopyAuto && n <= kCopyPipeDefaultMin));
    bool one = pipe || steps;          // all copies in one launch
    u64* bar = ctx->dev_tmp[dev] + 16;
    float ms = 0;
    double t0 = 0;
    for (int attempt = 0; attempt < 2; ++attempt) {
        if (one) HIPCK(hipMemsetAsync(bar, 0, 17 * 16 * sizeof(u64), s));   // top + 8 group counters + 8 release words
        t0 = now_s();
        HIPCK(hipEventRecord(e0, s));
        if (test_knobs().fail_copy) return fail(MPX_ERR_HIP, "copy failed after its start event (MPX_TEST fail_copy)");
        if (one && pipe) {
            const hipError_t e = launch_copy_pipe(dst, src, n, iters, bar, s, &grid, cc.upl, cc.hier);
            if (e == hipErrorInvalidValue) {
                // too large for a resident pipe grid (a forced form or shape):
                // a launch per copy instead
                (void)hipGetLastError();
                one = pipe = false;
                continue;
            }
            HIPCK(e);
        } else if (one)
            HIPCK(launch_copy_steps(dst, src, n, iters, bar, s, &grid, cc.shaped ? cc.shape : nullptr));
        else
            for (int i = 0; i < iters && n; ++i) HIPCK(launch_copy(dst, src, n, s, &grid));
        HIPCK(hipEventRecord(e1, s));
        HIPCK(hipEventSynchronize(e1));
        HIPCK(hipEventElapsedTime(&ms, e0, e1));
        if (!one) break;
        // k_copy_steps / k_copy_pipe gave up on its grid barrier (bar[1]):
        // not every workgroup became resident — e.g. other ranks' persistent
        // transfer kernels hold CUs of this GPU.  Copy again, a launch per copy
        // (no residency needed); that is the call's result and its time.
        u64 stop = 0;
        HIPCK(hipMemcpyAsync(&stop, bar + 1, sizeof stop, hipMemcpyDeviceToHost, s));
        HIPCK(hipStreamSynchronize(s));
        if (!stop) break;
        DBG("copy of %zu B: step barrier gave up, a launch per copy instead\n", n);
        one = false;
    }
    t->wall_s = now_s() - t0;
    t->device_s = ms * 1e-3;
    t->bytes = (uint64_t)n * (uint64_t)iters;
    t->launches = !n ? 0 : one ? 1 : iters;
    t->nwg = grid;
    t->protocol = !one ? kProtoCopy : pipe ? kProtoCopyPipe : kProtoCopySteps;
    return MPX_OK;
}

namespace {

// A local rank's own resources: mailbox, stream, events, status, scratch,
// checksum arrays and the check-mode receive ring (rk.dev current).
int attach_resources(Rank& rk) {
    HIPCK(hipDeviceGetPCIBusId(rk.bus_id, sizeof rk.bus_id, rk.dev));
    TRY(alloc_mailbox(rk));
    TRY(create_rank_stream(rk.dev, &rk.stream));
    HIPCK(hipMemsetAsync(rk.mb, 0, sizeof(Mailbox), rk.stream));
    HIPCK(rk.ev0.create());
    HIPCK(rk.ev1.create());
    HIPCK(hipHostMalloc(reinterpret_cast<void**>(&rk.status), sizeof(Status), hipHostMallocCoherent | hipHostMallocMapped));
    memset(rk.status, 0, sizeof(Status));
    HIPCK(hipMalloc(&rk.scratch, kScratchWords * sizeof(u64)));
    HIPCK(hipMemsetAsync(rk.scratch, 0, kScratchWords * sizeof(u64), rk.stream));
    TRY(ensure_csum(rk, 1024));
    HIPCK(hipStreamSynchronize(rk.stream));
    return MPX_OK;
}

// Frees what attach_resources allocated, on a failed attach: the stream is
// drained first and goes back to the pool (the teardown rule above
// create_rank_stream: free, never destroy).
void release_rank(Rank& rk) {
    if (rk.stream) (void)hipStreamSynchronize(rk.stream);
    if (rk.mb) (void)hipFree(rk.mb);
    if (rk.ring) (void)hipFree(rk.ring);
    if (rk.scratch) (void)hipFree(rk.scratch);
    if (rk.csum) (void)hipFree(rk.csum);
    for (void* q : rk.retired) (void)hipFree(q);
    if (rk.status) (void)hipHostFree(rk.status);
    rk.ev0.reset();
    rk.ev1.reset();
    if (rk.stream) release_rank_stream(rk.dev, rk.stream);
    (void)hipGetLastError();
    rk = Rank{};
}

// Peer access between `dev` and the GPU of every local rank (ctx->mu held).
int enable_peer_access(mpx_ctx* ctx, int dev) {
    for (int i = 0; i < MPX_MAX_RANKS; ++i) {
        const Rank& o = ctx->r[i];
        if (!o.local || o.dev == dev) continue;
        int can = 0;
        HIPCK(hipDeviceCanAccessPeer(&can, dev, o.dev));
        if (!can) return fail(MPX_ERR_UNSUPPORTED, "GPU %d cannot access GPU %d (no xGMI/P2P path)", dev, o.dev);
        for (int dir = 0; dir < 2; ++dir) {
            const int a = dir ? o.dev : dev, b = dir ? dev : o.dev;
            DeviceGuard ga(a);
            const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIPCK(e);
            (void)hipGetLastError();
        }
    }
    return MPX_OK;
}

}  // namespace

int mpx_rank_attach(mpx_ctx* ctx, int rank, int dev, void* tx, void* rx, size_t len) {
    if (!ctx) return fail(MPX_ERR_INVALID, "ctx is NULL");
    if (rank < 0 || rank >= ctx->nranks) return fail(MPX_ERR_INVALID, "rank %d not in [0,%d)", rank, ctx->nranks);
    if (!tx || !rx) return fail(MPX_ERR_INVALID, "NULL tx/rx");
    if (len > 0x7fffffffull) return fail(MPX_ERR_INVALID, "len %zu exceeds the reference's int buff_len", len);
    TRY(check_dev(dev));
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        if (ctx->r[rank].local || ctx->r[rank].imported) return fail(MPX_ERR_STATE, "rank %d already registered", rank);
        auto it = ctx->allocs.find(reinterpret_cast<uintptr_t>(rx));
        if (it == ctx->allocs.end() || it->second.dev != dev || it->second.bytes < len)
            return fail(MPX_ERR_INVALID, "rx must be an mpx_alloc base on device %d of >= %zu bytes", dev, len);
        auto jt = ctx->allocs.find(reinterpret_cast<uintptr_t>(tx));
        if (jt == ctx->allocs.end() || jt->second.dev != dev || jt->second.bytes < len)
            return fail(MPX_ERR_INVALID, "tx must be an mpx_alloc base on device %d of >= %zu bytes", dev, len);
    }
    DeviceGuard g(dev);
    HIPCK(g.err);
    Rank rk;
    rk.local = true;
    rk.dev = dev;
    rk.tx = static_cast<unsigned char*>(tx);
    rk.rx = static_cast<unsigned char*>(rx);
    rk.len = len;
    int st = attach_resources(rk);
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (st == MPX_OK) st = enable_peer_access(ctx, dev);
    if (st != MPX_OK) {
        release_rank(rk);   // nothing of a failed attach stays allocated
        return st;
    }
    if (ctx->import_dev < 0) ctx->import_dev = dev;
    ctx->r[rank] = std::move(rk);
    return MPX_OK;
}

int mpx_rank_export(mpx_ctx* ctx, int rank, void* desc) {
    if (!ctx || !desc) return fail(MPX_ERR_INVALID, "NULL argument");
    if (rank < 0 || rank >= ctx->nranks || !ctx->r[rank].local) return fail(MPX_ERR_STATE, "rank %d is not a local rank", rank);
    const Rank& rk = ctx->r[rank];
    RankDesc d;
    memset(&d, 0, sizeof d);
    memcpy(d.magic, "MPXRANK2", 8);
    d.abi = MPX_ABI_VERSION;
    d.rank = rank;
    d.dev = rk.dev;
    d.mb_kind = rk.mb_kind;
    d.pid = (int64_t)getpid();
    d.len = rk.len;
    memcpy(d.bus_id, rk.bus_id, sizeof d.bus_id);
    gethostname(d.host, sizeof d.host - 1);
    DeviceGuard g(rk.dev);
    DBG("export rank %d: rx %p mb %p (kind %d) dev %d\n", rank, (void*)rk.rx, (void*)rk.mb, rk.mb_kind, rk.dev);
    HIPCK(hipIpcGetMemHandle(&d.rx_handle, rk.rx));
    HIPCK(hipIpcGetMemHandle(&d.tx_handle, rk.tx));
    HIPCK(hipIpcGetMemHandle(&d.mb_handle, rk.mb));
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        TRY(ensure_ring(ctx->r[rank]));
    }
    d.ring_bytes = rk.ring_bytes;
    if (rk.ring) HIPCK(hipIpcGetMemHandle(&d.ring_handle, rk.ring));
    memset(desc, 0, MPX_RANK_DESC_BYTES);
    memcpy(desc, &d, sizeof d);
    return MPX_OK;
}

int mpx_rank_import(mpx_ctx* ctx, int rank, const void* desc) {
    if (!ctx || !desc) return fail(MPX_ERR_INVALID, "NULL argument");
    if (rank < 0 || rank >= ctx->nranks) return fail(MPX_ERR_INVALID, "rank %d not in [0,%d)", rank, ctx->nranks);
    RankDesc d;
    memcpy(&d, desc, sizeof d);
    if (memcmp(d.magic, "MPXRANK2", 8) != 0 || d.abi != MPX_ABI_VERSION || d.rank != rank)
        return fail(MPX_ERR_INVALID, "descriptor is not an mpx rank %d descriptor", rank);
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (ctx->r[rank].local || ctx->r[rank].imported) return fail(MPX_ERR_STATE, "rank %d already registered", rank);
    if (ctx->import_dev < 0) return fail(MPX_ERR_STATE, "attach a local rank before importing remote ranks");
    if (d.pid == (int64_t)getpid()) return fail(MPX_ERR_INVALID, "rank %d belongs to this process: attach it instead", rank);
    DeviceGuard g(ctx->import_dev);
    HIPCK(g.err);
    Rank rk;
    rk.imported = true;
    rk.dev = d.dev;
    memcpy(rk.bus_id, d.bus_id, sizeof rk.bus_id);
    rk.len = d.len;
    rk.mb_kind = d.mb_kind;
    void* p = nullptr;
    HIPCK(hipIpcOpenMemHandle(&p, d.mb_handle, hipIpcMemLazyEnablePeerAccess));
    ctx->ipc_opened.push_back(p);
    rk.mb = static_cast<Mailbox*>(p);
    HIPCK(hipIpcOpenMemHandle(&p, d.rx_handle, hipIpcMemLazyEnablePeerAccess));
    ctx->ipc_opened.push_back(p);
    rk.rx = static_cast<unsigned char*>(p);
    // tx is mapped on the first pull-mode call that loads from it
    // (ensure_peer_tx): a job that never pulls maps nothing more than before
    rk.tx_handle = d.tx_handle;
    rk.tx_handle_valid = true;
    rk.ring_bytes = d.ring_bytes;
    if (d.ring_bytes) {
        HIPCK(hipIpcOpenMemHandle(&p, d.ring_handle, hipIpcMemLazyEnablePeerAccess));
        ctx->ipc_opened.push_back(p);
        rk.ring = static_cast<unsigned char*>(p);
    }
    ctx->r[rank] = std::move(rk);
    return MPX_OK;
}

namespace {
// Argument checks and per-rank set-up shared by mpx_xfer_ex and mpx_xfer_arm.
int check_call(mpx_ctx* ctx, int mode, int my_group, int my_rank, int peer_rank, int iters, void* tx, void* rx,
               int buff_len, const mpx_xfer_opts* opts) {
    if (mode < MPX_MODE_PINGPONG || mode > MPX_MODE_UNIDIR) return fail(MPX_ERR_INVALID, "mode %d", mode);
    if (my_group != 0 && my_group != 1) return fail(MPX_ERR_INVALID, "group %d", my_group);
    if (my_rank < 0 || my_rank >= ctx->nranks || peer_rank < 0 || peer_rank >= ctx->nranks)
        return fail(MPX_ERR_INVALID, "ranks %d/%d", my_rank, peer_rank);
    // a rank paired with itself: only the symmetric non-blocking loop (Isend +
    // Irecv to itself, MPI's self-send) — the one-kernel loopback every engine
    // can run on one GPU (RCCL refuses two ranks on one device), and the form
    // a profiler that serialises dispatches can trace
    if (my_rank == peer_rank && mode != MPX_MODE_NONBLOCKING)
        return fail(MPX_ERR_INVALID, "rank %d paired with itself: only the non-blocking loop", my_rank);
    if (iters < 0 || buff_len < 0) return fail(MPX_ERR_INVALID, "iters %d, buff_len %d", iters, buff_len);
    Rank& me = ctx->r[my_rank];
    Rank& peer = ctx->r[peer_rank];
    if (!me.local) return fail(MPX_ERR_STATE, "rank %d is not attached in this process", my_rank);
    // RCCL addresses the peer by its communicator rank and maps nothing itself;
    // the kernel and SDMA engines write into the peer's rx and mailbox
    const bool rccl = ctx->engine == MPX_ENGINE_RCCL;
    if (!rccl && !peer.local && !peer.imported)
        return fail(MPX_ERR_STATE, "peer rank %d is unknown (attach or import it)", peer_rank);
    if (me.broken) return fail(MPX_ERR_STATE, "rank %d: a previous transfer timed out", my_rank);
    if (tx != me.tx || rx != me.rx) return fail(MPX_ERR_INVALID, "tx/rx are not rank %d's attached buffers", my_rank);
    if ((size_t)buff_len > me.len || (!rccl && (size_t)buff_len > peer.len))
        return fail(MPX_ERR_INVALID, "buff_len %d exceeds an attached length (%zu, %zu)", buff_len, me.len, peer.len);
    const int check = opts && opts->check;
    if (opts && (opts->flags & MPX_XFER_PULL) && ctx->engine == MPX_ENGINE_RCCL)
        return fail(MPX_ERR_UNSUPPORTED, "pull mode (MPX_XFER_PULL): the kernel and SDMA engines only");
    const bool pull = ctx->engine != MPX_ENGINE_RCCL && pull_requested(opts);
    if (check) TRY(ensure_csum(me, iters));
    // (pull mode receives into rx in order: no receive ring)
    if (check && !pull && mode == MPX_MODE_NONBLOCKING && ctx->engine != MPX_ENGINE_RCCL) {
        // both ends of the link, under the lock: the other rank's thread may
        // be here too, and both must see both rings before sizing the slots
        std::lock_guard<std::mutex> lk(ctx->mu);
        TRY(ensure_ring(me));
        TRY(ensure_ring(peer));
    }
    return MPX_OK;
}

// After a completed loop: its algorithmic bytes and, in check mode, every
// received payload's checksum against the peer's tx — in the non-blocking
// loop too, where each receive has a slot of its own (k_xfer_nbcheck /
// SdmaOps::nb_checked).
int finish_xfer(Rank& me, int mode, int my_group, int my_rank, int iters, int buff_len, const mpx_xfer_opts* opts,
                mpx_timing* t) {
    t->bytes = (uint64_t)buff_len * (uint64_t)iters * (mode == MPX_MODE_UNIDIR ? 1u : 2u);
    if (!(opts && opts->check) || iters <= 0) return MPX_OK;
    DeviceGuard g(me.dev);
    HIPCK(g.err);
    std::vector<u64> raw((size_t)iters);
    // the rank's own stream: a null-stream copy would wait for every
    // blocking stream of the device, i.e. for other pairs' kernels
    HIPCK(hipMemcpyAsync(raw.data(), me.csum, (size_t)iters * sizeof(u64), hipMemcpyDeviceToHost, me.stream));
    HIPCK(hipStreamSynchronize(me.stream));
    const bool ack = mode == MPX_MODE_UNIDIR && my_group == 1;
    const u64 n = ack ? 1 : (u64)buff_len;   // the ack is always 1 byte (mpi_perf.c:137,142)
    const u64 want = ack ? opts->expect_ack : opts->expect_checksum;
    int bad = 0;
    for (int i = 0; i < iters; ++i)
        if ((raw[i] ^ mix64_host(n)) != want) ++bad;
    t->check_failures = bad;
    t->check_iters = (uint64_t)iters;
    if (bad) return fail(MPX_ERR_CHECK, "rank %d: %d of %d received payloads failed the checksum", my_rank, bad, iters);
    return MPX_OK;
}

// does an armed call match the arguments mpx_xfer_ex was given?
bool armed_matches(const KernelCall& kc, int mode, int group, int peer_rank, int iters, long long len,
                   const mpx_xfer_opts* o) {
    return kc.mode == mode && kc.group == group && kc.peer_rank == peer_rank && kc.iters == iters && kc.len == len &&
           kc.check == ((o && o->check) ? 1 : 0) && kc.flags == (o ? o->flags : 0) && kc.nwg_opt == (o ? o->nwg : 0) &&
           kc.timeout_ms == (o ? o->timeout_ms : 0) && kc.expect == (o ? o->expect_checksum : 0) &&
           kc.expect_ack == (o ? o->expect_ack : 0);
}
}  // namespace

constexpr double kArmReadyWaitS = 5e-3;

int mpx_xfer_arm(mpx_ctx* ctx, int mode, int my_group, int my_rank, int peer_rank, int iters, void* tx, void* rx,
                 int buff_len, const mpx_xfer_opts* opts) {
    if (!ctx) return fail(MPX_ERR_INVALID, "NULL argument");
    TRY(check_call(ctx, mode, my_group, my_rank, peer_rank, iters, tx, rx, buff_len, opts));
    if (ctx->engine != MPX_ENGINE_KERNEL) return MPX_OK;   // nothing to launch ahead (include/mpx.h)
    Rank& me = ctx->r[my_rank];
    Rank& peer = ctx->r[peer_rank];
    if (me.armed) return fail(MPX_ERR_STATE, "rank %d is already armed (start or disarm it first)", my_rank);
    DeviceGuard g(me.dev);
    HIPCK(g.err);
    KernelCall* kc = new KernelCall;
    int st = prepare_call(ctx, me, peer, my_rank, peer_rank, mode, my_group, iters, buff_len, opts, kc);
    if (st != MPX_OK) {
        delete kc;
        return st;
    }
    st = launch_call(me, *kc, true);
    if (st != MPX_OK) {
        // not launched: give the numbers back, and the inline call the
        // caller falls back to posts the one the peer waits for.  Launched
        // (a failure after the enqueue): the kernel waits for a go it will
        // never get — cancel it as disarm does, which also returns the call
        // number (the kernel exits before posting its receives)
        if (kc->launched) {
            me.armed = kc;
            (void)disarm(me);
        } else {
            unprepare_call(me, *kc);
            delete kc;
        }
        return st;
    }
    // Until the whole grid runs (Status.ready), a start would also wait for
    // the rest of the launch (the dispatch of every workgroup, ~5-10 us after
    // the launch call): wait for it here, ahead of the host's barrier.  The
    // wait is bounded (a grid that cannot all be resident yet, e.g. ranks
    // sharing a busy GPU, still starts correctly, only later).
    const double until = now_s() + kArmReadyWaitS;
    while (!(kc->resident = __atomic_load_n(&me.status->ready, __ATOMIC_ACQUIRE) == kc->a.go_token) && now_s() < until)
        cpu_relax();
    me.armed = kc;
    return MPX_OK;
}

int mpx_xfer_disarm(mpx_ctx* ctx, int my_rank) {
    if (!ctx) return fail(MPX_ERR_INVALID, "NULL argument");
    if (my_rank < 0 || my_rank >= ctx->nranks || !ctx->r[my_rank].local)
        return fail(MPX_ERR_STATE, "rank %d is not a local rank", my_rank);
    Rank& me = ctx->r[my_rank];
    DeviceGuard g(me.dev);
    HIPCK(g.err);
    return disarm(me);
}

int mpx_xfer_ex(mpx_ctx* ctx, int mode, int my_group, int my_rank, int peer_rank, int iters, void* tx, void* rx,
                int buff_len, const mpx_xfer_opts* opts, mpx_timing* t) {
    if (!ctx || !t) return fail(MPX_ERR_INVALID, "NULL argument");
    memset(t, 0, sizeof *t);
    const double t_call = now_s();
    TRY(check_call(ctx, mode, my_group, my_rank, peer_rank, iters, tx, rx, buff_len, opts));
    Rank& me = ctx->r[my_rank];
    Rank& peer = ctx->r[peer_rank];
    const bool pull = ctx->engine != MPX_ENGINE_RCCL && pull_requested(opts);
    if (me.armed) {
        // start the armed call: one host store; the kernel has been waiting for it
        KernelCall& kc = *me.armed;
        if (!armed_matches(kc, mode, my_group, peer_rank, iters, buff_len, opts))
            return fail(MPX_ERR_STATE, "rank %d is armed for another call (disarm it first)", my_rank);
        DeviceGuard g(me.dev);
        HIPCK(g.err);
        const double t0 = now_s();
        __atomic_store_n(&me.status->go, kc.a.go_token, __ATOMIC_RELEASE);
        const int st = complete_call(me, kc, true, t_call, t0, t);
        delete me.armed;
        me.armed = nullptr;
        if (st != MPX_OK) return st;
        return finish_xfer(me, mode, my_group, my_rank, iters, buff_len, opts, t);
    }
    DeviceGuard g(me.dev);
    HIPCK(g.err);
    int st;
    switch (ctx->engine) {
        case MPX_ENGINE_KERNEL:
            st = run_kernel(ctx, me, peer, my_rank, peer_rank, mode, my_group, iters, buff_len, opts, t);
            break;
        case MPX_ENGINE_SDMA:
            st = pull && buff_len > 0 && !peer.tx ? ensure_peer_tx(ctx, peer, peer_rank) : MPX_OK;
            if (st == MPX_OK) st = run_sdma(me, peer, my_rank, peer_rank, mode, my_group, iters, buff_len, opts, t, pull);
            break;
        default: st = run_rccl(me, peer, my_rank, peer_rank, mode, my_group, iters, buff_len, opts, t); break;
    }
    if (st != MPX_OK) return st;
    return finish_xfer(me, mode, my_group, my_rank, iters, buff_len, opts, t);
}

namespace {
// RCCL connects a pair lazily, on its first send/receive: transport setup and
// the exchange of buffer handles, milliseconds across GPUs.  The reference's
// MPI does the same, and its record of run 0 — the only run that pays it in a
// reference job — is dropped (mpi_perf.c:545).  In all-pairs rounds every
// round meets new peers, so runs 1..N-2 would carry that setup inside their
// recorded time; a one-byte exchange here, once per pair, before the barrier,
// takes it out.  Both ranks of the pair call it (as they call the transfer),
// on the rank's stream, into scratch words no transfer uses.
int rccl_link(Rank& me, int my_rank, int peer_rank) {
    if (!me.comm) return fail(MPX_ERR_STATE, "rank %d has no RCCL communicator (mpx_rccl_init_*)", my_rank);
    if (me.rccl_linked[peer_rank]) return MPX_OK;
    DeviceGuard g(me.dev);
    HIPCK(g.err);
    NCCLCK(rccl_api().GroupStart());
    NCCLCK(rccl_api().Send(me.scratch + kScrLink, 1, ncclChar, peer_rank, me.comm, me.stream));
    NCCLCK(rccl_api().Recv(me.scratch + kScrLink + 1, 1, ncclChar, peer_rank, me.comm, me.stream));
    NCCLCK(rccl_api().GroupEnd());
    HIPCK(hipStreamSynchronize(me.stream));
    me.rccl_linked[peer_rank] = true;
    return MPX_OK;
}
}  // namespace

int mpx_xfer_prepare(mpx_ctx* ctx, int mode, int my_group, int my_rank, int peer_rank, int iters, int buff_len,
                     const mpx_xfer_opts* opts) {
    if (!ctx) return fail(MPX_ERR_INVALID, "NULL argument");
    if (mode < MPX_MODE_PINGPONG || mode > MPX_MODE_UNIDIR) return fail(MPX_ERR_INVALID, "mode %d", mode);
    if (my_rank < 0 || my_rank >= ctx->nranks || peer_rank < 0 || peer_rank >= ctx->nranks)
        return fail(MPX_ERR_INVALID, "ranks %d/%d", my_rank, peer_rank);
    if (iters < 0 || buff_len < 0) return fail(MPX_ERR_INVALID, "iters %d, buff_len %d", iters, buff_len);
    Rank& me = ctx->r[my_rank];
    Rank& peer = ctx->r[peer_rank];
    if (!me.local) return fail(MPX_ERR_STATE, "rank %d is not attached in this process", my_rank);
    if (ctx->engine == MPX_ENGINE_RCCL) return rccl_link(me, my_rank, peer_rank);
    // the SDMA engine builds its graph-captured chunks per (mode, side, peer,
    // B): what run_sdma replays (not used in check mode)
    if (ctx->engine != MPX_ENGINE_SDMA || (opts && opts->check) || !sdma_graphs_enabled() || iters < kSdmaGraphMin)
        return MPX_OK;
    if (!peer.local && !peer.imported) return fail(MPX_ERR_STATE, "peer rank %d is unknown", peer_rank);
    const bool pull = pull_requested(opts);   // pulled chunks copy from the peer's tx: mapped first
    if (pull && buff_len > 0 && !peer.tx) TRY(ensure_peer_tx(ctx, peer, peer_rank));
    DeviceGuard g(me.dev);
    HIPCK(g.err);
    const u64 tmo = timeout_ticks(opts);
    hipGraphExec_t x = nullptr;
    if (iters / kSdmaChunk > 0)
        TRY(sdma_chunk_graph(me, peer, my_rank, peer_rank, mode, my_group, buff_len, tmo, kSdmaChunk, &x, pull));
    if (iters % kSdmaChunk >= kSdmaGraphMin)
        TRY(sdma_chunk_graph(me, peer, my_rank, peer_rank, mode, my_group, buff_len, tmo, iters % kSdmaChunk, &x,
                             pull));
    return MPX_OK;
}

int mpx_xfer(mpx_ctx* ctx, int mode, int my_group, int my_rank, int peer_rank, int iters, void* tx, void* rx,
             int buff_len, double* sec) {
    mpx_timing t;
    const int st = mpx_xfer_ex(ctx, mode, my_group, my_rank, peer_rank, iters, tx, rx, buff_len, nullptr, &t);
    if (sec) *sec = t.wall_s;
    return st;
}

int mpx_shutdown(void) {
    StreamPool& p = pool();
    std::lock_guard<std::mutex> lk(p.mu);
    if (p.live_contexts != 0) return fail(MPX_ERR_STATE, "%d contexts are still alive", p.live_contexts);
    if (p.all.empty()) return MPX_OK;
    if (!callback_fence(p.all))
        return fail(MPX_ERR_TIMEOUT, "stream fence did not complete in 10 s: streams left to the runtime");
    // every stream is destroyed and forgotten, whatever one destroy returns
    // (a stream left in the pool after a failed destroy could be handed out
    // again, or destroyed twice by a second shutdown); the first error is
    // the result, reported after the caller's device is restored
    int prev = -1;
    (void)hipGetDevice(&prev);
    hipError_t first = hipSuccess;
    int first_dev = -1;
    for (auto& ds : p.all) {
        (void)hipSetDevice(ds.first);
        const hipError_t e = hipStreamDestroy(ds.second);
        if (e != hipSuccess && first == hipSuccess) {
            first = e;
            first_dev = ds.first;
        }
    }
    (void)hipGetLastError();
    if (prev >= 0) (void)hipSetDevice(prev);
    p.all.clear();
    p.idle.clear();
    if (first != hipSuccess)
        return fail(MPX_ERR_HIP, "hipStreamDestroy on device %d: %s", first_dev, hipGetErrorString(first));
    return MPX_OK;
}

int mpx_live_events(int* count) {
    if (!count) return fail(MPX_ERR_INVALID, "NULL argument");
    *count = live_events().load();
    return MPX_OK;
}

int mpx_last_phases(mpx_ctx* ctx, int rank, mpx_phases* out) {
    if (!ctx || !out) return fail(MPX_ERR_INVALID, "NULL argument");
    if (rank < 0 || rank >= ctx->nranks || !ctx->r[rank].local) return fail(MPX_ERR_STATE, "rank %d is not a local rank", rank);
    *out = ctx->r[rank].phases;
    return MPX_OK;
}

int mpx_barrier(mpx_ctx* ctx, int nthreads) {
    if (!ctx || nthreads < 1) return fail(MPX_ERR_INVALID, "bad argument");
    std::unique_lock<std::mutex> lk(ctx->bmu);
    const u64 gen = ctx->bgen;
    if (++ctx->bcount == nthreads) {
        ctx->bcount = 0;
        ++ctx->bgen;
        ctx->bcv.notify_all();
    } else {
        ctx->bcv.wait(lk, [&] { return ctx->bgen != gen; });
    }
    return MPX_OK;
}

int mpx_rccl_version(int* version, char* path, int len) {
    if (!version || !path || len < 64) return fail(MPX_ERR_INVALID, "bad argument");
    RCCL_LOADED();
    NCCLCK(rccl_api().GetVersion(version));
    snprintf(path, (size_t)len, "%s", rccl_api().path);
    return MPX_OK;
}

int mpx_rccl_get_unique_id(void* id) {
    if (!id) return fail(MPX_ERR_INVALID, "id is NULL");
    static_assert(sizeof(ncclUniqueId) == MPX_RCCL_ID_BYTES, "RCCL unique id size");
    RCCL_LOADED();
    ncclUniqueId u;
    NCCLCK(rccl_api().GetUniqueId(&u));
    memcpy(id, &u, sizeof u);
    return MPX_OK;
}

int mpx_rccl_init_rank(mpx_ctx* ctx, int rank, int nranks, const void* id) {
    if (!ctx || !id) return fail(MPX_ERR_INVALID, "NULL argument");
    if (rank < 0 || rank >= ctx->nranks || !ctx->r[rank].local) return fail(MPX_ERR_STATE, "rank %d is not attached", rank);
    Rank& rk = ctx->r[rank];
    if (rk.comm) return fail(MPX_ERR_STATE, "rank %d already has a communicator", rank);
    RCCL_LOADED();
    DeviceGuard g(rk.dev);
    HIPCK(g.err);
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    NCCLCK(rccl_api().CommInitRank(&rk.comm, nranks, u, rank));
    rk.comm_rank = rank;
    return MPX_OK;
}

int mpx_rccl_init_all(mpx_ctx* ctx) {
    if (!ctx) return fail(MPX_ERR_INVALID, "ctx is NULL");
    std::vector<int> devs;
    for (int i = 0; i < ctx->nranks; ++i) {
        if (!ctx->r[i].local) return fail(MPX_ERR_STATE, "rank %d is not attached locally", i);
        if (ctx->r[i].comm) return fail(MPX_ERR_STATE, "rank %d already has a communicator", i);
        devs.push_back(ctx->r[i].dev);
    }
    RCCL_LOADED();
    std::vector<ncclComm_t> comms(devs.size());
    NCCLCK(rccl_api().CommInitAll(comms.data(), (int)devs.size(), devs.data()));
    for (int i = 0; i < ctx->nranks; ++i) {
        ctx->r[i].comm = comms[i];
        ctx->r[i].comm_rank = i;
    }
    return MPX_OK;
}

}  // extern "C"
