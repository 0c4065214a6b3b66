// exit_stall_repro.hip — minimal repro of the exit stall of DESIGN.md §5
// "Streams and queues" (profiles/r02_exit_stall.txt), without libmpx.
//
//   exit_stall_repro <teardown> [iters]
//
// Two host threads, each with a CU-masked stream (hipExtStreamCreateWithCUMask,
// as libmpx's rank streams), enqueue `iters` x {64 KiB device-to-device
// hipMemcpyAsync, a one-lane kernel} — the SDMA engine's per-iteration shape —
// and drain with hipStreamSynchronize.  Then the streams are torn down with
// <teardown>, and the process returns from main:
//   none     : hipStreamDestroy right after the drain
//   delay    : 50 ms after the drain (libmpx's workaround until round 3)
//   hostfunc : a host function enqueued as each stream's last command, then
//              a second one; hipStreamDestroy once the second has run (so
//              the first has returned) and the stream drained again
//   keep     : no destroy (the runtime's exit teardown destroys them)
// Prints "exit" before returning from main; a run that prints it and never
// ends is the stall (the caller's timeout kills it).
//
//   exit_stall_repro cycle_fence|cycle_barrier [cycles]
//
// The same race inside one process (round 5, DESIGN.md §5 "Exit"): each
// cycle creates a CU-masked stream, runs a one-lane kernel, enqueues two host
// functions, spins until the second has run, and destroys the stream at once
// (cycle_fence: libmpx's callback_fence up to round 4), or first waits for
// two ordered hand-offs through the HSA async-events thread (cycle_barrier:
// event_thread_barrier in mpx_runtime.hip).  A watchdog prints
// "STALL at cycle k" and ends the process with status 3 when a cycle has not
// finished in 5 s; "cycles done" otherwise.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <atomic>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <thread>
#include <unistd.h>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            printf("FAIL %s: %s\n", #x, hipGetErrorString(e_));                 \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

__global__ void k_tick(unsigned long long* p) {
    if (threadIdx.x == 0) p[0] += 1;
}

static std::atomic<int> g_ran[2];
static void mark(void* arg) { g_ran[(int)(size_t)arg & 1].fetch_add(1); }

static bool on_loop(hsa_signal_value_t, void* arg) {
    static_cast<std::atomic<int>*>(arg)->store(1);
    return false;
}

// Two hand-offs in sequence through the async-events thread, which runs
// every handler (HIP's command-completion handlers included) serially: when
// the second has run, every handler whose signal was satisfied before the
// first was registered has returned.
static void event_thread_barrier() {
    static hsa_signal_t sig = [] {
        hsa_signal_t s;
        if (hsa_signal_create(0, 0, nullptr, &s) != HSA_STATUS_SUCCESS) { printf("FAIL hsa_signal_create\n"); exit(1); }
        return s;
    }();
    for (int k = 0; k < 2; ++k) {
        std::atomic<int> done{0};
        if (hsa_amd_signal_async_handler(sig, HSA_SIGNAL_CONDITION_EQ, 0, on_loop, &done) != HSA_STATUS_SUCCESS) {
            printf("FAIL hsa_amd_signal_async_handler\n");
            exit(1);
        }
        while (!done.load()) usleep(20);
    }
}

static std::atomic<long> g_cycle{-1};

static int cycles(bool barrier, int n) {
    CK(hipSetDevice(0));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int words = (prop.multiProcessorCount + 31) / 32;
    std::vector<uint32_t> mask((size_t)words, 0xffffffffu);
    unsigned long long* c;
    CK(hipMalloc(&c, 64));
    std::thread([n] {
        long last = -2;
        double still = 0;
        while (true) {
            usleep(100000);
            const long k = g_cycle.load();
            if (k >= n) return;
            if (k == last) {
                if ((still += 0.1) >= 5.0) {
                    printf("STALL at cycle %ld of %d\n", k, n);
                    fflush(stdout);
                    _exit(3);
                }
            } else {
                last = k;
                still = 0;
            }
        }
    }).detach();
    for (int k = 0; k < n; ++k) {
        g_cycle.store(k);
        hipStream_t st;
        CK(hipExtStreamCreateWithCUMask(&st, (uint32_t)words, mask.data()));
        hipLaunchKernelGGL(k_tick, dim3(1), dim3(64), 0, st, c);
        std::atomic<int> ran{0};
        auto bump = [](void* p) { static_cast<std::atomic<int>*>(p)->fetch_add(1); };
        CK(hipLaunchHostFunc(st, bump, &ran));
        CK(hipLaunchHostFunc(st, bump, &ran));
        while (ran.load() < 2) {
        }
        CK(hipStreamSynchronize(st));
        if (barrier) event_thread_barrier();
        CK(hipStreamDestroy(st));
    }
    g_cycle.store(n);
    CK(hipFree(c));
    printf("cycles done: %d\n", n);
    fflush(stdout);
    return 0;
}

int main(int argc, char** argv) {
    const char* how = argc > 1 ? argv[1] : "none";
    if (!strncmp(how, "cycle_", 6)) return cycles(!strcmp(how, "cycle_barrier"), argc > 2 ? atoi(argv[2]) : 2000);
    const int iters = argc > 2 ? atoi(argv[2]) : 300;
    CK(hipSetDevice(0));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int words = (prop.multiProcessorCount + 31) / 32;
    std::vector<uint32_t> mask((size_t)words, 0xffffffffu);
    hipStream_t st[2];
    unsigned char *a[2], *b[2];
    unsigned long long* c[2];
    for (int i = 0; i < 2; ++i) {
        CK(hipExtStreamCreateWithCUMask(&st[i], (uint32_t)words, mask.data()));
        CK(hipMalloc(&a[i], 65536));
        CK(hipMalloc(&b[i], 65536));
        CK(hipMalloc(&c[i], 64));
    }
    std::thread th[2];
    for (int i = 0; i < 2; ++i)
        th[i] = std::thread([&, i] {
            CK(hipSetDevice(0));
            for (int k = 0; k < iters; ++k) {
                CK(hipMemcpyAsync(b[i], a[i], 65536, hipMemcpyDeviceToDevice, st[i]));
                hipLaunchKernelGGL(k_tick, dim3(1), dim3(64), 0, st[i], c[i]);
            }
            CK(hipStreamSynchronize(st[i]));
        });
    for (auto& t : th) t.join();
    for (int i = 0; i < 2; ++i) {   // free, then destroy: the safe order
        CK(hipFree(a[i]));
        CK(hipFree(b[i]));
        CK(hipFree(c[i]));
    }
    if (!strcmp(how, "delay")) usleep(50000);
    if (!strcmp(how, "hostfunc")) {
        for (int i = 0; i < 2; ++i) {
            CK(hipLaunchHostFunc(st[i], mark, (void*)(size_t)i));
            CK(hipLaunchHostFunc(st[i], mark, (void*)(size_t)i));
        }
        for (int i = 0; i < 2; ++i) {
            while (g_ran[i].load() < 2) usleep(100);
            CK(hipStreamSynchronize(st[i]));
        }
    }
    if (strcmp(how, "keep"))
        for (int i = 0; i < 2; ++i) CK(hipStreamDestroy(st[i]));
    printf("exit\n");
    fflush(stdout);
    return 0;
}
