// go_latency_probe.hip — how fast does a host store reach a polling kernel?
// A persistent one-lane kernel loops: poll the "go" word for value k, then
// store k into a host-mapped "ack" word; the host stores k, spins until the
// ack shows k, and records the round trip (median over many).  Two places
// for the go word:
//   host : hipHostMalloc'd (coherent, mapped) — what Status.go is today
//   dev  : (argument "dev" only) device memory written by the CPU through its
//          pointer (hipExtMallocWithFlags fine-grained).  On the round-4 box
//          the pointer is a device-only address (no host pointer) and the
//          host's first store never completed: the probe hung until its
//          time limit (profiles/r04_go_latency_probe.jsonl) — so the go word
//          stays in host memory.
// Prints one JSON line per place.
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/go_latency_probe tools/go_latency_probe.hip
//   tools/go_latency_probe [rounds] [dev]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

typedef unsigned long long u64;

__global__ void k_echo(const u64* go, u64* ack, u64 rounds) {
    for (u64 k = 1; k <= rounds; ++k) {
        u64 v;
        do {
            v = __hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (v == ~0ull) return;   // abort
            __builtin_amdgcn_s_sleep(2);
        } while (v != k);
        __hip_atomic_store(ack, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int run(const char* label, volatile u64* go_host_view, u64* go_dev_ptr, volatile u64* ack, u64 rounds) {
    *go_host_view = 0;
    *ack = 0;
    hipStream_t s;
    if (hipStreamCreate(&s) != hipSuccess) return 1;
    hipLaunchKernelGGL(k_echo, dim3(1), dim3(64), 0, s, go_dev_ptr, (u64*)ack, rounds);
    std::vector<double> rt;
    rt.reserve(rounds);
    for (u64 k = 1; k <= rounds; ++k) {
        const double t0 = now_us();
        __atomic_store_n((u64*)go_host_view, k, __ATOMIC_RELEASE);
        while (__atomic_load_n((u64*)ack, __ATOMIC_ACQUIRE) != k) {
            if (now_us() - t0 > 1e6) {
                *go_host_view = ~0ull;
                hipStreamSynchronize(s);
                printf("{\"place\": \"%s\", \"error\": \"no echo within 1 s at round %llu\"}\n", label, k);
                return 1;
            }
            __builtin_ia32_pause();
        }
        rt.push_back(now_us() - t0);
    }
    hipStreamSynchronize(s);
    hipStreamDestroy(s);
    std::sort(rt.begin(), rt.end());
    printf("{\"place\": \"%s\", \"rounds\": %llu, \"rtt_us_median\": %.3f, \"p10\": %.3f, \"p90\": %.3f}\n", label,
           rounds, rt[rt.size() / 2], rt[rt.size() / 10], rt[rt.size() * 9 / 10]);
    fflush(stdout);
    return 0;
}

int main(int argc, char** argv) {
    const u64 rounds = argc > 1 ? strtoull(argv[1], nullptr, 10) : 20000;
    const bool try_dev = argc > 2 && !strcmp(argv[2], "dev");
    u64 *go_h = nullptr, *ack = nullptr;
    if (hipHostMalloc((void**)&go_h, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return 2;
    if (hipHostMalloc((void**)&ack, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return 2;
    u64* go_h_dev = nullptr;
    hipHostGetDevicePointer((void**)&go_h_dev, go_h, 0);
    if (run("host", go_h, go_h_dev, ack, rounds)) return 1;
    if (!try_dev) return 0;
    u64* go_d = nullptr;
    if (hipExtMallocWithFlags((void**)&go_d, 64, hipDeviceMallocFinegrained) != hipSuccess) {
        printf("{\"place\": \"dev\", \"error\": \"hipExtMallocWithFlags fine-grained failed\"}\n");
        return 0;
    }
    hipPointerAttribute_t attr;
    memset(&attr, 0, sizeof attr);
    hipPointerGetAttributes(&attr, go_d);
    printf("{\"place\": \"dev\", \"pointer_type\": %d, \"hostPointer\": \"%p\", \"devicePointer\": \"%p\"}\n",
           (int)attr.type, attr.hostPointer, attr.devicePointer);
    fflush(stdout);
    volatile u64* view = (volatile u64*)go_d;   // the host stores through the device pointer (large BAR)
    *view = 0x1234;                              // faults here if the CPU cannot map it
    if (*view != 0x1234) {
        printf("{\"place\": \"dev\", \"error\": \"host write/read-back mismatch\"}\n");
        return 0;
    }
    return run("dev", view, go_d, ack, rounds);
}
