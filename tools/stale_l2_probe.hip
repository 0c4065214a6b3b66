// stale_l2_probe.hip — can a receiver's check read see a stale L2 copy of rx
// after a writer outside its L2 replaced the bytes in memory mid-kernel?
//
// That is the situation of the kernel engine across GPUs:
// the peer's pushes arrive over xGMI into this GPU's memory, not through this
// GPU's L2, while the receiver's persistent k_xfer is running and may have
// rx lines in its L2 from an earlier check.  A one-GPU box cannot run two
// GPUs, so the writer here is another client of memory:
//   sdma    hipMemcpyAsync(..., hipMemcpyDeviceToDeviceNoCU): a copy engine,
//           which writes memory without passing any XCD's L2 — the closest
//           stand-in for a remote GPU's writes;
//   ksc1    a kernel on another stream storing with sc0|sc1 (write-through,
//           the kernel engine's own push stores);
//   kplain  the same with plain stores (reaches memory at the writer's end).
//
// One trial: rx = pattern A; the probe kernel (one workgroup per CU, each
// owning a chunk) reads its chunk (LOAD1), reports arrival in host memory and
// spins on a host flag; the host runs the writer (rx = pattern B), waits for
// it, sets the flag; the probe then acquires (ACQ) and reads again (LOAD2),
// counting words still A (stale) and words neither A nor B.
//   LOAD1 / LOAD2   plain | sys (buffer loads, sc0|sc1 — k_xfer's check loads)
//   ACQ             none | agent | system (__builtin_amdgcn_fence acquire;
//                   k_xfer's sum_chunk uses system, then sys loads)
// Prints one JSON line per (writer, LOAD1, ACQ, LOAD2).  Every spin is
// bounded (2 s on the device, 5 s on the host), so a lost flag ends the run.
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/stale_l2_probe tools/stale_l2_probe.hip
//   tools/stale_l2_probe [bytes=4194304] [trials=3]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned long long u64;

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            printf("FAIL %s: %s\n", #x, hipGetErrorString(e_));                          \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

constexpr unsigned kA = 0x11111111u, kB = 0x22222222u;

constexpr int kPlain = 0, kSys = 17;   // 17 = sc0 | sc1 (no volatile bit: gfx950 lowers volatile as sc0 sc1)
constexpr unsigned kRsrcWord3 = 0x00020000;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, kRsrcWord3);
}
__device__ __forceinline__ u64 ld_sys(const u64* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(u64* p, u64 v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ unsigned block_sum(unsigned v) {
    __shared__ unsigned s[4];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
    __syncthreads();
    const unsigned t = s[0] + s[1] + s[2] + s[3];
    __syncthreads();
    return t;
}

// out[3*b + {0,1,2}] = {LOAD1 words != A, LOAD2 words == A, LOAD2 words not A/B}
template <int LOAD1, int ACQ, int LOAD2>
__global__ __launch_bounds__(256) void k_probe(const unsigned char* rx, unsigned chunk, u64* arrive,
                                                const u64* go, u64 epoch, unsigned* out) {
    const __amdgpu_buffer_rsrc_t r = rsrc(rx + (size_t)blockIdx.x * chunk, chunk);
    const int nv = (int)(chunk / 16);
    unsigned bad1 = 0;
    for (int v = threadIdx.x; v < nv; v += 256) {
        const v4u x = __builtin_amdgcn_raw_buffer_load_b128(r, v * 16, 0, LOAD1);
        bad1 += (x.x != kA) + (x.y != kA) + (x.z != kA) + (x.w != kA);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ int timed_out;
    if (threadIdx.x == 0) {
        timed_out = 0;
        st_sys(&arrive[blockIdx.x], epoch);
        const u64 t0 = __builtin_amdgcn_s_memrealtime();
        while (ld_sys(go) < epoch) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) { timed_out = 1; break; }   // 2 s at 100 MHz
            __builtin_amdgcn_s_sleep(2);
        }
        if constexpr (ACQ == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if constexpr (ACQ == 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    unsigned stale = 0, other = 0;
    for (int v = threadIdx.x; v < nv; v += 256) {
        const v4u x = __builtin_amdgcn_raw_buffer_load_b128(r, v * 16, 0, LOAD2);
        stale += (x.x == kA) + (x.y == kA) + (x.z == kA) + (x.w == kA);
        other += (x.x != kA && x.x != kB) + (x.y != kA && x.y != kB) + (x.z != kA && x.z != kB) +
                 (x.w != kA && x.w != kB);
    }
    bad1 = block_sum(bad1);
    stale = block_sum(stale);
    other = block_sum(other);
    if (threadIdx.x == 0) {
        out[3 * blockIdx.x] = bad1 + (timed_out ? 0x40000000u : 0u);
        out[3 * blockIdx.x + 1] = stale;
        out[3 * blockIdx.x + 2] = other;
    }
}

template <int AUX>
__global__ __launch_bounds__(256) void k_write(unsigned char* rx, size_t n) {
    const __amdgpu_buffer_rsrc_t r = rsrc(rx, (unsigned)n);
    const v4u b = {kB, kB, kB, kB};
    for (size_t v = (size_t)blockIdx.x * 256 + threadIdx.x; v < n / 16; v += (size_t)gridDim.x * 256)
        __builtin_amdgcn_raw_buffer_store_b128(b, r, (unsigned)(v * 16), 0, AUX);
}

typedef void (*probe_fn)(const unsigned char*, unsigned, u64*, const u64*, u64, unsigned*);
static const char* kLoad[2] = {"plain", "sys"};
static const char* kAcq[3] = {"none", "agent", "system"};
template <int L1, int A, int L2>
static void* fn() { return reinterpret_cast<void*>(&k_probe<L1, A, L2>); }
static void* probe_of(int l1, int a, int l2) {
    void* t[2][3][2] = {
        {{fn<kPlain, 0, kPlain>(), fn<kPlain, 0, kSys>()}, {fn<kPlain, 1, kPlain>(), fn<kPlain, 1, kSys>()},
         {fn<kPlain, 2, kPlain>(), fn<kPlain, 2, kSys>()}},
        {{fn<kSys, 0, kPlain>(), fn<kSys, 0, kSys>()}, {fn<kSys, 1, kPlain>(), fn<kSys, 1, kSys>()},
         {fn<kSys, 2, kPlain>(), fn<kSys, 2, kSys>()}}};
    return t[l1][a][l2];
}

static double now_s() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 0) : ((size_t)4 << 20);
    const int trials = argc > 2 ? atoi(argv[2]) : 3;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int grid = prop.multiProcessorCount;   // one workgroup per CU: all co-resident
    const unsigned chunk = (unsigned)((n / grid) & ~(size_t)15);
    if (chunk < 16) { printf("FAIL bytes too small\n"); return 1; }
    unsigned char *rx, *srcB;
    CK(hipMalloc(&rx, n));
    CK(hipMalloc(&srcB, n));
    CK(hipMemset(srcB, 0x22, n));
    u64 *arrive, *go;
    CK(hipHostMalloc(reinterpret_cast<void**>(&arrive), sizeof(u64) * grid, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc(reinterpret_cast<void**>(&go), sizeof(u64), hipHostMallocCoherent | hipHostMallocMapped));
    memset(arrive, 0, sizeof(u64) * grid);
    *go = 0;
    unsigned* out;
    CK(hipMalloc(&out, sizeof(unsigned) * 3 * grid));
    unsigned* hout = (unsigned*)malloc(sizeof(unsigned) * 3 * grid);
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    static const char* kWriter[3] = {"sdma", "ksc1", "kplain"};
    u64 epoch = 0;
    for (int w = 0; w < 3; ++w)
        for (int l1 = 0; l1 < 2; ++l1)
            for (int a = 0; a < 3; ++a)
                for (int l2 = 0; l2 < 2; ++l2) {
                    unsigned long long stale = 0, other = 0, bad1 = 0;
                    int lost = 0;
                    for (int t = 0; t < trials; ++t) {
                        ++epoch;
                        CK(hipMemsetAsync(rx, 0x11, n, s1));
                        CK(hipMemsetAsync(out, 0, sizeof(unsigned) * 3 * grid, s1));
                        CK(hipStreamSynchronize(s1));
                        hipLaunchKernelGGL(reinterpret_cast<probe_fn>(probe_of(l1, a, l2)), dim3(grid), dim3(256), 0,
                                           s1, rx, chunk, arrive, go, epoch, out);
                        CK(hipGetLastError());
                        const double t0 = now_s();
                        for (;;) {
                            int k = 0;
                            while (k < grid && __atomic_load_n(&arrive[k], __ATOMIC_ACQUIRE) >= epoch) ++k;
                            if (k == grid) break;
                            if (now_s() - t0 > 5.0) { lost = 1; break; }
                        }
                        if (w == 0) {
                            CK(hipMemcpyAsync(rx, srcB, n, hipMemcpyDeviceToDeviceNoCU, s2));
                        } else if (w == 1) {
                            hipLaunchKernelGGL(k_write<17>, dim3(64), dim3(256), 0, s2, rx, n);
                        } else {
                            hipLaunchKernelGGL(k_write<0>, dim3(64), dim3(256), 0, s2, rx, n);
                        }
                        CK(hipGetLastError());
                        CK(hipStreamSynchronize(s2));
                        __atomic_store_n(go, epoch, __ATOMIC_RELEASE);
                        CK(hipStreamSynchronize(s1));
                        CK(hipMemcpy(hout, out, sizeof(unsigned) * 3 * grid, hipMemcpyDeviceToHost));
                        for (int b = 0; b < grid; ++b) {
                            if (hout[3 * b] & 0x40000000u) lost = 1;
                            bad1 += hout[3 * b] & 0x3fffffffu;
                            stale += hout[3 * b + 1];
                            other += hout[3 * b + 2];
                        }
                    }
                    printf("{\"writer\": \"%s\", \"load1\": \"%s\", \"acquire\": \"%s\", \"load2\": \"%s\", "
                           "\"bytes\": %zu, \"trials\": %d, \"words_per_trial\": %zu, \"stale_words\": %llu, "
                           "\"other_words\": %llu, \"load1_bad\": %llu, \"lost_flag\": %d}\n",
                           kWriter[w], kLoad[l1], kAcq[a], kLoad[l2], n, trials, (size_t)chunk / 4 * grid, stale,
                           other, bad1, lost);
                    fflush(stdout);
                }
    CK(hipStreamDestroy(s1));
    CK(hipStreamDestroy(s2));
    return 0;
}
