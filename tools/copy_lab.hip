// copy_lab.hip — standalone tuning lab for the HBM copy kernel (not product
// code; the product kernel is k_copy in mpi-perf_amd/csrc/mpx_kernels.hip).
// Times every variant over a 1 GiB copy with HIP events (avg of 20 launches,
// best of 5 reps) and checks the output.  One JSON line per variant.
//   hipcc --offload-arch=gfx950 -O3 -o tools/copy_lab tools/copy_lab.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

constexpr unsigned kW3 = 0x00020000;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, kW3);
}

// A: block-contiguous chunk, plain/nt pointer loads (product form)
template <int T, int U, bool NT>
__global__ __launch_bounds__(T) void kA(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n16) {
    const size_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const size_t lo = (size_t)blockIdx.x * per;
    const size_t end = lo + per < n16 ? lo + per : n16;
    size_t i = lo + threadIdx.x;
    for (; i + (U - 1) * T < end; i += U * T) {
        v4u r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) r[u] = NT ? __builtin_nontemporal_load(s + i + u * T) : s[i + u * T];
#pragma unroll
        for (int u = 0; u < U; ++u) { if (NT) __builtin_nontemporal_store(r[u], d + i + u * T); else d[i + u * T] = r[u]; }
    }
    for (; i < end; i += T) d[i] = s[i];
}

// B: block-contiguous chunk with buffer ops and explicit cache-policy aux
template <int T, int U, int LA, int SA>
__global__ __launch_bounds__(T) void kB(const unsigned char* s, unsigned char* d, size_t n, size_t per) {
    const size_t lo = (size_t)blockIdx.x * per;
    if (lo >= n) return;
    const unsigned bytes = (unsigned)(lo + per < n ? per : n - lo);
    const __amdgpu_buffer_rsrc_t rs = rsrc(s + lo, bytes), rd = rsrc(d + lo, bytes);
    unsigned o = threadIdx.x * 16;
    for (; o + (U - 1) * T * 16 < bytes; o += U * T * 16) {
        v4u r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) r[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, o + u * T * 16, 0, LA);
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_amdgcn_raw_buffer_store_b128(r[u], rd, o + u * T * 16, 0, SA);
    }
    for (; o < bytes; o += T * 16)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, LA), rd, o, 0, SA);
}

// C: wave tiles — each wave copies a contiguous (U KiB) tile per step, tiles
// assigned grid-stride over all waves (DRAM-page-friendly, no block chunk)
template <int T, int U, bool NT>
__global__ __launch_bounds__(T) void kC(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n16) {
    const size_t waves = (size_t)gridDim.x * (T / 64);
    const size_t w = (size_t)blockIdx.x * (T / 64) + (threadIdx.x >> 6);
    const unsigned lane = threadIdx.x & 63;
    const size_t tile = 64 * U;   // 16-B units per wave tile
    for (size_t t = w * tile; t < n16; t += waves * tile) {
        v4u r[U];
        if (t + tile <= n16) {
#pragma unroll
            for (int u = 0; u < U; ++u) r[u] = NT ? __builtin_nontemporal_load(s + t + u * 64 + lane) : s[t + u * 64 + lane];
#pragma unroll
            for (int u = 0; u < U; ++u) { if (NT) __builtin_nontemporal_store(r[u], d + t + u * 64 + lane); else d[t + u * 64 + lane] = r[u]; }
        } else {
            for (size_t i = t + lane; i < n16; i += 64) d[i] = s[i];
        }
    }
}

// D: persistent block-contiguous, XCD-aware: blocks b, b+8, b+16.. run on one
// XCD; give each XCD one contiguous eighth of the buffer
template <int T, int U>
__global__ __launch_bounds__(T) void kD(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n16) {
    const unsigned G = gridDim.x, b = blockIdx.x;
    const unsigned xcd = b & 7, k = b >> 3, per_xcd = G >> 3;
    const unsigned vb = xcd * per_xcd + k;       // virtual block: contiguous per XCD
    const size_t per = (n16 + G - 1) / G;
    const size_t lo = (size_t)vb * per;
    const size_t end = lo + per < n16 ? lo + per : n16;
    size_t i = lo + threadIdx.x;
    for (; i + (U - 1) * T < end; i += U * T) {
        v4u r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) r[u] = __builtin_nontemporal_load(s + i + u * T);
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_nontemporal_store(r[u], d + i + u * T);
    }
    for (; i < end; i += T) d[i] = s[i];
}


// E: one step per block, no loop: block b copies units [b*T*U, (b+1)*T*U)
template <int T, int U>
__global__ __launch_bounds__(T) void kE(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n16) {
    const size_t base = (size_t)blockIdx.x * (T * U) + threadIdx.x;
    if (base + (U - 1) * T < n16) {
        v4u r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) r[u] = __builtin_nontemporal_load(s + base + u * T);
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_nontemporal_store(r[u], d + base + u * T);
    } else {
        for (size_t i = base; i < n16; i += T) d[i] = s[i];
    }
}
template <int T, int U> void runE(const void* s, void* d, size_t n, int, int, hipStream_t st) {
    const size_t n16 = n / 16, g = (n16 + T * U - 1) / (T * U);
    hipLaunchKernelGGL((kE<T, U>), dim3((unsigned)g), dim3(T), 0, st, (const v4u*)s, (v4u*)d, n16);
}
// R / W: one-direction ceilings of the same shape (one 16-B unit per lane,
// one step per workgroup): R reads src (nontemporal) and folds it into one
// word per workgroup; W stores a constant.  Timed traffic is B per launch;
// the lab's rate column counts 2B, so halve it for these two.
__global__ __launch_bounds__(256) void kR(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n16) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    v4u r = {0, 0, 0, 0};
    if (i < n16) r = __builtin_nontemporal_load(s + i);
    unsigned x = r.x ^ r.y ^ r.z ^ r.w;
    for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o);
    if (x == 0x9e3779b9u && threadIdx.x == 0) d[blockIdx.x] = r;   // keeps the loads live
}
__global__ __launch_bounds__(256) void kW(const v4u* __restrict__, v4u* __restrict__ d, size_t n16) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const v4u v = {(unsigned)i, 1u, 2u, 3u};
    if (i < n16) __builtin_nontemporal_store(v, d + i);
}
void runR(const void* s, void* d, size_t n, int, int, hipStream_t st) {
    hipLaunchKernelGGL(kR, dim3((unsigned)((n / 16 + 255) / 256)), dim3(256), 0, st, (const v4u*)s, (v4u*)d, n / 16);
}
void runW(const void* s, void* d, size_t n, int, int, hipStream_t st) {
    hipLaunchKernelGGL(kW, dim3((unsigned)((n / 16 + 255) / 256)), dim3(256), 0, st, (const v4u*)s, (v4u*)d, n / 16);
}
// M: the runtime's own device-to-device copy
void runM(const void* s, void* d, size_t n, int, int, hipStream_t st) { (void)hipMemcpyAsync(d, s, n, hipMemcpyDeviceToDevice, st); }

__global__ void kfill(unsigned* p, size_t n4) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += gridDim.x * 256ull) p[i] = (unsigned)(i * 2654435761u) ^ 0x5a5a1234u;
}
__global__ void kcmp(const unsigned* a, const unsigned* b, size_t n4, unsigned* bad) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += gridDim.x * 256ull)
        if (a[i] != b[i]) atomicAdd(bad, 1u);
}

struct Var { const char* name; int grid, threads; void (*run)(const void*, void*, size_t, int, int, hipStream_t); };

template <int T, int U, bool NT> void runA(const void* s, void* d, size_t n, int g, int, hipStream_t st) {
    hipLaunchKernelGGL((kA<T, U, NT>), dim3(g), dim3(T), 0, st, (const v4u*)s, (v4u*)d, n / 16);
}
template <int T, int U, int LA, int SA> void runB(const void* s, void* d, size_t n, int g, int, hipStream_t st) {
    size_t per = ((n + g - 1) / g + 15) & ~(size_t)15;
    hipLaunchKernelGGL((kB<T, U, LA, SA>), dim3(g), dim3(T), 0, st, (const unsigned char*)s, (unsigned char*)d, n, per);
}
template <int T, int U, bool NT> void runC(const void* s, void* d, size_t n, int g, int, hipStream_t st) {
    hipLaunchKernelGGL((kC<T, U, NT>), dim3(g), dim3(T), 0, st, (const v4u*)s, (v4u*)d, n / 16);
}
template <int T, int U> void runD(const void* s, void* d, size_t n, int g, int, hipStream_t st) {
    hipLaunchKernelGGL((kD<T, U>), dim3(g), dim3(T), 0, st, (const v4u*)s, (v4u*)d, n / 16);
}

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], 0, 0) : (1ull << 30);
    const char* only = argc > 2 ? argv[2] : nullptr;
    // optional placement offsets (argv[3] dst, argv[4] src, bytes): where the
    // two buffers sit relative to each other in the HBM channel interleave
    const size_t doff = argc > 3 ? strtoull(argv[3], 0, 0) : 0, soff = argc > 4 ? strtoull(argv[4], 0, 0) : 0;
    void *s, *d, *s0, *d0;
    unsigned* bad;
    CK(hipMalloc(&s0, n + soff));
    CK(hipMalloc(&d0, n + doff));
    s = (char*)s0 + soff;
    d = (char*)d0 + doff;
    CK(hipMalloc(&bad, 4));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipLaunchKernelGGL(kfill, dim3(4096), dim3(256), 0, st, (unsigned*)s, n / 4);
    CK(hipStreamSynchronize(st));
    // aux: sc0 = 1, nt = 2, sc1 = 16 (gfx940-family buffer cache policy bits)
    std::vector<Var> vs = {
        {"A_t256_u2_nt_g65536 (product)", 65536, 256, runA<256, 2, true>},
        {"E_t256_u1", 0, 256, runE<256, 1>},
        {"E_t256_u2", 0, 256, runE<256, 2>},
        {"E_t256_u4", 0, 256, runE<256, 4>},
        {"E_t512_u1", 0, 512, runE<512, 1>},
        {"E_t512_u2", 0, 512, runE<512, 2>},
        {"E_t1024_u1", 0, 1024, runE<1024, 1>},
        {"E_t1024_u2", 0, 1024, runE<1024, 2>},
        {"E_t128_u2", 0, 128, runE<128, 2>},
        {"E_t64_u4", 0, 64, runE<64, 4>},
        {"A_t256_u1_nt_g262144", 262144, 256, runA<256, 1, true>},
        {"A_t512_u1_nt_g131072", 131072, 512, runA<512, 1, true>},
        {"M_hipMemcpyAsync_D2D", 0, 0, runM},
        {"R_read_only (rate x0.5 = read GB/s)", 0, 256, runR},
        {"W_write_only (rate x0.5 = write GB/s)", 0, 256, runW},
        {"A_t256_u2_nt_g65536 (product, again)", 65536, 256, runA<256, 2, true>},
        {"E_t256_u1 (again)", 0, 256, runE<256, 1>},
        {"E_t512_u1 (again)", 0, 512, runE<512, 1>},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int L = 20;
    for (const Var& v : vs) {
        if (only && !strstr(v.name, only)) continue;
        CK(hipMemsetAsync(d, 0, n, st));
        v.run(s, d, n, v.grid, v.threads, st);   // warm
        CK(hipGetLastError());
        CK(hipMemsetAsync(bad, 0, 4, st));
        hipLaunchKernelGGL(kcmp, dim3(4096), dim3(256), 0, st, (const unsigned*)s, (const unsigned*)d, n / 4, bad);
        unsigned nb = 0;
        CK(hipMemcpyAsync(&nb, bad, 4, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        double best = 0, sum = 0;
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipEventRecord(e0, st));
            for (int l = 0; l < L; ++l) v.run(s, d, n, v.grid, v.threads, st);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double gbps = 2.0 * n * L / (ms * 1e-3) / 1e9;
            sum += gbps;
            if (gbps > best) best = gbps;
        }
        printf("{\"variant\": \"%s\", \"bytes\": %zu, \"dst_off\": %zu, \"src_off\": %zu, \"hbm_GBps_best\": %.1f, \"hbm_GBps_mean\": %.1f, \"bad_words\": %u}\n",
               v.name, n, doff, soff, best, sum / 5, nb);
        fflush(stdout);
    }
    return 0;
}
