// mpx_kernels.hip — CDNA4 (gfx950) device code of libmpx.
//
// Kernels
//   k_copy      local HBM copy, one 16-B unit per lane, one step per block (config 2)
//   k_xfer      the reference's three transfer loops as ONE persistent launch
//               per rank: pushes go straight into the peer's HBM over xGMI,
//               receives are device-side polls of the rank's mailbox
//               (do_mpi_benchmark*, /root/reference/mpi_perf.c:66-145)
//   k_fill      tx fill (memset 'a'/'b', mpi_perf.c:244-251, or a seeded pattern)
//   k_checksum  order-independent 64-bit payload checksum
//   k_signal / k_wait   one-lane flag store / bounded poll (SDMA engine)
//
// Memory-ordering contract (see DESIGN.md "Hand-off"):
//  * bulk payload: 16-B buffer stores with sc0|sc1 (system-scope write-through),
//    every storing wave `s_waitcnt vmcnt(0)`, workgroup barrier, then ONE lane
//    stores the workgroup's flag with a system-scope relaxed store;
//  * LL payload (<= 8 KiB, or a 1-byte ack): the data IS the flag — 8-byte
//    {tag, 4 payload bytes} granules, each written by one system-scope store;
//  * receivers poll with system-scope relaxed loads (sc0 sc1) and bounded
//    spins (s_memrealtime deadline); after a timeout every workgroup exits.
#include "mpx_internal.h"

namespace mpx {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

constexpr u64 kGolden = 0x9E3779B97F4A7C15ull;
constexpr int kAuxSys = 17;                 // buffer cache policy: sc0 | sc1
constexpr int kAuxSysNt = 19;               // sc0 | nt | sc1 (MPX_XFER_STREAM)
constexpr int kAuxSysVol = (int)0x80000011u; // sc0 | sc1, volatile (re-issued every poll)
constexpr int kLLUnits = kLLGranules / 2;    // 16-B LL units (two granules each)
constexpr int kLLUnitsPerLane = kLLUnits / kBlock;
constexpr unsigned kRsrcWord3 = 0x00020000; // raw buffer, 32-bit data format

__device__ __forceinline__ u64 mix64(u64 z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
// checksum term of little-endian 64-bit word w at word index k
__device__ __forceinline__ u64 csum_term(u64 w, u64 k) { return mix64(w + (k + 1) * kGolden); }
// MPX_FILL_SPLITMIX word k
__device__ __forceinline__ u64 fill_word(u64 key, u64 k) { return mix64((key ^ k) + kGolden); }

__device__ __forceinline__ u64 ld_sys(const u64* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(u64* p, u64 v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ u64 now_ticks() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, kRsrcWord3);
}

// 64-bit sum over the workgroup; result valid in thread 0.
__device__ __forceinline__ u64 block_sum(u64 v, u64* lds4) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) lds4[wave] = v;
    __syncthreads();
    u64 s = 0;
    if (threadIdx.x == 0) s = lds4[0] + lds4[1] + lds4[2] + lds4[3];
    __syncthreads();
    return s;
}

// ---------------------------------------------------------------------------
// k_copy: dst[0:n) = src[0:n).  n16 = n / 16 vector units; the tail bytes are
// copied by block 0.  Every lane keeps U independent 16-B loads in flight.
//   CONTIG = false: grid-stride over the whole buffer (unit i, i+G, ...)
//   CONTIG = true : block b owns one contiguous chunk, swept 4 KiB per step
//   LDNT / STNT   : nontemporal (streaming) loads / stores
// launch_copy runs one form: U = 1, nontemporal both ways, one step per block.
// ---------------------------------------------------------------------------
template <bool NT>
__device__ __forceinline__ v4u ld16(const v4u* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st16(v4u* p, v4u v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <int U, bool LDNT, bool STNT, bool CONTIG>
__global__ __launch_bounds__(kBlock) void k_copy(const v4u* __restrict__ src, v4u* __restrict__ dst,
                                                size_t n16, unsigned tail) {
    size_t i, end, stride;
    if constexpr (CONTIG) {
        const size_t per = (n16 + gridDim.x - 1) / gridDim.x;
        const size_t lo = (size_t)blockIdx.x * per;
        end = lo + per < n16 ? lo + per : n16;
        i = lo + threadIdx.x;
        stride = kBlock;
    } else {
        end = n16;
        i = (size_t)blockIdx.x * kBlock + threadIdx.x;
        stride = (size_t)gridDim.x * kBlock;
    }
    for (; i + (U - 1) * stride < end; i += U * stride) {
        v4u r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) r[u] = ld16<LDNT>(src + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) st16<STNT>(dst + i + u * stride, r[u]);
    }
    for (; i < end; i += stride) st16<STNT>(dst + i, ld16<LDNT>(src + i));
    if (blockIdx.x == 0 && threadIdx.x < tail) {
        const unsigned char* s8 = reinterpret_cast<const unsigned char*>(src + n16);
        unsigned char* d8 = reinterpret_cast<unsigned char*>(dst + n16);
        d8[threadIdx.x] = s8[threadIdx.x];
    }
}

// ---------------------------------------------------------------------------
// k_copy_steps: all `iters` copies dst[0:n) = src[0:n) of one mpx_copy call in
// ONE launch (the reference's loop, mpi_perf.c:70, run on the device like
// k_xfer runs the pair loop).  Below a few MiB a launch of k_copy costs
// 2.1-2.5 us whatever it moves (profiles/r01_cfg2_copy_sweep.jsonl), so the
// sweep's small sizes measured dispatch, not memory.  Every lane owns the
// same 16-B units every step (grid-stride, U = ceil(n16 / (grid*256)) per
// lane); between steps a grid barrier: one lane per workgroup counts in
// (optionally after draining its stores) and waits for the whole grid, so
// step s+1's loads start only after every store of
// step s was issued — back-to-back copies, not an overlapped pipeline.  The
// grid (<= 4 workgroups per CU, 12 VGPRs) is always co-resident.
// ---------------------------------------------------------------------------
// Each lane issues the loads of up to kCopyStepsBatch of its units before
// the first store, so a step costs about one memory latency per batch, not
// one per unit (the grid is sized to give every lane <= one batch per step
// below 1 MiB).
constexpr int kCopyStepsBatch = 8;

template <int T, bool XCD>
__global__ __launch_bounds__(T) void k_copy_steps(const v4u* __restrict__ src, v4u* __restrict__ dst, size_t n16,
                                                 unsigned tail, int iters, u64* bar, int drain, int one_xcd) {
    // one_xcd: the grid is 8x the working workgroups and only those with
    // blockIdx % 8 == 0 work (the rest exit at once), so that with the
    // round-robin dispatch seen on gfx950 every barrier arrival comes from
    // XCD 0.  A placement heuristic, speed only: dispatch -> XCD placement is
    // undefined (MI355X_MICROARCH.md), and the working set is correct
    // wherever it lands (sized to stay resident; the barrier is bounded)
    if (one_xcd && (blockIdx.x & 7)) return;
    const unsigned wg = one_xcd ? blockIdx.x >> 3 : blockIdx.x;
    const u64 g = one_xcd ? gridDim.x >> 3 : gridDim.x;
    const size_t stride = (size_t)g * T;
    const size_t first = (size_t)wg * T + threadIdx.x;
    // XCD = true: two-level arrival.  Workgroups are dispatched round-robin
    // over the 8 XCDs, so workgroup b counts in on its XCD's counter
    // bar[16 * (1 + b % 8)] (8 counters, 128 B apart, in parallel instead of
    // one hot word); the last arriver of each XCD then counts that XCD in on
    // bar[0].
    const int x = (int)(wg & 7);
    const u64 nx = (g - (u64)x + 7) / 8;            // workgroups on this XCD
    const u64 groups = g < 8 ? g : 8;
    const bool one_unit = n16 <= stride;   // at most one unit per lane: no batch
    __shared__ int s_stop;
    for (int s = 0; s < iters; ++s) {
        if (one_unit) {
            if (first < n16) __builtin_nontemporal_store(__builtin_nontemporal_load(src + first), dst + first);
        } else for (size_t base = first; base < n16; base += kCopyStepsBatch * stride) {
            v4u r[kCopyStepsBatch];
#pragma unroll
            for (int u = 0; u < kCopyStepsBatch; ++u)
                if (base + u * stride < n16) r[u] = __builtin_nontemporal_load(src + base + u * stride);
#pragma unroll
            for (int u = 0; u < kCopyStepsBatch; ++u)
                if (base + u * stride < n16) __builtin_nontemporal_store(r[u], dst + base + u * stride);
        }
        if (wg == 0 && threadIdx.x < tail) {
            const unsigned char* s8 = reinterpret_cast<const unsigned char*>(src + n16);
            reinterpret_cast<unsigned char*>(dst + n16)[threadIdx.x] = s8[threadIdx.x];
        }
        if (s + 1 == iters) break;
        if (drain) drain_stores();
        __syncthreads();
        if (g == 1) continue;                       // one workgroup: __syncthreads is the barrier
        if (threadIdx.x == 0) {
            s_stop = 0;
            u64 want;
            if constexpr (XCD) {
                const u64 old = __hip_atomic_fetch_add(bar + 16 * (1 + x), 1ull, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
                if (old + 1 == nx * (u64)(s + 1))
                    __hip_atomic_fetch_add(bar, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                want = groups * (u64)(s + 1);
            } else {
                __hip_atomic_fetch_add(bar, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                want = g * (u64)(s + 1);
            }
            // bounded: the grid is sized to be resident, but a workgroup that
            // never arrives must not hold the GPU: after 1 s the workgroup
            // stops and flags bar[1], which mpx_copy reports as a timeout
            const u64 t0 = now_ticks();
            u64 spins = 0;
            while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
                if ((++spins & 255) == 0 && now_ticks() - t0 > 100000000ull) {
                    __hip_atomic_store(&bar[1], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    s_stop = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
        if (s_stop) return;
    }
}

// ---------------------------------------------------------------------------
// k_copy_pipe: the same `iters` back-to-back copies in ONE launch, for the
// sizes where k_copy_steps pays three memory round trips per copy (loads,
// then the stores' completion — __syncthreads drains them —, then the grid
// barrier's atomic and poll; profiles/r03_copy_cliff_*).  Here a copy's step
// costs about one:
//  * four "copy" waves own UPL 16-B units per lane; copy s+1's loads are
//    issued BEFORE copy s's stores (src is read-only while the copies run,
//    and dst is written only by the stores), so they are in flight during
//    copy s's grid barrier; two register sets, unrolled by two, no moves;
//  * a fifth wave runs the grid barrier: its vector-memory counter holds
//    only the barrier's atomic and poll, so waiting for the poll never waits
//    for the copy waves' stores.  Workgroup barriers are plain s_barrier
//    (no fence: nothing drains); the copy waves wait only for their own
//    loads of the next copy (vmcnt counts in issue order, and those loads
//    are older than this copy's stores).
// Copy s+1's stores are issued only after every workgroup has issued copy
// s's stores (the grid barrier orders issue); the kernel's end makes every
// store visible, as a launch per copy does.
// ---------------------------------------------------------------------------
constexpr int kPipeCopyWaves = 4;
constexpr int kPipeThreads = (kPipeCopyWaves + 1) * 64;   // + the barrier wave
constexpr int kAuxNt = 2;                                 // buffer op: nt (streaming)


__device__ __forceinline__ void wg_barrier_nofence() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // LDS (s_stop) before the barrier
    __builtin_amdgcn_s_barrier();
    // LLVM models s_barrier as touching no memory: without a compiler barrier
    // after it too, the s_stop read or the next copy's stores could be
    // scheduled above it
    asm volatile("" ::: "memory");
}

// Branch-free copy-wave code: every unit is a buffer op whose resource ends at
// n16 units (out-of-range loads return 0, out-of-range stores are dropped),
// so the compiler can count each wait exactly (a guarded unit made it wait
// for every outstanding load, the next copy's included).  The < 16 tail bytes
// go the same way through a resource that is empty except in workgroup 0's
// first wave.
template <int UPL>
// (no __restrict__ on src: with it the optimiser may assume src's bytes never
// change during the kernel and keep the first copy's values for every copy)
__global__ __launch_bounds__(kPipeThreads) void k_copy_pipe(const v4u* src, v4u* dst,
                                                          size_t n16, unsigned tail, int iters, u64* bar,
                                                          int hier) {
    __shared__ int s_stop;
    if (threadIdx.x >= kPipeCopyWaves * 64) {
        // the barrier wave: one grid barrier per copy boundary.  hier = 0:
        // one counter (bar[0]) that every workgroup counts in on and polls.
        // hier = 1 (A/B): workgroup b counts in on its group's counter
        // bar[16 (1 + b % 8)]; the last of a group counts the group in on
        // bar[0]; the last group writes every group's release word
        // bar[16 (9 + g)], which that group's workgroups poll — 8 same-address
        // queues in parallel instead of one.
        const unsigned grid = gridDim.x;
        const unsigned g = blockIdx.x & 7;
        const u64 ng = (grid - g + 7) / 8;                   // workgroups in group g
        const u64 groups = grid < 8 ? grid : 8;
        for (int s = 0; s + 1 < iters; ++s) {
            wg_barrier_nofence();                      // every copy wave issued copy s's stores
            if (threadIdx.x == kPipeCopyWaves * 64) {
                s_stop = 0;
                u64 want;
                const u64* poll;
                if (hier) {
                    const u64 old = __hip_atomic_fetch_add(bar + 16 * (1 + g), 1ull, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT);
                    if (old + 1 == ng * (u64)(s + 1)) {
                        const u64 t = __hip_atomic_fetch_add(bar, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (t + 1 == groups * (u64)(s + 1))
                            for (u64 k = 0; k < groups; ++k)
                                __hip_atomic_store(bar + 16 * (9 + k), (u64)(s + 1), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
                    }
                    want = (u64)(s + 1);
                    poll = bar + 16 * (9 + g);
                } else {
                    __hip_atomic_fetch_add(bar, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    want = (u64)grid * (u64)(s + 1);
                    poll = bar;
                }
                const u64 t0 = now_ticks();
                u64 spins = 0;
                while (__hip_atomic_load(poll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
                    if ((++spins & 255) == 0 && now_ticks() - t0 > 100000000ull) {
                        // 1 s: a workgroup never arrived (bar[1] -> mpx_copy's fallback)
                        __hip_atomic_store(&bar[1], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        s_stop = 1;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            wg_barrier_nofence();
            if (s_stop) return;
        }
        return;
    }
    const unsigned stride16 = gridDim.x * (kPipeCopyWaves * 64) * 16u;     // bytes between a lane's units
    const unsigned first16 = (blockIdx.x * (kPipeCopyWaves * 64) + threadIdx.x) * 16u;
    const unsigned body = (unsigned)(n16 * 16);
    const __amdgpu_buffer_rsrc_t rs = rsrc(src, body), rd = rsrc(dst, body);
    // wave-uniform, made scalar so the tail resources live in SGPRs
    const unsigned tb = __builtin_amdgcn_readfirstlane((blockIdx.x == 0 && threadIdx.x < 64) ? tail : 0u);
    const __amdgpu_buffer_rsrc_t ts = rsrc(reinterpret_cast<const unsigned char*>(src) + body, tb);
    const __amdgpu_buffer_rsrc_t td = rsrc(reinterpret_cast<unsigned char*>(dst) + body, tb);
    v4u a[UPL], b[UPL];
    unsigned char ta, tb8;
    auto load = [&](v4u (&r)[UPL], unsigned char& t) {
        // a compiler barrier: the buffer-load builtin is a plain memory read to
        // the optimiser, which would otherwise reuse the previous copy's values
        asm volatile("" ::: "memory");
#pragma unroll
        for (int u = 0; u < UPL; ++u)
            r[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, first16 + u * stride16, 0, kAuxNt);
        t = __builtin_amdgcn_raw_buffer_load_b8(ts, threadIdx.x, 0, 0);
    };
    auto store = [&](v4u (&r)[UPL], unsigned char t) {
#pragma unroll
        for (int u = 0; u < UPL; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(r[u], rd, first16 + u * stride16, 0, kAuxNt);
        __builtin_amdgcn_raw_buffer_store_b8(t, td, threadIdx.x, 0, 0);
    };
    // both workgroup barriers of a grid barrier; false: the barrier gave up
    auto grid_barrier = [&]() -> bool {
        wg_barrier_nofence();
        wg_barrier_nofence();
        return !s_stop;
    };
    // copy s+1's loads are issued before copy s's stores (src is read-only
    // while the copies run), so they fly during copy s's grid barrier
    load(a, ta);
    for (int s = 0;;) {
        if (s + 1 == iters) { store(a, ta); break; }
        load(b, tb8);
        store(a, ta);
        if (!grid_barrier()) break;
        if (++s + 1 == iters) { store(b, tb8); break; }
        load(a, ta);
        store(b, tb8);
        if (!grid_barrier()) break;
        ++s;
    }
}

// ---------------------------------------------------------------------------
// k_fill
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_fill(unsigned char* p, size_t n, int pattern, u64 arg) {
    const size_t nw = n / 8;
    const size_t stride = (size_t)gridDim.x * kBlock;
    u64* p64 = reinterpret_cast<u64*>(p);
    const u64 bytew = (arg & 0xff) * 0x0101010101010101ull;
    for (size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x; k < nw; k += stride)
        p64[k] = pattern == MPX_FILL_BYTE ? bytew : fill_word(arg, k);
    const unsigned tail = (unsigned)(n & 7);
    if (blockIdx.x == 0 && threadIdx.x < tail) {
        const u64 w = pattern == MPX_FILL_BYTE ? bytew : fill_word(arg, nw);
        p[nw * 8 + threadIdx.x] = (unsigned char)(w >> (8 * threadIdx.x));
    }
}

// ---------------------------------------------------------------------------
// k_checksum: *out += sum_k csum_term(word_k, k) over the zero-padded 64-bit
// words of p[0:n).  Integer adds commute, so the result is bit-exact whatever
// the order; the host finishes it with ^ mix64(n).
// ---------------------------------------------------------------------------
__device__ __forceinline__ u64 tail_word(const unsigned char* p, size_t off, size_t n) {
    u64 w = 0;
    for (size_t b = 0; off + b < n && b < 8; ++b) w |= (u64)p[off + b] << (8 * b);
    return w;
}

__global__ __launch_bounds__(kBlock) void k_checksum(const unsigned char* p, size_t n, u64* out) {
    __shared__ u64 lds4[4];
    const size_t n16 = n / 16;
    const size_t stride = (size_t)gridDim.x * kBlock;
    const v4u* p16 = reinterpret_cast<const v4u*>(p);
    u64 acc = 0;
    for (size_t v = (size_t)blockIdx.x * kBlock + threadIdx.x; v < n16; v += stride) {
        const v4u x = p16[v];
        acc += csum_term(((u64)x.y << 32) | x.x, 2 * v);
        acc += csum_term(((u64)x.w << 32) | x.z, 2 * v + 1);
    }
    if (blockIdx.x == 0 && threadIdx.x < 2) {
        const size_t off = n16 * 16 + 8 * threadIdx.x;
        if (off < n) acc += csum_term(tail_word(p, off, n), off / 8);
    }
    const u64 s = block_sum(acc, lds4);
    if (threadIdx.x == 0 && s) atomicAdd(out, s);
}

// ---------------------------------------------------------------------------
// SDMA-engine helpers: one lane stores / polls a mailbox flag.  The value is
// v, plus *base when base is set: a graph-captured chunk of the loop
// (run_sdma) carries sequence numbers relative to a device-side base that
// k_seqbase sets before the first replay and advances at the end of each.
// ---------------------------------------------------------------------------
__device__ __forceinline__ u64 rel(const u64* base, u64 v) { return base ? ld_sys(base) + v : v; }

__global__ void k_signal(u64* flag, const u64* base, u64 v) {
    if (threadIdx.x == 0) st_sys(flag, rel(base, v));
}

// A wait of a call whose earlier wait already gave up returns at once: the
// stream then drains in microseconds instead of one deadline per remaining
// wait (a peer that stopped — e.g. its process exited on an error — would
// otherwise hold this stream, and the exit of this process, for deadline x
// the hundreds of waits a checked loop enqueues).
__global__ void k_wait(const u64* flag, const u64* base, u64 v, Status* st, u64 timeout_ticks) {
    if (threadIdx.x != 0) return;
    if (__hip_atomic_load(&st->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) return;
    const u64 want = rel(base, v);
    const u64 t0 = now_ticks();
    u64 spins = 0, seen;
    while ((seen = ld_sys(flag)) < want) {
        if ((++spins & 255) == 0 && now_ticks() - t0 > timeout_ticks) {
            st->seen = seen;   // diagnostics, read by the host after the stream drains
            st->want = want;
            __hip_atomic_store(&st->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// base[0..1] = {tx, rx} (add = 0), or base[0..1] += {tx, rx} (add = 1)
__global__ void k_seqbase(u64* base, u64 tx, u64 rx, int add) {
    if (threadIdx.x != 0) return;
    st_sys(base, add ? ld_sys(base) + tx : tx);
    st_sys(base + 1, add ? ld_sys(base + 1) + rx : rx);
}

// ---------------------------------------------------------------------------
// k_xfer: the transfer loop.  One launch runs all `iters` iterations of one
// rank's side; the peer runs its own launch on its own GPU at the same time.
// ---------------------------------------------------------------------------
// phase stamps of workgroup 0 (Loop::ts)
enum { kTsEntry = 0, kTsPosted = 1, kTsFirst = 2, kTsLoop = 3 };

template <int MODE>
struct Loop {
    const XferArgs& a;
    int* s_abort;      // LDS: this workgroup gave up
    u64* lds4;         // LDS scratch for block_sum
    v4u* s_tx;         // LDS: this workgroup's staged chunk of tx (a.stage)
    // LL payload of this side's sends, held in VGPRs for the whole launch:
    // pre[j] = tx bytes [8u, 8u+8) of unit u = threadIdx.x + j*kBlock.  tx is
    // read-only while the loop runs (the reference re-sends the same buffer
    // every iteration, mpi_perf.c:72,80,135), so a send is stores only — no
    // tx load on the latency path.
    u64 pre[kLLUnitsPerLane];
    u64* s_seen = nullptr;   // LDS, pull mode: the peer's ready word as last read
    // a.stage: s_tx holds this workgroup's chunk once the first push (which
    // reads tx from memory and fills s_tx on the way) is done
    mutable bool staged = false;
    mutable u64 ts[4] = {0, 0, 0, 0};   // workgroup 0's phase stamps (stamp)
    mutable u64 rdone = 0, rdig = 0;    // workgroup 0, thread 0: the call's receive
                                        // count and digest (finish_last writes them)

    __device__ void preload_ll(long long n) {
#pragma unroll
        for (int j = 0; j < kLLUnitsPerLane; ++j) {
            const long long off = 8ll * ((int)threadIdx.x + j * kBlock);
            u64 w = 0;
            if (off + 8 <= n) {
                w = *reinterpret_cast<const u64*>(a.tx + off);
            } else {
                for (long long b = 0; off + b < n; ++b) w |= (u64)a.tx[off + b] << (8 * b);
            }
            pre[j] = w;
        }
    }

    __device__ bool aborted() const { return *s_abort != 0; }

    // Record a timeout: LDS flag for this workgroup, device word for the
    // others (scratch[1]), host-mapped status for the host.
    __device__ void give_up(int iter) const {
        *s_abort = 1;
        __hip_atomic_store(&a.gbar[1], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&a.status->where, (unsigned)iter + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&a.status->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // every 64 spins: deadline or another workgroup's abort
    __device__ bool should_stop(u64 spins, u64 t0) const {
        if ((spins & 63) != 0) return false;
        if (*s_abort) return true;
        if (__hip_atomic_load(&a.gbar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return true;
        return now_ticks() - t0 > a.timeout_ticks;
    }

    __device__ bool is_ll(long long n) const { return MODE != MPX_MODE_NONBLOCKING && n <= a.ll_max; }

    // ---- send: push n bytes of tx[0:n) into the peer's rx -------------------
    // LL: one workgroup; every 16-B store carries two granules {payload:32,
    // tag:32} (each 8-B half lands untorn), so 8 payload bytes per store.
    __device__ void push_ll(long long n, u64 seq) const {
        if (blockIdx.x != 0) return;
        const int ng = n > 0 ? (int)((n + 3) >> 2) : 1;   // a 0-byte message is one empty granule
        const int nu = (ng + 1) >> 1;                      // 16-B units
        const unsigned tag = ll_tag(seq);
        const __amdgpu_buffer_rsrc_t dst = rsrc(&a.peer_mb->ll[a.my_slot][0], (unsigned)(nu * 16));
#pragma unroll
        for (int j = 0; j < kLLUnitsPerLane; ++j) {
            const int u = (int)threadIdx.x + j * kBlock;
            if (u < nu) {
                const v4u v = {(unsigned)pre[j], tag, (unsigned)(pre[j] >> 32), tag};
                __builtin_amdgcn_raw_buffer_store_b128(v, dst, (unsigned)u * 16, 0, kAuxSys);
            }
        }
    }

    // this workgroup's chunk [lo, hi) of a bulk push of n bytes
    __device__ void chunk_of(long long n, long long* lo, long long* hi) const {
        const long long chunk = (((n + a.nwg - 1) / a.nwg) + 15) & ~15ll;
        *lo = (long long)blockIdx.x * chunk;
        *hi = *lo + chunk < n ? *lo + chunk : n;
    }

    // LDS staging (a.stage): each pushing workgroup keeps its chunk's 16-B
    // units of tx in LDS for the whole launch; every push after the first
    // reads LDS (ds_read_b128) instead of HBM/L2, so the per-iteration
    // critical path is LDS -> remote store.  The first push reads tx from
    // memory and fills LDS on the way (STAGE below): no separate staging pass
    // stands between the start of the call and its first byte on the link.
    // tx is read-only while the loop runs.  Lane t handles units t, t+kBlock,
    // ... in every pass, so it reads back only LDS words it wrote itself.
    template <int AUX, bool STAGE>
    __device__ __forceinline__ void push_units(const v4u* src, __amdgpu_buffer_rsrc_t dst, int nv) const {
        int v = threadIdx.x;
        for (; v + 3 * kBlock < nv; v += 4 * kBlock) {
            const v4u r0 = src[v], r1 = src[v + kBlock], r2 = src[v + 2 * kBlock], r3 = src[v + 3 * kBlock];
            __builtin_amdgcn_raw_buffer_store_b128(r0, dst, v * 16, 0, AUX);
            __builtin_amdgcn_raw_buffer_store_b128(r1, dst, (v + kBlock) * 16, 0, AUX);
            __builtin_amdgcn_raw_buffer_store_b128(r2, dst, (v + 2 * kBlock) * 16, 0, AUX);
            __builtin_amdgcn_raw_buffer_store_b128(r3, dst, (v + 3 * kBlock) * 16, 0, AUX);
            if (STAGE) {
                s_tx[v] = r0;
                s_tx[v + kBlock] = r1;
                s_tx[v + 2 * kBlock] = r2;
                s_tx[v + 3 * kBlock] = r3;
            }
        }
        for (; v < nv; v += kBlock) {
            const v4u r = src[v];
            __builtin_amdgcn_raw_buffer_store_b128(r, dst, v * 16, 0, AUX);
            if (STAGE) s_tx[v] = r;
        }
    }
    template <bool STAGE>
    __device__ __forceinline__ void push_units_aux(const v4u* src, __amdgpu_buffer_rsrc_t dst, int nv) const {
        if (a.stream) push_units<kAuxSysNt, STAGE>(src, dst, nv);
        else push_units<kAuxSys, STAGE>(src, dst, nv);
    }

    // publish = false: the stores are issued but not drained and no flag is
    // stored (non-blocking mode publishes every a.nb_publish pushes, see k_xfer).
    // dst_base: the peer's receive slot (default: its rx).  skip (test knob
    // MPX_TEST_SKIP_PUSH): no payload stores, the flag is still published.
    __device__ void push_bulk(long long n, u64 seq, bool publish = true, unsigned char* dst_base = nullptr,
                              bool skip = false) const {
        const int w = blockIdx.x;
        if (w >= a.nwg) return;
        long long lo, hi;
        chunk_of(n, &lo, &hi);
        if (lo < hi) {
            const unsigned bytes = (unsigned)(hi - lo);
            const __amdgpu_buffer_rsrc_t dst = rsrc((dst_base ? dst_base : a.peer_rx) + lo, bytes);
            const int nv = (int)(bytes >> 4);
            const v4u* txv = reinterpret_cast<const v4u*>(a.tx + lo);
            if (a.stage && !staged) {
                if (!skip) {
                    push_units_aux<true>(txv, dst, nv);
                } else {
                    for (int v = threadIdx.x; v < nv; v += kBlock) s_tx[v] = txv[v];   // stage only
                }
            } else if (!skip) {
                push_units_aux<false>(a.stage ? s_tx : txv, dst, nv);
            }
            const unsigned tail = bytes & 15;
            if (threadIdx.x < tail && !skip) {
                const unsigned o = (unsigned)nv * 16 + threadIdx.x;
                __builtin_amdgcn_raw_buffer_store_b8(a.tx[lo + o], dst, o, 0, kAuxSys);
            }
        }
        staged = true;
        if (!publish) return;
        drain_stores();                 // every storing wave
        __syncthreads();
        if (threadIdx.x == 0) st_sys(&a.peer_mb->flag[a.my_slot][w], seq);
    }

    __device__ void send(long long n, u64 seq, bool skip = false) const {
        if (is_ll(n)) { if (!skip) push_ll(n, seq); else push_ll_tags_only(n, seq); }
        else push_bulk(n, seq, true, nullptr, skip);
    }

    // test knob: an LL message whose payload was "lost" — the tags arrive (so
    // the receiver completes), the data words carry a fixed wrong pattern
    __device__ void push_ll_tags_only(long long n, u64 seq) const {
        if (blockIdx.x != 0) return;
        const int ng = n > 0 ? (int)((n + 3) >> 2) : 1;
        const int nu = (ng + 1) >> 1;
        const unsigned tag = ll_tag(seq);
        const __amdgpu_buffer_rsrc_t dst = rsrc(&a.peer_mb->ll[a.my_slot][0], (unsigned)(nu * 16));
        for (int u = threadIdx.x; u < nu; u += kBlock) {
            const v4u v = {~0u, tag, ~0u, tag};
            __builtin_amdgcn_raw_buffer_store_b128(v, dst, (unsigned)u * 16, 0, kAuxSys);
        }
    }

    // ---- receive: wait until the peer's push `seq` of n bytes has landed ----
    // LL receive: every lane issues the loads of ALL its units (up to 4)
    // back to back, then checks the tags — one memory round trip per poll,
    // not one per unit.
    // One 16-B sc0|sc1 volatile load per unit, both granule tags checked
    // (the sender tags both halves of every unit).  Against the earlier 8-B
    // granule loads it halves the load count: 4 KiB ping-pong 4.32 -> 2.56 us
    // per iteration (profiles/r01_ll_ab.jsonl, r01_ll_preload_ab.jsonl).
    __device__ bool wait_ll(long long n, u64 seq, int iter) const {
        const int ng = n > 0 ? (int)((n + 3) >> 2) : 1;
        const int nu = (ng + 1) >> 1;
        const int mine = nu > (int)threadIdx.x ? (nu - (int)threadIdx.x + kBlock - 1) / kBlock : 0;
        const unsigned tag = ll_tag(seq);
        const __amdgpu_buffer_rsrc_t src = rsrc(&a.my_mb->ll[a.peer_slot][0], (unsigned)(nu * 16));
        v4u x[kLLUnitsPerLane];
        if (mine > 0) {
            const u64 t0 = now_ticks();
            u64 spins = 0;
            for (;;) {
#pragma unroll
                for (int j = 0; j < kLLUnitsPerLane; ++j)
                    if (j < mine)
                        x[j] = __builtin_amdgcn_raw_buffer_load_b128(src, ((unsigned)threadIdx.x + j * kBlock) * 16, 0,
                                                                     kAuxSysVol);
                bool ok = true;
#pragma unroll
                for (int j = 0; j < kLLUnitsPerLane; ++j)
                    if (j < mine) ok &= (x[j].y == tag) & (x[j].w == tag);
                if (ok) break;
                if (should_stop(++spins, t0)) { give_up(iter); break; }
                __builtin_amdgcn_s_sleep(0);
            }
            if (blockIdx.x == 0 && !*s_abort) {
                // write-through (sc0 sc1) like every other store into rx, so
                // the bytes are in memory once the call's completion word is
                const __amdgpu_buffer_rsrc_t rr = rsrc(a.rx, (unsigned)n);
#pragma unroll
                for (int j = 0; j < kLLUnitsPerLane; ++j) {
                    if (j >= mine) break;
                    const long long off = 8ll * ((int)threadIdx.x + j * kBlock);
                    const u64 d = ((u64)x[j].z << 32) | x[j].x;
                    if (off + 8 <= n) {
                        const unsigned lo = (unsigned)d, hi = (unsigned)(d >> 32);
                        __builtin_amdgcn_raw_buffer_store_b32(lo, rr, (unsigned)off, 0, kAuxSys);
                        __builtin_amdgcn_raw_buffer_store_b32(hi, rr, (unsigned)off + 4, 0, kAuxSys);
                    } else {
                        for (long long b = 0; off + b < n; ++b)
                            __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(d >> (8 * b)), rr, (unsigned)(off + b),
                                                                 0, kAuxSys);
                    }
                }
            }
        }
        __syncthreads();
        return !aborted();
    }

    __device__ bool wait_bulk(u64 seq, int iter) const {
        if (threadIdx.x < 64) {
            const u64* f = &a.my_mb->flag[a.peer_slot][0];
            const u64 t0 = now_ticks();
            u64 spins = 0;
            for (;;) {
                bool ok = true;
                for (int j = threadIdx.x; j < a.nwg; j += 64) ok &= ld_sys(f + j) >= seq;
                if (__all(ok)) break;
                if (should_stop(++spins, t0)) {
                    if (threadIdx.x == 0) give_up(iter);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
        return !aborted();
    }

    __device__ bool recv(long long n, u64 seq, int iter) const {
        return is_ll(n) ? wait_ll(n, seq, iter) : wait_bulk(seq, iter);
    }

    // ---- matched-receive order (Mailbox.posted) -----------------------------
    // This call's receives are posted: the peer may now push its call a.call
    // into this rank's rx / ring / LL zone.  The kernel is the first command
    // of the call on this rank's stream, so every workgroup of the previous
    // call has finished (checks, poison stores and all) and the host has
    // finished whatever it did with rx between the calls.
    __device__ void post_receives() const {
        if (blockIdx.x == 0 && threadIdx.x == 0) st_sys(&a.peer_mb->posted[a.my_slot], a.call);
    }
    __device__ bool peer_posted() const { return ld_sys(&a.my_mb->posted[a.peer_slot]) >= a.call; }
    // Before this side's first push of the call: wait for the peer's post.
    // Once per call, not per iteration.
    __device__ bool wait_posted() const {
        if (threadIdx.x == 0) {
            const u64 t0 = now_ticks();
            u64 spins = 0;
            while (!peer_posted()) {
                if (should_stop(++spins, t0)) { give_up(0); break; }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        stamp(kTsPosted);
        __syncthreads();
        return !aborted();
    }

    // ---- check mode: checksum the received payload, then poison it ----------
    // The poison guarantees the NEXT iteration's checksum only passes if the
    // next payload really overwrote every byte.
    // The last iteration is not poisoned: rx ends holding the last payload,
    // as the reference's rx does.
    __device__ void check(long long n, int iter) const {
        const u64 poison = 0x5a5a5a5a5a5a5a5aull ^ (u64)iter;
        const bool last = iter + 1 == a.iters;
        u64 acc = 0;
        if (is_ll(n)) {
            // unpacked by workgroup 0 with write-through stores: read back
            // the same way (sc0 sc1 loads: no L1 line of an earlier
            // iteration's read can serve them)
            if (blockIdx.x == 0) {
                const __amdgpu_buffer_rsrc_t rr = rsrc(a.rx, (unsigned)n);
                for (long long k = threadIdx.x; 8 * k < n; k += kBlock) {
                    const unsigned o = (unsigned)(8 * k);
                    u64 w = 0;
                    if (8 * k + 8 <= n) {
                        w = (u64)__builtin_amdgcn_raw_buffer_load_b32(rr, o, 0, kAuxSys) |
                            ((u64)__builtin_amdgcn_raw_buffer_load_b32(rr, o + 4, 0, kAuxSys) << 32);
                    } else {
                        for (long long b = 0; 8 * k + b < n; ++b)
                            w |= (u64)__builtin_amdgcn_raw_buffer_load_b8(rr, o + (unsigned)b, 0, kAuxSys) << (8 * b);
                    }
                    acc += csum_term(w, k);
                }
                __syncthreads();
                if (!last) {
                    for (long long o = threadIdx.x; o < n; o += kBlock)
                        __builtin_amdgcn_raw_buffer_store_b8((unsigned char)poison, rr, (unsigned)o, 0, kAuxSys);
                    drain_stores();   // the poison lands before the next payload's unpack
                }
            }
        } else if ((int)blockIdx.x < a.nwg) {
            acc = sum_chunk(a.rx, n, poison, last);
        }
        const u64 s = block_sum(acc, lds4);
        if (threadIdx.x == 0 && s) atomicAdd(&a.csum[iter], s);
    }

    // This workgroup's chunk of a bulk payload of n bytes at `base` that the
    // peer stored: system-scope acquire, sc0|sc1 loads, the lane's partial
    // checksum returned; then poison stores (write-through) unless `keep`,
    // drained before returning.
    __device__ u64 sum_chunk(unsigned char* base, long long n, u64 poison, bool keep) const {
        u64 acc = 0;
        if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        drain_stores();
        __syncthreads();
        long long lo, hi;
        chunk_of(n, &lo, &hi);
        if (lo < hi) {
            const unsigned bytes = (unsigned)(hi - lo);
            const __amdgpu_buffer_rsrc_t r = rsrc(base + lo, bytes);
            const int nv = (int)(bytes >> 4);
            const v4u pv = {(unsigned)poison, (unsigned)(poison >> 32), (unsigned)poison, (unsigned)(poison >> 32)};
            for (int v = threadIdx.x; v < nv; v += kBlock) {
                const v4u x = __builtin_amdgcn_raw_buffer_load_b128(r, v * 16, 0, kAuxSys);
                const u64 k = (u64)(lo / 8) + 2 * (u64)v;
                acc += csum_term(((u64)x.y << 32) | x.x, k);
                acc += csum_term(((u64)x.w << 32) | x.z, k + 1);
                if (!keep) __builtin_amdgcn_raw_buffer_store_b128(pv, r, v * 16, 0, kAuxSys);
            }
            const unsigned tail = bytes & 15;   // only the last workgroup
            if (threadIdx.x < 2 && 8 * threadIdx.x < tail) {
                const long long off = lo + (long long)nv * 16 + 8 * threadIdx.x;
                u64 w = 0;
                for (long long b = 0; b < 8 && off + b < n; ++b) {
                    const unsigned char c = __builtin_amdgcn_raw_buffer_load_b8(r, (unsigned)(off - lo + b), 0, kAuxSys);
                    w |= (u64)c << (8 * b);
                }
                acc += csum_term(w, (u64)off / 8);
            }
            __syncthreads();
            if (!keep && threadIdx.x < tail)
                __builtin_amdgcn_raw_buffer_store_b8((unsigned char)poison, r, (unsigned)nv * 16 + threadIdx.x, 0, kAuxSys);
        }
        drain_stores();
        return acc;
    }

    // ---- receive accounting ------------------------------------------------
    // Ping-pong / unidir: every receive is counted when it completes (a
    // blocking Recv).  At the end the last workgroup to finish (all chunk
    // checksums are in by then) adds up the finished checksums of the `done`
    // receives (check mode) and stores the count and digest.
    __device__ void account(u64 done, long long n_recv) const {
        u64 part = 0;
        if (a.check) {
            const u64 fmix = mix64((u64)n_recv);
            for (u64 j = threadIdx.x; j < done; j += kBlock)
                part += __hip_atomic_load(&a.csum[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ^ fmix;
        }
        const u64 s = a.check ? block_sum(part, lds4) : 0;
        if (threadIdx.x == 0) {
            rdone = done;
            rdig = s;
        }
    }

    // ---- armed calls (mpx_xfer_arm) ----------------------------------------
    // The kernel was launched before the host's barrier; the loop starts when
    // the host stores this call's token into Status.go (mpx_xfer_ex after the
    // barrier) — MPI's persistent-request split (MPI_Send_init ... MPI_Start).
    // Workgroup 0 polls the host word and hands its verdict to the others in
    // scratch word kScrGo.  False: cancelled (mpx_xfer_disarm) or no start
    // within go_timeout_ticks (then Status.err = 2): no transfer at all.
    // Every other workgroup counts itself in (kScrReady) when it starts to
    // wait; once all have, workgroup 0 stores the token into Status.ready —
    // the whole grid is resident and waiting — which mpx_xfer_arm waits for,
    // so a start right after the host's barrier does not also pay the rest of
    // the launch.
    __device__ bool wait_go() const {
        if (!a.go_token) return true;
        __shared__ int s_go;
        if (threadIdx.x == 0) {
            const u64 t0 = now_ticks();
            u64 spins = 0, w = 0;
            if (blockIdx.x == 0) {
                bool told = false;
                for (;;) {
                    if (!told && __hip_atomic_load(&a.gbar[kScrReady], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                                     (u64)gridDim.x - 1) {
                        st_sys(&a.status->ready, a.go_token);
                        told = true;
                    }
                    const u64 v = ld_sys(&a.status->go);
                    if (v == a.go_token) { w = 1; break; }
                    if (v == (a.go_token | kGoCancel)) { w = 2; break; }
                    if ((++spins & 63) == 0 && now_ticks() - t0 > a.go_timeout_ticks) {
                        __hip_atomic_store(&a.status->err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        w = 2;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                __hip_atomic_store(&a.gbar[kScrGo], w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                __hip_atomic_fetch_add(&a.gbar[kScrReady], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                // (workgroup 0 answers within its own deadline; one second
                // more bounds this wait should it never run)
                while ((w = __hip_atomic_load(&a.gbar[kScrGo], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0) {
                    if ((++spins & 63) == 0 && now_ticks() - t0 > a.go_timeout_ticks + 100000000ull) { w = 2; break; }
                    __builtin_amdgcn_s_sleep(2);
                }
            }
            s_go = (int)w;
        }
        __syncthreads();
        return s_go == 1;
    }

    // ---- call phases and the end of the call --------------------------------
    // Workgroup 0 stamps the call's start (Status.t_entry) as its first action
    // and, on a side that pushes first, the moment the peer's receives were
    // seen posted (t_posted): the host splits a call's wall time into launch,
    // wait for the peer, transfer and completion with them (mpx_last_phases).
    // The stamps stay in workgroup 0's registers (ts) until it ends the call
    // (finish_last): a store to host memory here would make the loop's next
    // drain wait for its PCIe round trip.
    __device__ void stamp(int k) const {
        if (blockIdx.x == 0 && threadIdx.x == 0) ts[k] = now_ticks();
    }
    // Every workgroup calls it last.  Workgroup 0 ends the call: the others
    // count themselves out (release) and exit; workgroup 0 waits until all
    // have (acquire) — they are done with the scratch words, the status
    // fields and their checksums by then — and returns true.  The others end
    // early where they can (the last receive of a side that only waits for
    // it, see k_xfer), so their count is usually in before workgroup 0 looks.
    __device__ bool last_to_finish() const {
        drain_stores();    // every wave: its stores of the call (rx unpacks, poison) are in memory
        __syncthreads();
        if (gridDim.x == 1) return true;   // (no counter round trip for a 1-workgroup grid)
        // What workgroup 0 needs from the others is in memory once their
        // waves have drained (above): their payload, poison and rx stores
        // are write-through (sc0 sc1) and their checksums atomics.  So the
        // count is a relaxed add after the drain — an agent-scope release
        // would add an L2 write-back (buffer_wbl2) with nothing to write —
        // and workgroup 0 polls it with relaxed loads and invalidates (one
        // acquire) once, not on every poll.
        if (blockIdx.x != 0) {
            if (threadIdx.x == 0)
                __hip_atomic_fetch_add(&a.gbar[kScrFin], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        if (threadIdx.x == 0) {
            while (__hip_atomic_load(&a.gbar[kScrFin], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != (u64)gridDim.x - 1)
                __builtin_amdgcn_s_sleep(1);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        __syncthreads();
        return true;
    }
    // Workgroup 0, last (every store of the call has drained: last_to_finish):
    // the call's end line (Status.fin: receive count and digest, phase stamps,
    // exit time, the sealed completion word) in ONE store of eight lanes of
    // wave 0, then scratch words [0..3] back to zero for the rank's next call
    // (so no memset precedes a launch; the next call's kernel starts only
    // after this one has retired).
    __device__ void finish_last() const {
        if (threadIdx.x >= 64) return;
        const u64 t_end = now_ticks();
        const u64 v0 = __shfl(rdone, 0, 64), v1 = __shfl(rdig, 0, 64), v2 = __shfl(ts[kTsEntry], 0, 64),
                  v3 = __shfl(ts[kTsPosted], 0, 64), v4 = __shfl(ts[kTsFirst], 0, 64), v5 = __shfl(ts[kTsLoop], 0, 64),
                  v6 = __shfl(t_end, 0, 64);
        const u64 w = fin_word(a.done_token, v0, v1, v2, v3, v4, v5, v6);
        const int l = (int)threadIdx.x;
        const u64 mine = l == 0 ? v0 : l == 1 ? v1 : l == 2 ? v2 : l == 3 ? v3 : l == 4 ? v4 : l == 5 ? v5
                                                                                         : l == 6 ? v6 : w;
        if (l < 8) st_sys(&a.status->fin.recv_done + l, mine);
        if (l == 0) {
            for (int k = 0; k < 4; ++k) __hip_atomic_store(&a.gbar[k], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&a.gbar[kScrGo], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&a.gbar[kScrReady], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }

    // ---- non-blocking check mode (k_xfer_nbcheck) ----------------------------
    // receive slot j of the rank whose rx / ring these are (ring_slot)
    __device__ unsigned char* slot_base(unsigned char* rx0, unsigned char* ring0, int j) const {
        const int s = ring_slot(j, a.iters, a.slots);
        return s == 0 ? rx0 : ring0 + (long long)(s - 1) * a.len;
    }

    // Check this workgroup's chunk of receive j: checksum + poison its slot
    // (the last receive stays in rx unpoisoned), add the chunk sum into
    // csum[j], count the chunk in cnt[j], then hand the slot back to the
    // sender (credit) — after the poison stores drained, so none can land on
    // the next payload.
    __device__ void check_nb(int j) const {
        const long long n = a.len;
        if (a.lag_ticks && (int)blockIdx.x == a.lag_wg && j + 1 == a.iters) {
            // test knob (MPX_TEST_LAG_WG): this workgroup is late to check the
            // call's last receive, so the call ends well after the peer's
            if (threadIdx.x == 0) {
                const u64 t0 = now_ticks();
                while (now_ticks() - t0 < a.lag_ticks) __builtin_amdgcn_s_sleep(127);
            }
            __syncthreads();
        }
        const u64 poison = 0x5a5a5a5a5a5a5a5aull ^ (u64)j;
        const u64 acc = sum_chunk(slot_base(a.rx, a.ring, j), n, poison, j + 1 == a.iters);
        const u64 s = block_sum(acc, lds4);
        if (threadIdx.x == 0) {
            if (s) atomicAdd(&a.csum[j], s);
            __hip_atomic_fetch_add(&a.cnt[j], 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            st_sys(&a.peer_mb->credit[a.my_slot][blockIdx.x], a.rx_seq0 + (u64)j + 1);
        }
    }

    // Wait until ready() holds (evaluated by every lane, all must agree),
    // checking — in order — every receive of this workgroup's chunk that
    // lands meanwhile.  Both sides do this whenever they wait, so a sender
    // waiting for a free slot never starves the receiver that must free it.
    template <class Ready>
    __device__ bool nb_wait(Ready ready, int* next, int iter) const {
        u64 t0 = now_ticks(), spins = 0;
        for (;;) {
            if (__syncthreads_and(ready())) return true;
            const bool landed = __syncthreads_or(
                threadIdx.x == 0 && *next < a.iters &&
                ld_sys(&a.my_mb->flag[a.peer_slot][blockIdx.x]) >= a.rx_seq0 + (u64)*next + 1);
            if (landed) {
                check_nb(*next);
                ++*next;
                t0 = now_ticks();
                continue;
            }
            if (__syncthreads_or(threadIdx.x == 0 && should_stop(++spins, t0))) {
                if (threadIdx.x == 0) give_up(iter);
                __syncthreads();
                return false;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }

    // Waitall over receives [lo, hi) (workgroup 0): each is complete once
    // every workgroup has checked its chunk; count them and add their
    // finished checksums into the digest (thread 0's registers).
    __device__ bool nb_waitall(int lo, int hi, u64* done, u64* dig, u64 fmix, int* next, int iter) const {
        const u64 want = (u64)a.nwg;
        const bool ok = nb_wait(
            [&] {
                bool r = true;
                for (int j = lo + (int)threadIdx.x; j < hi; j += kBlock)
                    r &= __hip_atomic_load(&a.cnt[j], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >= want;
                return r;
            },
            next, iter);
        if (!ok) return false;
        u64 part = 0;
        for (int j = lo + (int)threadIdx.x; j < hi; j += kBlock)
            part += __hip_atomic_load(&a.csum[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ^ fmix;
        const u64 s = block_sum(part, lds4);
        *done += (u64)(hi - lo);
        *dig += s;
        return true;
    }

    // all workgroups finished check(): the 1-WG ack must not overtake a poison
    __device__ bool grid_sync(int iter) const {
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_fetch_add(&a.gbar[0], 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            if (blockIdx.x == 0) {
                const u64 want = (u64)gridDim.x * (u64)(iter + 1);
                const u64 t0 = now_ticks();
                u64 spins = 0;
                while (__hip_atomic_load(&a.gbar[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
                    if (should_stop(++spins, t0)) { give_up(iter); break; }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
        }
        __syncthreads();
        return !aborted();
    }

    // ---- pull mode (k_xfer_pull) ---------------------------------------------
    // Bounded one-lane poll of a word this rank's workgroup reads; `sys` =
    // a word the peer writes (system scope), else a device-local counter.
    template <bool SYS>
    __device__ bool poll_ge(const u64* p, u64 want, int iter) const {
        if (threadIdx.x == 0) {
            const u64 t0 = now_ticks();
            u64 spins = 0;
            for (;;) {
                const u64 v = SYS ? ld_sys(p) : __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                if (v >= want) break;
                if (should_stop(++spins, t0)) { give_up(iter); break; }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
        return !aborted();
    }

    // Send (workgroup 0): tx holds push `seq` — one system-scope store into
    // the peer's ready word.  tx is read-only while the loop runs and the
    // reference re-sends the same buffer every iteration (mpi_perf.c:74,80,
    // 99,105,136), so no byte moves here.  `landed` > 0: first wait until
    // that many chunks of this call's receives are in rx (a blocking Recv
    // completes before the next Send, mpi_perf.c:75-80).
    __device__ bool pull_send(u64 seq, u64 landed, int iter) const {
        if (blockIdx.x != 0) return true;
        if (landed && !poll_ge<false>(&a.gbar[kScrLanded], landed, iter)) return false;
        if (threadIdx.x == 0) st_sys(&a.peer_mb->ready[a.my_slot], seq);
        return true;
    }

    // This workgroup's chunk of a pull: units from the peer's tx into rx, 8
    // loads in flight per lane.  Loads are sc0|sc1 (system scope: each
    // iteration's bytes come from the peer's memory, not from a line this
    // GPU cached in an earlier iteration or call); stores are sc0|sc1
    // write-through, as a push lands, so check mode and the host read what
    // arrived.  Units past the chunk are out of the resources' range (loads
    // return 0, stores are dropped), so the loop has no per-unit branch.
    __device__ void pull_units(__amdgpu_buffer_rsrc_t src, __amdgpu_buffer_rsrc_t dst, int nv) const {
        constexpr int D = 8;
        for (int v = threadIdx.x; v < nv; v += D * kBlock) {
            v4u r[D];
#pragma unroll
            for (int j = 0; j < D; ++j)
                r[j] = __builtin_amdgcn_raw_buffer_load_b128(src, (unsigned)(v + j * kBlock) * 16, 0, kAuxSys);
#pragma unroll
            for (int j = 0; j < D; ++j)
                __builtin_amdgcn_raw_buffer_store_b128(r[j], dst, (unsigned)(v + j * kBlock) * 16, 0, kAuxSys);
        }
    }

    // Wait until the peer's ready word covers push `seq`.  The value last
    // read is kept in LDS (s_seen): one read that shows a later push covers
    // every push up to it, so the word is polled only when behind.
    __device__ bool wait_ready(u64 seq, int iter) const {
        if (threadIdx.x == 0 && *s_seen < seq) {
            const u64* p = &a.my_mb->ready[a.peer_slot];
            const u64 t0 = now_ticks();
            u64 spins = 0;
            for (;;) {
                const u64 v = ld_sys(p);
                if (v >= seq) { *s_seen = v; break; }
                if (should_stop(++spins, t0)) { give_up(iter); break; }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
        return !aborted();
    }

    // Receive (every workgroup, grid = nwg): wait for the peer's ready word,
    // load this workgroup's chunk of the peer's tx into rx, check it (check
    // mode).  `publish` > 0: then drain, return the chunk to the peer (credit
    // = seq: its tx chunk may change again, for every push up to seq) and
    // count `publish` receives of this workgroup landed.  The non-blocking
    // loop publishes every nb_publish receives (and at the last): the others
    // are loads and stores only, with no drain between them.
    __device__ bool pull_recv(long long n, u64 seq, int iter, u64 publish = 1) const {
        if (!wait_ready(seq, iter)) return false;
        // system-scope acquire (buffer_inv sc0 sc1: the L2's lines of
        // non-local memory, i.e. a peer GPU's tx, are dropped, so every
        // iteration's loads cross the link), completed before any wave loads
        // (every wave drains; draining only the fencing wave read the same:
        // profiles/r03_pull_publish_ab.jsonl)
        if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        drain_stores();
        __syncthreads();
        if (a.lag_ticks && (int)blockIdx.x == a.lag_wg && iter + 1 == a.iters) {
            // test knob (MPX_TEST_LAG_WG): this workgroup is late to load the
            // call's last payload, so the peer's call must wait for it
            if (threadIdx.x == 0) {
                const u64 t0 = now_ticks();
                while (now_ticks() - t0 < a.lag_ticks) __builtin_amdgcn_s_sleep(127);
            }
            __syncthreads();
        }
        long long lo, hi;
        chunk_of(n, &lo, &hi);
        if (lo < hi) {
            const unsigned bytes = (unsigned)(hi - lo);
            const __amdgpu_buffer_rsrc_t src = rsrc(a.peer_tx + lo, bytes);
            const __amdgpu_buffer_rsrc_t dst = rsrc(a.rx + lo, bytes);
            const int nv = (int)(bytes >> 4);
            if (a.skip_push != iter + 1) {             // test knob: this payload is "lost"
                pull_units(src, dst, nv);
                const unsigned tail = bytes & 15;
                if (threadIdx.x < tail) {
                    const unsigned o = (unsigned)nv * 16 + threadIdx.x;
                    __builtin_amdgcn_raw_buffer_store_b8(__builtin_amdgcn_raw_buffer_load_b8(src, o, 0, kAuxSys), dst, o,
                                                         0, kAuxSys);
                }
            }
        }
        if (a.check) check(n, iter);                   // (drains first: sum_chunk)
        if (!publish) return true;
        drain_stores();                                // loads and stores of every wave
        __syncthreads();
        if (threadIdx.x == 0) {
            st_sys(&a.peer_mb->credit[a.my_slot][blockIdx.x], seq);
            __hip_atomic_fetch_add(&a.gbar[kScrLanded], publish, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
        return true;
    }

    // Workgroup 0: every chunk of this side's sends up to `seq` was loaded
    // by the peer (its credits), so tx may change once the call returns —
    // MPI_Send's buffer-reuse rule, and the non-blocking loop's Waitall over
    // the send requests (mpi_perf.c:110,122).
    __device__ bool wait_pulled(u64 seq, int iter) const {
        if (blockIdx.x != 0) return true;
        if (threadIdx.x < 64) {
            const u64* c = &a.my_mb->credit[a.peer_slot][0];
            const u64 t0 = now_ticks();
            u64 spins = 0;
            for (;;) {
                bool ok = true;
                for (int j = threadIdx.x; j < a.nwg; j += 64) ok &= ld_sys(c + j) >= seq;
                if (__all(ok)) break;
                if (should_stop(++spins, t0)) {
                    if (threadIdx.x == 0) give_up(iter);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
        return !aborted();
    }
};

// One instantiation per (mode, side): each carries only its own loop, so
// register pressure stays within 4 waves per SIMD (<= 128 VGPRs, no spills)
// and four k_xfer workgroups fit on a CU — pairs that share one GPU
// (loopback ranks, -g maps) keep every workgroup resident.
template <int MODE, int GROUP>
__global__ __launch_bounds__(kBlock, 4) void k_xfer(XferArgs a) {
    __shared__ int s_abort;
    __shared__ u64 lds4[4];
    extern __shared__ v4u s_tx[];            // a.stage: dynamic LDS = one chunk
    if (threadIdx.x == 0) s_abort = 0;
    Loop<MODE> L{a, &s_abort, lds4, s_tx, {}};
    if (!L.wait_go()) {
        if (L.last_to_finish()) L.finish_last();
        return;
    }
    L.stamp(kTsEntry);
    const long long n = a.len;
    // the size this side sends: B, or the 1-byte ack of unidir group 0
    const long long send_len = (MODE == MPX_MODE_UNIDIR && GROUP == 0) ? 1 : n;
    const bool ll_send = blockIdx.x == 0 && L.is_ll(send_len);
    if (ll_send) L.preload_ll(send_len);
    u64 txs = a.tx_seq0, rxs = a.rx_seq0;
    u64 done = 0;                                       // receives completed (Status.recv_done)
    int inflight = 0;
    L.post_receives();
    // A side whose first action is a push waits for the peer's post.  Group 0
    // of ping-pong / unidir pushes only after its first receive, which the
    // peer sent after it saw this side's post, so its peer has started too.
    constexpr bool push_first = MODE == MPX_MODE_NONBLOCKING || GROUP == 1;
    const bool go = !push_first || a.iters == 0 || L.wait_posted();
    // Group 1's last receive (ping-pong, unidir) without check mode: only
    // workgroup 0 waits for it (it counts receives and ends the call); the
    // others have nothing left to do once their last push is out, so they
    // leave, and their finish count is in before workgroup 0 needs it.
    const bool last_recv_wg0 = !a.check && blockIdx.x != 0;
    for (int i = 0; go && i < a.iters; ++i) {
        const bool skip = a.skip_push == i + 1;        // test knob only
        if constexpr (MODE == MPX_MODE_PINGPONG) {    // mpi_perf.c:70-82
            if constexpr (GROUP == 1) {
                L.send(n, ++txs, skip);                // Send(tx, B, tag 1)
                if (i + 1 == a.iters && last_recv_wg0) break;
                if (!L.recv(n, ++rxs, i)) break;       // Recv(rx, B, tag 2)
                ++done;
                if (a.check) L.check(n, i);
            } else {
                if (!L.recv(n, ++rxs, i)) break;       // Recv(rx, B, tag 1)
                ++done;
                if (a.check) L.check(n, i);
                L.send(n, ++txs, skip);                // Send(tx, B, tag 2)
            }
            if (i == 0) L.stamp(kTsFirst);
        } else if constexpr (MODE == MPX_MODE_UNIDIR) {  // mpi_perf.c:132-144
            if constexpr (GROUP == 1) {
                L.send(n, ++txs, skip);                // Send(tx, B)
                if (i + 1 == a.iters && last_recv_wg0) break;
                if (!L.recv(1, ++rxs, i)) break;       // Recv(rx, 1) — the ack
                ++done;
                if (a.check) L.check(1, i);
            } else {
                if (!L.recv(n, ++rxs, i)) break;       // Recv(rx, B)
                ++done;
                if (a.check) { L.check(n, i); if (!L.grid_sync(i)) break; }
                L.send(1, ++txs, skip);                // Send(tx, 1)
            }
            if (i == 0) L.stamp(kTsFirst);
        } else {                                       // mpi_perf.c:95-124
            // Isend + Irecv, slot `inflight`.  A receiver waits only at the
            // window flush (i = 255 mod 256) and at the end, so a push needs
            // its drain + flag only every a.nb_publish iterations (a divisor
            // of 256), at slot 254 (the last receive a flush waits for) and
            // at the last one: the drain's link round trip is paid once per
            // nb_publish pushes instead of once per push, and no flush waits
            // for the slot-255 push the reference leaves pending.
            const int slot = i % kNbWindow;
            L.push_bulk(n, ++txs, (i + 1) % a.nb_publish == 0 || slot == kNbWindow - 2 || i + 1 == a.iters,
                        nullptr, skip);
            if (inflight == kNbWindow - 1) {
                // Waitall(255, ...): receives of slots 0..254 (iterations
                // i-255 .. i-1); the receive posted in slot 255 (this
                // iteration) is not among them (mpi_perf.c:110-111)
                if (!L.wait_bulk(rxs + i, i)) break;
                done += (u64)inflight;
                inflight = 0;
            } else {
                ++inflight;
            }
        }
    }
    L.stamp(kTsLoop);
    if constexpr (MODE == MPX_MODE_NONBLOCKING) {
        if (inflight > 0 && !L.aborted() && L.wait_bulk(rxs + a.iters, a.iters - 1))   // final Waitall(inflight)
            done += (u64)inflight;
        if (blockIdx.x == 0 && threadIdx.x == 0) L.rdone = done;
        if (L.last_to_finish()) L.finish_last();
    } else if (L.last_to_finish()) {
        L.account(done, (MODE == MPX_MODE_UNIDIR && GROUP == 1) ? 1 : n);
        L.finish_last();
    }
}

// The non-blocking loop in check mode (mpi_perf.c:95-124 with every payload
// checksummed).  The reference posts up to 256 receives into ONE rx
// (:100,104); here every receive lands in a slot of its own (ring_slot), so
// each payload can be checksummed before anything overwrites it.  A sender
// reuses a slot only after the receiver handed it back (Mailbox.credit);
// every wait checks the receives that land meanwhile, so neither side can
// starve the other.  Each workgroup pushes and checks its own chunk.  The
// windowing is the reference's: Waitall(255) at slot 255 over slots 0..254,
// the final Waitall(inflight); workgroup 0 counts exactly those receives and
// digests their checksums.  The receives the reference leaves pending (slot
// 255 of each full window) are still checked — every payload is — but not
// counted.  Grid = a.nwg; all workgroups push B bytes.
__global__ __launch_bounds__(kBlock, 4) void k_xfer_nbcheck(XferArgs a) {
    __shared__ int s_abort;
    __shared__ u64 lds4[4];
    extern __shared__ v4u s_tx[];
    if (threadIdx.x == 0) s_abort = 0;
    Loop<MPX_MODE_NONBLOCKING> L{a, &s_abort, lds4, s_tx, {}};
    if (!L.wait_go()) {
        if (L.last_to_finish()) L.finish_last();
        return;
    }
    L.stamp(kTsEntry);
    const long long n = a.len;
    const int w = blockIdx.x;
    const u64 fmix = mix64((u64)n);
    const u64* credit = &a.my_mb->credit[a.peer_slot][w];
    int next = 0, inflight = 0;
    u64 done = 0, dig = 0;
    // The peer's receive slots are free for this call only once the peer's
    // kernel of this call runs (Mailbox.posted): its previous kernel — every
    // workgroup's checks and poison stores of the previous call, whatever
    // that call's length, width and slot layout — has finished by then.
    // Credits alone cannot say so: they are per workgroup, and the previous
    // call's last credits already satisfy this call's first S pushes.
    L.post_receives();
    bool ok = a.iters == 0 || L.nb_wait([&] { return threadIdx.x != 0 || L.peer_posted(); }, &next, 0);
    L.stamp(kTsPosted);
    for (int i = 0; i < a.iters && ok; ++i) {
        // slot ring_slot(i) was last used by push i - S of this call: wait
        // for its credit
        if (i >= a.slots) {
            const u64 want = a.tx_seq0 + (u64)(i - a.slots + 1);
            ok = L.nb_wait([&] { return threadIdx.x != 0 || ld_sys(credit) >= want; }, &next, i);
            if (!ok) break;
        }
        L.push_bulk(n, a.tx_seq0 + (u64)i + 1, true, L.slot_base(a.peer_rx, a.peer_ring, i), a.skip_push == i + 1);
        if (inflight == kNbWindow - 1) {               // Waitall(255): iterations i-255 .. i-1
            ok = L.nb_wait([&] { return next >= i; }, &next, i);
            if (ok && w == 0) ok = L.nb_waitall(i - inflight, i, &done, &dig, fmix, &next, i);
            inflight = 0;
        } else {
            ++inflight;
        }
    }
    if (ok && inflight > 0) {                          // Waitall(inflight)
        ok = L.nb_wait([&] { return next >= a.iters; }, &next, a.iters - 1);
        if (ok && w == 0) ok = L.nb_waitall(a.iters - inflight, a.iters, &done, &dig, fmix, &next, a.iters - 1);
    }
    // every payload: also the receives the reference leaves pending
    if (ok) L.nb_wait([&] { return next >= a.iters; }, &next, a.iters - 1);
    if (w == 0 && threadIdx.x == 0) {
        L.rdone = done;
        L.rdig = dig;
    }
    if (L.last_to_finish()) L.finish_last();
}

// k_xfer_pull: the three loops with every B-byte payload PULLED by its
// receiver (MPX_XFER_PULL; SURVEY.md §7 step 4, "try pull as well").  A send
// is one store into the peer's ready word (Loop::pull_send); the receiver's
// workgroups load their chunks of the sender's tx over xGMI into their own rx
// (Loop::pull_recv).  A receive is complete once every workgroup's chunk
// is in (the local landed counter); the sender's tx is free again once every
// chunk's credit came back, which each sending side waits for before its
// kernel ends.  rx is only ever written by its own rank's kernel, so no
// payload of the next call can land before this rank's next call starts.
// LL messages stay pushes (their data is their flag), and so does the
// unidir 1-byte ack (mpi_perf.c:137,142).  Grid: nwg for a side that
// receives B-byte payloads, 1 for unidir group 1 (it only publishes and
// takes acks).
template <int MODE, int GROUP>
__global__ __launch_bounds__(kBlock, 4) void k_xfer_pull(XferArgs a) {
    __shared__ int s_abort;
    __shared__ u64 lds4[4];
    __shared__ u64 s_seen;
    if (threadIdx.x == 0) {
        s_abort = 0;
        s_seen = 0;
    }
    Loop<MODE> L{a, &s_abort, lds4, nullptr, {}, &s_seen};
    if (!L.wait_go()) {
        if (L.last_to_finish()) L.finish_last();
        return;
    }
    L.stamp(kTsEntry);
    const long long n = a.len;
    const u64 nw = (u64)a.nwg;
    if (MODE == MPX_MODE_UNIDIR && GROUP == 0 && blockIdx.x == 0) L.preload_ll(1);   // the ack's byte
    __syncthreads();
    u64 txs = a.tx_seq0, rxs = a.rx_seq0, done = 0, pending = 0;
    L.post_receives();
    bool ok = true;
    int inflight = 0;
    for (int i = 0; ok && i < a.iters; ++i) {
        if constexpr (MODE == MPX_MODE_PINGPONG) {    // mpi_perf.c:70-82
            if constexpr (GROUP == 1) {
                ok = L.pull_send(++txs, nw * (u64)i, i) && L.pull_recv(n, ++rxs, i);   // Send(tag 1), Recv(tag 2)
            } else {
                ok = L.pull_recv(n, ++rxs, i) && L.pull_send(++txs, nw * (u64)(i + 1), i);   // Recv(tag 1), Send(tag 2)
            }
            if (ok) ++done;
        } else if constexpr (MODE == MPX_MODE_UNIDIR) {  // mpi_perf.c:132-144
            if constexpr (GROUP == 1) {
                ok = L.pull_send(++txs, 0, i) && L.recv(1, ++rxs, i);   // Send(tx, B), Recv(rx, 1)
                if (ok) {
                    ++done;
                    if (a.check) L.check(1, i);
                }
            } else {
                ok = L.pull_recv(n, ++rxs, i);           // Recv(rx, B)
                if (ok) ++done;
                // Send(tx, 1) once every chunk is in (workgroup 0's LL push)
                if (ok && blockIdx.x == 0) ok = L.template poll_ge<false>(&a.gbar[kScrLanded], nw * (u64)(i + 1), i);
                if (ok) L.send(1, ++txs);
            }
        } else {                                       // mpi_perf.c:95-124
            // Isend + Irecv, slot `inflight`; the receive is published (drain,
            // credit, landed count) every nb_publish receives and at the last
            // one — kNbWindow is a multiple of nb_publish, so slot 255 (the
            // flush) is always a publish point
            ++pending;
            const bool pub = (i + 1) % a.nb_publish == 0 || i + 1 == a.iters;
            ok = L.pull_send(++txs, 0, i) && L.pull_recv(n, ++rxs, i, pub ? pending : 0);
            if (pub) pending = 0;
            if (ok && inflight == kNbWindow - 1) {
                // Waitall(255): every workgroup waits until all chunks of
                // receives 0..i are in (so none runs into the next window
                // ahead of the count), workgroup 0 for the peer's loads of
                // sends 0..254 (iterations i-255 .. i-1)
                ok = L.template poll_ge<false>(&a.gbar[kScrLanded], nw * (u64)(i + 1), i) && L.wait_pulled(txs - 1, i);
                done += (u64)inflight;
                inflight = 0;
            } else {
                ++inflight;
            }
        }
    }
    // every send of the call loaded by the peer before tx may change again
    const bool sent_bulk = MODE != MPX_MODE_UNIDIR || GROUP == 1;
    if (ok && sent_bulk && a.iters > 0 && !a.no_pull_wait) ok = L.wait_pulled(txs, a.iters - 1);
    if constexpr (MODE == MPX_MODE_NONBLOCKING) {
        // final Waitall(inflight); then workgroup 0 counts and digests the
        // receives the reference waits for (all but slot 255 of each full
        // window)
        if (blockIdx.x == 0) {
            if (ok && a.iters > 0) ok = L.template poll_ge<false>(&a.gbar[kScrLanded], nw * (u64)a.iters, a.iters - 1);
            if (ok) done += (u64)inflight;
            u64 part = 0;
            if (ok && a.check) {
                const u64 fmix = mix64((u64)n);
                for (int j = threadIdx.x; j < a.iters; j += kBlock)
                    if (j % kNbWindow != kNbWindow - 1)
                        part += __hip_atomic_load(&a.csum[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ^ fmix;
            }
            const u64 s = block_sum(part, lds4);
            if (threadIdx.x == 0) {
                L.rdone = done;
                L.rdig = s;
            }
        }
        if (L.last_to_finish()) L.finish_last();
    } else if (L.last_to_finish()) {
        L.account(done, (MODE == MPX_MODE_UNIDIR && GROUP == 1) ? 1 : n);
        L.finish_last();
    }
}

// stream engines' receive accounting (launch_account)
__global__ __launch_bounds__(kBlock) void k_account(Status* st, const u64* csum, int j0, int count, u64 fmix) {
    __shared__ u64 lds4[4];
    u64 part = 0;
    if (csum)
        for (int j = threadIdx.x; j < count; j += kBlock) part += csum[j0 + j] ^ fmix;
    const u64 s = block_sum(part, lds4);
    if (threadIdx.x == 0) {
        const u64 d = __hip_atomic_load(&st->recv_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const u64 g = __hip_atomic_load(&st->recv_digest, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&st->recv_done, d + (u64)count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&st->recv_digest, g + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
hipError_t launch_xfer(const XferArgs& a, int grid, hipStream_t s) {
    (void)hipGetLastError();   // drop a stale error of an earlier, ignored call
    void (*k)(XferArgs) = nullptr;
    if (a.pull) {
        switch (a.mode) {
            case MPX_MODE_PINGPONG: k = a.group ? k_xfer_pull<MPX_MODE_PINGPONG, 1> : k_xfer_pull<MPX_MODE_PINGPONG, 0>; break;
            case MPX_MODE_UNIDIR: k = a.group ? k_xfer_pull<MPX_MODE_UNIDIR, 1> : k_xfer_pull<MPX_MODE_UNIDIR, 0>; break;
            case MPX_MODE_NONBLOCKING: k = k_xfer_pull<MPX_MODE_NONBLOCKING, 0>; break;   // both sides alike
            default: return hipErrorInvalidValue;
        }
        hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), 0, s, a);
        return hipGetLastError();
    }
    switch (a.mode) {
        case MPX_MODE_PINGPONG: k = a.group ? k_xfer<MPX_MODE_PINGPONG, 1> : k_xfer<MPX_MODE_PINGPONG, 0>; break;
        case MPX_MODE_UNIDIR: k = a.group ? k_xfer<MPX_MODE_UNIDIR, 1> : k_xfer<MPX_MODE_UNIDIR, 0>; break;
        case MPX_MODE_NONBLOCKING:   // both sides alike
            k = a.check ? k_xfer_nbcheck : k_xfer<MPX_MODE_NONBLOCKING, 0>;
            break;
        default: return hipErrorInvalidValue;
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), (unsigned)a.stage, s, a);
    return hipGetLastError();
}

// One k_copy form, from the tuning sweeps (DESIGN.md "k_copy tuning"): ONE
// 16-B unit per lane and ONE step per block — grid = n/4 KiB workgroups of
// 256 lanes, no cap, nontemporal loads and stores.  6.51-6.53 TB/s of HBM
// traffic at 256 MiB, 1 GiB and 4 GiB alike (profiles/r01_copy_lab_onestep.jsonl),
// against 6.0 / 5.45 TB/s for the earlier contiguous-chunk form and 4.76 TB/s
// for hipMemcpyAsync device-to-device.  The 39 other instantiations of round
// 1-3's variant knob (unroll x load/store policy x layout) are gone; their
// evidence stays in profiles/copy_sweep_r01.jsonl and r01_copy_policy_*.
hipError_t launch_copy(void* dst, const void* src, size_t n, hipStream_t s, int* grid_out) {
    const size_t n16 = n / 16;
    const unsigned tail = (unsigned)(n & 15);
    size_t grid = (n16 + (size_t)kBlock - 1) / (size_t)kBlock;
    if (grid < 1) grid = 1;
    if (grid > ((size_t)1 << 31) - 1) return hipErrorInvalidValue;
    if (grid_out) *grid_out = (int)grid;
    (void)hipGetLastError();   // drop a stale error of an earlier, ignored call
    hipLaunchKernelGGL((k_copy<1, true, true, false>), dim3((unsigned)grid), dim3(kBlock), 0, s,
                       reinterpret_cast<const v4u*>(src), reinterpret_cast<v4u*>(dst), n16, tail);
    return hipGetLastError();
}

hipError_t launch_copy_steps(void* dst, const void* src, size_t n, int iters, u64* bar, hipStream_t s,
                             int* grid_out, const int* shape) {
    // Defaults from the A/Bs: at most 64 workgroups and one hot counter
    // (fewer arrivals beat more lanes: 1 MiB 2.08 us vs 2.40 with 256,
    // profiles/r02_copy_steps_variants.jsonl); no store drain before arrival
    // (the barrier orders issue, not acknowledgement: -0.05..0.1 us per step).
    // Workgroups of 1024 lanes, one unit per lane: 16 KiB per workgroup per
    // step, so up to 16 KiB a copy is ONE workgroup and its steps need no
    // grid barrier (__syncthreads ends a step), and up to 1 MiB at most 64
    // workgroups arrive at the barrier.  Against the 256-lane grid sized for
    // 1-8 units per lane: 8 KiB 0.96 -> 0.62 us per copy, 16 KiB 0.99 ->
    // 0.70, 32-64 KiB 1.29-1.34 -> 1.12-1.15, 256-512 KiB 1.71-1.86 ->
    // 1.48-1.67, 128 KiB and 1 MiB unchanged; one wide workgroup with more
    // units per lane loses from 32 KiB (one CU's bandwidth)
    // (profiles/r02_copy_steps_wgsize.jsonl).  Above 1 MiB (only when
    // MPX_COPY_STEPS_MAX raises the switch) the 64 workgroups are 256 lanes
    // with 8 units per lane, all loads of a step in flight at once: 2 MiB
    // 2.35 us against 2.56-3.07 with 1024 lanes x 2
    // (r02_copy_steps_wgsize_mid.jsonl, r02_copy_sweep_state.jsonl).
    // `shape` (tests only: MPX_COPY="steps:..." via mpx_copy) overrides
    // {grid_cap, xcd, drain, upl, threads, one_xcd}.
    // Default-policy loads instead of nontemporal ones change nothing here,
    // fresh or after 1 GiB copies evicted src (r02_copy_steps_ldpolicy.jsonl,
    // measured with a knob since removed).
    // One XCD: from 32 KiB to 512 KiB every working workgroup sits on XCD 0
    // (8x the grid, the others exit at once), so the barrier's arrivals stay
    // within one XCD: 32-64 KiB 1.16-1.20 -> 1.02 us per copy (512 lanes),
    // 128 KiB 1.42 -> 1.12, 256 KiB 1.49 -> 1.25, 512 KiB 1.66 -> 1.53
    // (1024 lanes); at 1 MiB XCD 0's 32 CUs are too few (2.12 vs 1.98)
    // (profiles/r02_copy_steps_onexcd.jsonl).
    int cap = 64, xcd = 0, drain = 0, threads = 1024, upl = 1, one_xcd = 0;
    if (n > ((size_t)16 << 10) && n <= ((size_t)512 << 10)) {
        one_xcd = 1;
        threads = n <= ((size_t)128 << 10) ? 512 : 1024;
    } else if (n > ((size_t)1 << 20)) {
        threads = kBlock;
        upl = 8;
    }
    if (shape) {
        cap = shape[0]; xcd = shape[1]; drain = shape[2]; upl = shape[3]; threads = shape[4]; one_xcd = shape[5];
    }
    if (threads != 512 && threads != 1024) threads = kBlock;
    // the grid barrier needs every workgroup resident: at most the waves of
    // kCopyStepsMaxGrid 256-lane workgroups (4 per CU), whatever the width
    int max_grid = kCopyStepsMaxGrid * kBlock / threads;
    if (one_xcd) {           // the working workgroups share XCD 0's 32 CUs
        max_grid /= 8;
        xcd = 0;
    }
    if (cap < 1 || cap > max_grid) cap = max_grid;
    if (upl < 1) upl = 1;
    const size_t n16 = n / 16;
    size_t grid = (n16 + (size_t)threads * upl - 1) / ((size_t)threads * upl);
    if (grid > (size_t)cap) grid = (size_t)cap;
    if (grid < 1) grid = 1;
    if (grid_out) *grid_out = (int)grid;
    (void)hipGetLastError();   // drop a stale error of an earlier, ignored call
    void (*k)(const v4u*, v4u*, size_t, unsigned, int, u64*, int, int) =
        threads == 1024 ? (xcd ? k_copy_steps<1024, true> : k_copy_steps<1024, false>)
        : threads == 512 ? (xcd ? k_copy_steps<512, true> : k_copy_steps<512, false>)
                         : (xcd ? k_copy_steps<kBlock, true> : k_copy_steps<kBlock, false>);
    hipLaunchKernelGGL(k, dim3((unsigned)(one_xcd ? grid * 8 : grid)), dim3((unsigned)threads), 0, s,
                       reinterpret_cast<const v4u*>(src), reinterpret_cast<v4u*>(dst), n16, (unsigned)(n & 15), iters,
                       bar, drain, one_xcd);
    return hipGetLastError();
}

// All `iters` copies in one k_copy_pipe launch: UPL units per lane chosen so
// the grid (<= kCopyPipeMaxGrid workgroups of 320 lanes, all resident) covers
// n; returns hipErrorInvalidValue when n is too large for a resident grid.
hipError_t launch_copy_pipe(void* dst, const void* src, size_t n, int iters, u64* bar, hipStream_t s,
                            int* grid_out, int upl_force, int hier_force) {
    const size_t n16 = n / 16;
    const size_t lanes = (size_t)kPipeCopyWaves * 64;
    // resident grid: 5-wave workgroups, as many per CU as the VGPRs allow
    // (UPL 16: 208 VGPRs, one per CU; UPL 8: 112, three; UPL <= 4: six)
    auto cap_of = [](int u) -> size_t { return u >= 16 ? 256 : u >= 8 ? 512 : (size_t)kCopyPipeMaxGrid; };
    // Shape.  Up to 1 MiB: 8 units per lane and one barrier counter — few
    // wide workgroups (16-32), because one counter's cost grows with its
    // arrivals (at 2 MiB: 64 workgroups 2.11 us per copy, 256 4.04, 512 7.8;
    // r03_copy_pipe_ab.jsonl).  Above: the two-level barrier (8 group
    // counters in parallel, per-group release words) with up to 256
    // workgroups of 4-16 units per lane: 4 MiB 2.56-2.59 us, 8 MiB 3.2-3.9,
    // 16 MiB 4.3-6.0 against 2.9-3.0 / 3.2-4.2 / 5.0-6.8 for a launch per
    // copy.  The one-counter form with 64+ workgroups read 3.07-3.14 at 2 MiB
    // in three of four bench.py sweeps (2.08-2.14 in a fresh process), and
    // 4.3-6.2 at 4-8 MiB after 1 GiB copies (r03_copy_pipe_hier.jsonl,
    // r03_copy_pipe_state.jsonl).
    const bool big = n > ((size_t)1 << 20);
    int upl = big ? 4 : 8;
    while (big && upl < 16 && (n16 + lanes * upl - 1) / (lanes * upl) > 256) upl *= 2;
    if (upl_force > 0) upl = upl_force;   // tests: every units-per-lane form
    upl = upl <= 1 ? 1 : upl <= 2 ? 2 : upl <= 4 ? 4 : upl <= 8 ? 8 : 16;
    size_t grid = (n16 + lanes * upl - 1) / (lanes * upl);
    while (grid > cap_of(upl) && upl < 16) {
        upl *= 2;
        grid = (n16 + lanes * upl - 1) / (lanes * upl);
    }
    if (grid > cap_of(upl) || n >= ((size_t)1 << 32)) return hipErrorInvalidValue;
    if (grid < 1) grid = 1;
    if (grid_out) *grid_out = (int)grid;
    // (nontemporal loads: default-policy ones read the same, fresh or after
    // 1 GiB copies, 2-8 MiB within 0.03 us: profiles/r03_copy_pipe_state.jsonl)
    void (*k)(const v4u*, v4u*, size_t, unsigned, int, u64*, int) =
        upl <= 1 ? k_copy_pipe<1> : upl <= 2 ? k_copy_pipe<2> : upl <= 4 ? k_copy_pipe<4>
        : upl <= 8 ? k_copy_pipe<8> : k_copy_pipe<16>;
    const int hier = hier_force >= 0 ? (hier_force != 0) : (big ? 1 : 0);   // tests: both barrier forms
    (void)hipGetLastError();   // drop a stale error of an earlier, ignored call
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(kPipeThreads), 0, s, reinterpret_cast<const v4u*>(src),
                       reinterpret_cast<v4u*>(dst), n16, (unsigned)(n & 15), iters, bar, hier);
    return hipGetLastError();
}

hipError_t launch_fill(void* p, size_t n, int pattern, u64 arg, hipStream_t s) {
    size_t grid = (n / 8 + kBlock - 1) / kBlock;
    if (grid > 4096) grid = 4096;
    if (grid < 1) grid = 1;
    (void)hipGetLastError();   // drop a stale error of an earlier, ignored call
    hipLaunchKernelGGL(k_fill, dim3((unsigned)grid), dim3(kBlock), 0, s, reinterpret_cast<unsigned char*>(p), n,
                       pattern, arg);
    return hipGetLastError();
}

hipError_t launch_checksum(const void* p, size_t n, u64* out_dev, hipStream_t s) {
    size_t grid = (n / 16 + kBlock - 1) / kBlock;
    if (grid > 2048) grid = 2048;
    if (grid < 1) grid = 1;
    (void)hipGetLastError();   // drop a stale error of an earlier, ignored call
    hipLaunchKernelGGL(k_checksum, dim3((unsigned)grid), dim3(kBlock), 0, s, reinterpret_cast<const unsigned char*>(p),
                       n, out_dev);
    return hipGetLastError();
}

hipError_t launch_signal(u64* flag, const u64* base, u64 value, hipStream_t s) {
    (void)hipGetLastError();   // drop a stale error of an earlier, ignored call
    hipLaunchKernelGGL(k_signal, dim3(1), dim3(64), 0, s, flag, base, value);
    return hipGetLastError();
}

hipError_t launch_wait(const u64* flag, const u64* base, u64 value, Status* st, u64 timeout_ticks, hipStream_t s) {
    (void)hipGetLastError();   // drop a stale error of an earlier, ignored call
    hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, s, flag, base, value, st, timeout_ticks);
    return hipGetLastError();
}

hipError_t launch_seqbase(u64* base, u64 tx, u64 rx, int add, hipStream_t s) {
    (void)hipGetLastError();   // drop a stale error of an earlier, ignored call
    hipLaunchKernelGGL(k_seqbase, dim3(1), dim3(64), 0, s, base, tx, rx, add);
    return hipGetLastError();
}

hipError_t launch_account(Status* st, const u64* csum, int j0, int count, long long n, hipStream_t s) {
    const u64 z = (u64)n;
    u64 m = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;   // mix64(n), host side
    m = (m ^ (m >> 27)) * 0x94d049bb133111ebull;
    m ^= m >> 31;
    (void)hipGetLastError();   // drop a stale error of an earlier, ignored call
    hipLaunchKernelGGL(k_account, dim3(1), dim3(kBlock), 0, s, st, csum, j0, count, m);
    return hipGetLastError();
}

}  // namespace mpx
