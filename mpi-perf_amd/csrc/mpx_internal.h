// mpx_internal.h — types shared by the libmpx runtime (mpx_runtime.hip) and
// its device code (mpx_kernels.hip).  Not part of the C-ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include "../../include/mpx.h"

typedef unsigned long long u64;

namespace mpx {

constexpr int kBlock = 256;              // threads per workgroup = 4 wave64
constexpr int kMaxPushWG = 256;          // flag slots per (receiver, sender) link
constexpr int kLLMaxBytes = 8192;        // messages <= this go as LL granules
constexpr int kLLGranules = kLLMaxBytes / 4;   // 4 payload bytes per granule
constexpr int kNbWindow = 256;           // MAX_REQ_NUM, mpi_perf.c:88
constexpr int kStageMaxBytes = 60 << 10; // LDS-staged tx chunk per workgroup, max
                                         // (under a 64 KiB per-workgroup LDS limit)

// Protocol ids reported in mpx_timing.protocol
enum Proto { kProtoLL = 0, kProtoBulk = 1, kProtoSdma = 2, kProtoRccl = 3, kProtoCopy = 4, kProtoCopySteps = 5,
             kProtoCopyPipe = 6, kProtoPull = 7, kProtoSdmaPull = 8 };

// One rank's receive mailbox, in that rank's HBM (uncached / fine-grained so a
// poll sees stores that arrive over xGMI).  Written ONLY by the peers, polled
// only by the owner.
//   flag[s][w]   : sequence number of the last bulk push workgroup w of sender
//                  rank s finished into this rank's rx (written with one
//                  system-scope store after that workgroup's payload drained)
//   ll[s][g]     : LL granule g of the current small message from sender s:
//                  {tag:32 | payload:32}, tag = ll_tag(seq), one 8-byte store
//   credit[s][w] : sequence number of the last of THIS rank's pushes whose
//                  chunk w rank s is done with: non-blocking check mode —
//                  checksummed (and poisoned), i.e. the ring slot it used is
//                  free again; pull mode — loaded from this rank's tx, i.e.
//                  that chunk of tx may change again
//   ready[s]     : pull mode (MPX_XFER_PULL) — sequence number of the last
//                  push rank s made available in its tx (one store per send,
//                  by the sender; the receiver loads the bytes itself)
//   posted[s]    : "receives posted", written by rank s: the number of the
//                  latest transfer call between s and this rank that s has
//                  started.  It grows by one per call on both sides
//                  (Rank.calls), so no call's value equals an earlier call's.
//                  Rank s stores it as the first action of its call (its
//                  stream has then finished all of its previous call's work);
//                  this rank pushes no byte of call k into s's rx, ring or LL
//                  zone before it reads posted[s] >= k.  That is MPI's
//                  matched-receive order (mpi_perf.c:75,79,100,104,137,141):
//                  a payload of call k lands only under a receive of call k.
struct Mailbox {
    u64 flag[MPX_MAX_RANKS][kMaxPushWG];
    u64 ll[MPX_MAX_RANKS][kLLGranules];
    u64 credit[MPX_MAX_RANKS][kMaxPushWG];
    u64 posted[MPX_MAX_RANKS];
    u64 ready[MPX_MAX_RANKS];
};

// The end of a kernel-engine call: ONE 64-byte line of the host-mapped
// status, written by workgroup 0 with a single eight-lane store once every
// other store of the call has drained (Loop::finish_last).  The host spins on
// `word` = (u32)token | seal << 32, where the seal hashes the other seven
// words with the token: a line that became visible piecemeal does not match
// and is read again.  No drain sits between the line's fields and the word
// the host waits for — one PCIe write instead of a write, an
// acknowledgement and another write at the end of every call.
struct alignas(64) Fin {
    u64 recv_done;          // receives completed
    u64 recv_digest;        // check mode: sum of their finished checksums
    // phases (s_memrealtime, 100 MHz ticks), stamped by workgroup 0:
    u64 t_entry;            // started (after the go of an armed call)
    u64 t_posted;           // this side may push: the peer's receives are
                            // posted (0: this side pushes only after a receive)
    u64 t_first;            // the loop's first iteration done
    u64 t_loop;             // left the loop
    u64 t_exit;             // the call's end (every workgroup done)
    u64 word;               // fin_word(...): the host's completion word
};
__host__ __device__ inline u64 fin_mix(u64 z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__host__ __device__ inline u64 fin_word(u64 token, u64 v0, u64 v1, u64 v2, u64 v3, u64 v4, u64 v5, u64 v6) {
    u64 h = fin_mix(token ^ 0x6a09e667f3bcc909ull);
    h = fin_mix(h ^ v0);
    h = fin_mix(h ^ v1);
    h = fin_mix(h ^ v2);
    h = fin_mix(h ^ v3);
    h = fin_mix(h ^ v4);
    h = fin_mix(h ^ v5);
    h = fin_mix(h ^ v6);
    return (token & 0xffffffffull) | (h << 32);
}

// Per-rank host-mapped status words (written by the device, read by the host
// after the stream drains, or — the kernel engine — once `fin` is sealed).
struct Status {
    unsigned int err;       // bit0: a wait timed out
    unsigned int where;     // 1 + iteration index of the first timeout
    u64 spins;              // diagnostics: polls of the last wait
    // receive accounting of the last call, counted on the device where the
    // reference's call returns a receive (Recv, or Waitall for the
    // non-blocking loop, mpi_perf.c:75,79,110-111,122-123,137,141)
    u64 recv_done;          // receives completed (stream engines; the kernel
    u64 recv_digest;        // engine's are in fin) / check mode digest
    u64 seen, want;         // stream engines: flag value seen / awaited by the
                            // wait that timed out (diagnostics)
    u64 go;                 // armed call (mpx_xfer_arm): the host stores the
                            // call's token here to start it, token | kGoCancel
                            // to end it without a transfer
    u64 ready;              // armed call: its token once every workgroup is
                            // resident and waiting for go
    Fin fin;                // kernel engine: the end of the last call
};
constexpr u64 kGoCancel = 1ull << 63;

// Device scratch words of a rank ([0..3]: zero when a kernel-engine call
// starts — zeroed at attach, and reset by the last workgroup of every call, so
// no memset precedes the launch):
//   [0] grid-barrier counter  [1] abort word  [2] finished workgroups
//   [3] pull mode: chunks landed in rx this call (all receives, all workgroups)
//   [4..5] SDMA engine's device-side sequence base {tx, rx}
//   [6..7] RCCL engine's one-byte link set-up exchange
//   [8] armed call: workgroup 0's go verdict for the others (1 go, 2 cancel),
//       reset with [0..3]
//   [9] armed call: workgroups other than 0 waiting for go, reset with [0..3]
constexpr int kScratchWords = 16;
constexpr int kScrBar = 0, kScrAbort = 1, kScrFin = 2, kScrLanded = 3, kScrSeqBase = 4, kScrLink = 6, kScrGo = 8,
              kScrReady = 9;

// Non-blocking check mode ("ring"): receive j of a call with `iters`
// iterations lands in slot (iters-1-j) mod S of the receiver, where slot 0 is
// rx itself (so rx ends holding the last payload, as in the reference) and
// slot s >= 1 is ring + (s-1)*B.  S = min(256, 1 + ring_bytes / B), computed
// from the RECEIVER's ring on both sides of the link.
inline int ring_slots(unsigned long long ring_bytes, long long len) {
    if (len <= 0) return kNbWindow;
    const unsigned long long s = 1 + ring_bytes / (unsigned long long)len;
    return s < (unsigned long long)kNbWindow ? (int)s : kNbWindow;
}
__host__ __device__ inline int ring_slot(int j, int iters, int slots) { return (iters - 1 - j) % slots; }

// Arguments of one transfer loop on one rank (kernel engine).
struct XferArgs {
    const unsigned char* tx;     // local tx
    unsigned char* rx;           // local rx
    unsigned char* peer_rx;      // the peer's rx, mapped into this process
    Mailbox* my_mb;              // local mailbox (polled)
    Mailbox* peer_mb;            // peer's mailbox (written)
    Status* status;              // host-mapped
    u64* csum;                   // [iters] raw checksum sums (check mode)
    u64* gbar;                   // grid-barrier counter (check mode), zeroed
    u64 tx_seq0;                 // my last push seq on this link before the call
    u64 rx_seq0;                 // peer's last push seq on this link
    u64 timeout_ticks;           // s_memrealtime ticks (100 MHz) per wait
    long long len;               // B
    int iters;
    int mode;                    // enum mpx_mode
    int group;                   // 1 = sender side (group 1), 0 = group 0
    int my_slot;                 // my rank = my slot in the peer's mailbox
    int peer_slot;               // peer rank = its slot in my mailbox
    int nwg;                     // bulk push workgroups (same on both sides)
    int check;                   // 1 = checksum + poison each received payload
    int ll_max;                  // messages <= ll_max bytes use LL (<= kLLMaxBytes);
                                 // same on both sides of the link
    int stream;                  // 1: bulk payload stores add the nt hint (sc0 sc1 nt)
    int nb_publish;              // non-blocking mode: drain + flag every nb_publish
                                 // pushes (divides kNbWindow) and at the last
    int stage;                   // bytes of dynamic LDS holding this workgroup's
                                 // chunk of tx (0: bulk pushes read tx from HBM)
    // non-blocking check mode (k_xfer_nbcheck)
    unsigned char* ring;         // my receive slots 1..slots-1
    unsigned char* peer_ring;    // the peer's, mapped here
    u64* cnt;                    // [iters] workgroups done checking receive j
    int slots;                   // S: receive slots per link (ring_slots)
    int skip_push;               // test knob: 1 + iteration whose payload stores
                                 // are skipped (flag still published); 0 = off
    u64 call;                    // number of this call on the link (Mailbox.posted)
    int lag_wg;                  // test knob (MPX_TEST_LAG_WG): workgroup that stalls
    u64 lag_ticks;               //   lag_ticks before checking (non-blocking check
                                 //   mode) or pulling (pull mode) the call's last
                                 //   receive; 0 = off
    // pull mode (MPX_XFER_PULL, k_xfer_pull): bulk payloads are loaded by the
    // receiver from the sender's tx instead of stored by the sender
    const unsigned char* peer_tx;   // the peer's tx, mapped into this process
    int pull;                    // 1 = this call's bulk payloads are pulled
    int no_pull_wait;            // test knob (MPX_TEST_NO_PULL_WAIT): a sending side
                                 // ends without waiting for the peer's loads of tx
    u64 done_token;              // stored into Status.done by the last workgroup
    u64 go_token;                // armed call: wait for Status.go == go_token first
                                 // (0: start at once)
    u64 go_timeout_ticks;        // armed call: how long the kernel waits for go
};

// LL threshold of a link.  Within one GPU the bulk path's extra hop (payload
// drain, then flag) is cheap and bulk wins above ~2 KiB (loopback sweep,
// profiles/r01_loopback_sweep.jsonl; on the final LL path ping-pong from
// 3 KiB, r02_ll_threshold_ab.jsonl); across xGMI that hop is a full link
// round trip, so LL is kept up to its 8 KiB landing zone.
inline int ll_max_bytes(bool same_device) { return same_device ? 2048 : kLLMaxBytes; }

// LL granule tag for push sequence number `seq` (>= 1): never 0, so a zeroed
// mailbox can never match, and distinct for seqs < 2^31 apart.
__host__ __device__ inline unsigned ll_tag(u64 seq) {
    return (unsigned)(seq & 0x7fffffffull) | 0x80000000u;
}

// Workgroups of a bulk push of `len` bytes.  Both sides of a link evaluate
// this on the same inputs, so the receiver knows how many flags to expect.
constexpr long long kMinPushChunk = 1024;   // bytes per pushing workgroup, at least (run_kernel)
inline int bulk_nwg(long long len, bool same_device) {
    // ~32 KiB per workgroup across xGMI (enough 16-B stores in flight to
    // cover the link's bandwidth-delay product), 16 KiB within one GPU.
    const long long per = same_device ? (16 << 10) : (32 << 10);
    long long n = (len + per - 1) / per;
    // within one GPU both kernels of a pair, and of every other pair that
    // shares the GPU, must stay resident together: 128 keeps two pairs'
    // check-mode launches (4 x 128 workgroups) at half the chip's 4 per CU
    const long long cap = 128;
    if (n < 1) n = 1;
    if (n > cap) n = cap;
    return (int)n;
}

// Launchers implemented in mpx_kernels.hip
hipError_t launch_xfer(const XferArgs& a, int grid, hipStream_t s);
hipError_t launch_copy(void* dst, const void* src, size_t n, hipStream_t s, int* grid_out);
// all `iters` copies in one launch with a grid barrier between steps; *bar
// must be 0 at launch
constexpr int kCopyStepsMaxGrid = 1024;   // 4 workgroups per CU: always co-resident
// copies up to 1 MiB run as k_copy_steps: faster than a launch per copy
// there (1 MiB 1.94-2.0 vs 2.4-2.7 us).  At 2 MiB one launch is faster in a
// fresh process (2.32-2.38 vs 2.42-2.94 us with 64 workgroups on one barrier
// counter, on three boxes) but bistable: after bench.py's headline and sweep
// it read 3.4-3.9 us on two boxes where a launch per copy read 2.6-3.0
// (profiles/r02_copy_steps_wgsize_mid.jsonl, r02_copy_sweep_state.jsonl), so
// the switch stays at 1 MiB; above it a launch per copy is as fast or faster
// (16 MiB 4.22 vs 5.15-5.95; r02_copy_steps_upl.jsonl, r02_copy_steps_mid.jsonl)
constexpr size_t kCopyStepsDefaultMax = (size_t)1 << 20;
// k_copy_pipe's range: (512 KiB, 16 MiB] (shape rule and numbers at
// launch_copy_pipe).  Per copy, in bench.py's sweep (right after the 1 GiB
// headline) and in fresh processes, against k_copy_steps / a launch per
// copy: 1 MiB 1.67-2.1 us (2.0 / 2.3-3.0), 4 MiB 2.56-2.59 (3.0 / 2.9-3.0),
// 8 MiB 3.2-3.9 (4.2 / 3.2-4.2), 16 MiB 4.3-6.0 (- / 5.0-6.8).  512 KiB:
// 1.56 vs the one-XCD steps form's 1.64 (kept).  16 MiB is the resident
// limit of 256 workgroups x 16 units per lane (r03_copy_pipe_ab.jsonl,
// r03_copy_pipe_state.jsonl, r03_copy_pipe_hier.jsonl).
constexpr size_t kCopyPipeDefaultMin = (size_t)512 << 10;
constexpr size_t kCopyPipeDefaultMax = (size_t)16 << 20;
hipError_t launch_copy_steps(void* dst, const void* src, size_t n, int iters, u64* bar, hipStream_t s,
                             int* grid_out, const int* shape = nullptr);
// all `iters` copies in one k_copy_pipe launch (copy s+1's loads in flight
// across copy s's grid barrier, a dedicated barrier wave); *bar must be 0
constexpr int kCopyPipeMaxGrid = 768;     // 320-lane workgroups, 3 per CU: resident
hipError_t launch_copy_pipe(void* dst, const void* src, size_t n, int iters, u64* bar, hipStream_t s,
                            int* grid_out, int upl_force = 0, int hier_force = -1);
hipError_t launch_fill(void* p, size_t n, int pattern, u64 arg, hipStream_t s);
hipError_t launch_checksum(const void* p, size_t n, u64* out_dev, hipStream_t s);
hipError_t launch_signal(u64* flag, const u64* base, u64 value, hipStream_t s);
hipError_t launch_wait(const u64* flag, const u64* base, u64 value, Status* st, u64 timeout_ticks, hipStream_t s);
hipError_t launch_seqbase(u64* base, u64 tx, u64 rx, int add, hipStream_t s);
// stream engines' receive accounting: st->recv_done += count and, when csum is
// set, st->recv_digest += sum_j (csum[j] ^ mix64(n)) over j in [j0, j0+count)
hipError_t launch_account(Status* st, const u64* csum, int j0, int count, long long n, hipStream_t s);

}  // namespace mpx
