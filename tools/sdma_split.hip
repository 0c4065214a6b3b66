// sdma_split.hip — does one device-to-device copy split over k streams run on
// k copy engines at once?  hipMemcpyDeviceToDeviceNoCU (copy engines only),
// on one GPU: the whole copy on one stream, or k equal slices on k streams
// (fork/join with events), k = 1, 2, 4.  Prints one JSON line per (bytes, k):
// the best of 5 timed batches of 10 copies.
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/sdma_split tools/sdma_split.hip
//   tools/sdma_split
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            printf("FAIL %s: %s\n", #x, hipGetErrorString(e_));                          \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

int main() {
    const size_t top = (size_t)64 << 20;
    char *src, *dst;
    CK(hipMalloc(&src, top));
    CK(hipMalloc(&dst, top));
    CK(hipMemset(src, 0x5a, top));
    hipStream_t s[4];
    for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    hipEvent_t e0, e1, fork, join[4];
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    for (auto& x : join) CK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
    for (size_t n : {(size_t)1 << 20, (size_t)4 << 20, (size_t)16 << 20, top}) {
        for (int k : {1, 2, 4}) {
            float best = 1e30f;
            for (int rep = 0; rep < 6; ++rep) {
                CK(hipEventRecord(e0, s[0]));
                for (int it = 0; it < 10; ++it) {
                    if (k == 1) {
                        CK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDeviceNoCU, s[0]));
                        continue;
                    }
                    CK(hipEventRecord(fork, s[0]));
                    const size_t part = n / k;
                    for (int j = 0; j < k; ++j) {
                        if (j) CK(hipStreamWaitEvent(s[j], fork, 0));
                        CK(hipMemcpyAsync(dst + j * part, src + j * part, j + 1 == k ? n - j * part : part,
                                          hipMemcpyDeviceToDeviceNoCU, s[j]));
                        if (j) CK(hipEventRecord(join[j], s[j]));
                    }
                    for (int j = 1; j < k; ++j) CK(hipStreamWaitEvent(s[0], join[j], 0));
                }
                CK(hipEventRecord(e1, s[0]));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep > 0 && ms < best) best = ms;   // rep 0 warms up
            }
            const double per = best * 1e-3 / 10;
            printf("{\"bytes\": %zu, \"streams\": %d, \"us_per_copy\": %.2f, \"GBps\": %.1f}\n", n, k, per * 1e6,
                   n / per / 1e9);
            fflush(stdout);
        }
    }
    return 0;
}
