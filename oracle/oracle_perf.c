/*
 * oracle_perf.c — CLI over the CPU restatement (mpx_oracle.c): runs `-r` runs
 * of `-p` concurrent pairs with the reference's loop semantics on host
 * threads and prints one JSON object per run.  TEST INFRASTRUCTURE: bench.py
 * times it as cpu_baseline "kind": "port" when the compiled reference
 * (oracle/_ref) is not available.  Flags follow mpi_perf.c:276.
 */
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include "mpx_oracle.h"
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

int main(int argc, char **argv)
{
    int ppn = 1, iters = 10, B = 456131, uni = 0, nb = 0, runs = 1, opt;
    while ((opt = getopt(argc, argv, "p:i:b:u:x:r:")) != -1) {
        switch (opt) {
        case 'p': ppn = atoi(optarg); break;
        case 'i': iters = atoi(optarg); break;
        case 'b': B = atoi(optarg); break;
        case 'u': uni = atoi(optarg); break;
        case 'x': nb = atoi(optarg); break;
        case 'r': runs = atoi(optarg); break;
        default: fprintf(stderr, "usage: oracle_perf -p ppn -i iters -b bytes [-u 1|-x 1] -r runs\n"); return 2;
        }
    }
    if (ppn < 1 || iters < 0 || B < 0 || runs < 1) return 2;
    const int mode = uni ? ORACLE_UNIDIR : (nb ? ORACLE_NONBLOCKING : ORACLE_PINGPONG);
    oracle_rank_stats *st = calloc((size_t)(2 * ppn), sizeof *st);
    for (int r = 0; r < runs; ++r) {
        double mx = 0;
        if (oracle_run_pairs(ppn, mode, iters, (size_t)B, st, &mx)) return 1;
        const double bytes = (double)B * iters * (uni ? 1 : 2) * ppn;
        printf("{\"run\": %d, \"ppn\": %d, \"mode\": %d, \"bytes\": %d, \"iters\": %d, \"max_time_s\": %.9f, "
               "\"aggregate_GBps\": %.6f, \"g1_digest\": %llu, \"g0_digest\": %llu}\n",
               r, ppn, mode, B, iters, mx, mx > 0 ? bytes / mx / 1e9 : 0.0,
               (unsigned long long)st[0].recv_digest, (unsigned long long)st[ppn].recv_digest);
        fflush(stdout);
    }
    free(st);
    return 0;
}
