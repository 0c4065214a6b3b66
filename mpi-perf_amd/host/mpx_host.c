/*
 * mpx_host.c — host-side logic of mpx_perf (see mpx_host.h).  Pure C.
 * Reference: /root/reference/mpi_perf.c (cited per function).
 */
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include "mpx_host.h"

#include <arpa/inet.h>
#include <ctype.h>
#include <fcntl.h>
#include <netdb.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

void mpxh_defaults(mpxh_options *o)
{
    memset(o, 0, sizeof *o);
    o->use_dotnet = 0;              /* mpi_perf.c:388 */
    o->uni_dir = 0;                 /* :389 */
    o->iters = MPXH_DEF_ITERS;      /* :390 */
    o->buff_sz = MPXH_DEF_BUF_SZ;   /* :391 */
    o->num_runs = 1;                /* :392 */
    o->engine = 0;
    o->timeout_ms = 10000;
    o->arm = 1;
}

int mpxh_engine_from_name(const char *s)
{
    if (!strcmp(s, "kernel") || !strcmp(s, "0")) return 0;
    if (!strcmp(s, "sdma") || !strcmp(s, "1")) return 1;
    if (!strcmp(s, "rccl") || !strcmp(s, "2")) return 2;
    return -1;
}

const char *mpxh_engine_name(int e)
{
    return e == 0 ? "kernel" : e == 1 ? "sdma" : e == 2 ? "rccl" : "?";
}

/* mpi_perf.c:20-32 — the reference's text verbatim, then the new flags */
void mpxh_print_usage(FILE *f)
{
    fprintf(f, "Usage: <program> \n\
		    -f <group1-hosts>\n\
		    -n <group1-size> \n\
		    -d <use-dotnet 0|1>\n\
		    -p <ppn> \n -i <iters>\n\
		    -b <buffer-size>\n\
		    -u <uni-directional (MPI-only) 0|1>\n\
		    -r <number-of-runs>\n\
		    -l <logfolder>\n\
		    -x <use non-blocking MPI calls>");
    fprintf(f, "\n\
		    MI355X extensions:\n\
		    -w <ranks (one GPU each; default 2*ppn)>\n\
		    -g <rank->GPU list, e.g. 0,1,2,3>\n\
		    -e <engine kernel|sdma|rccl>\n\
		    -a <all-pairs circle-method rounds 0|1>\n\
		    -c <checksum every payload 0|1|2 (2: seeded-pattern payloads)>\n\
		    -S <min:max power-of-two message-size sweep>\n\
		    -t <device wait timeout ms>\n\
		    -A <launch each run's kernel before the barrier 0|1 (default 1)>\n");
}

/* parse_args, mpi_perf.c:273-339 */
int mpxh_parse_args(mpxh_options *o, int argc, char **argv)
{
    int opt;
    optind = 1;
    opterr = 0;
    while ((opt = getopt(argc, argv, ":f:n:d:p:i:b:u:h:r:l:x:w:e:a:c:S:t:g:A:")) != -1) {
        switch (opt) {
        case 'f': strncpy(o->group1_hostfile, optarg, MPXH_MAX_HOST - 1); break;
        case 'n': o->group_size = atoi(optarg); break;
        case 'd': o->use_dotnet = atoi(optarg); break;
        case 'p': o->ppn = atoi(optarg); break;
        case 'i': o->iters = atoi(optarg); break;
        case 'b': o->buff_sz = atoi(optarg); break;
        case 'u': o->uni_dir = atoi(optarg); break;
        case 'r': o->num_runs = atoi(optarg); break;
        case 'x': o->nonblocking = atoi(optarg); break;
        case 'l': strncpy(o->logfolder, optarg, MPXH_MAX_HOST - 1); break;
        case 'w': o->world = atoi(optarg); break;
        case 'e':
            o->engine = mpxh_engine_from_name(optarg);
            if (o->engine < 0) return MPXH_PARSE_BAD_VALUE;
            break;
        case 'a': o->all_pairs = atoi(optarg); break;
        case 'c': o->check = atoi(optarg); break;
        case 'S': {
            char *colon = strchr(optarg, ':');
            if (!colon) return MPXH_PARSE_BAD_VALUE;
            o->sweep_min = atoi(optarg);
            o->sweep_max = atoi(colon + 1);
            if (o->sweep_min < 1 || o->sweep_max < o->sweep_min) return MPXH_PARSE_BAD_VALUE;
            break;
        }
        case 't': o->timeout_ms = atoi(optarg); break;
        case 'g': strncpy(o->gpus, optarg, sizeof o->gpus - 1); break;
        case 'A': o->arm = atoi(optarg); break;
        default: return MPXH_PARSE_USAGE; /* includes -h and a missing value */
        }
    }
    mpxh_uuid(o->uuid);
    return MPXH_PARSE_OK;
}

/* mpi_perf.c:399-403 */
int mpxh_validate(const mpxh_options *o, int world, FILE *err)
{
    if (o->group_size <= 0) goto invalid;
    if (!o->uni_dir) {
        if (o->ppn == 0) return 2; /* world_size / (2 * ppn): integer division by zero */
        if (o->group_size != world / (2 * o->ppn)) goto invalid;
    }
    return 0;
invalid:
    fprintf(err, "invalid group_size: %d, world_size: %d, ppn: %d\n", o->group_size, world, o->ppn);
    return 1;
}

/* mpi_perf.c:405-418 */
char *mpxh_read_group1(const char *path, int group_size)
{
    FILE *f = fopen(path, "r");
    if (!f) return NULL;
    char *lines = (char *)calloc((size_t)(group_size > 0 ? group_size : 1), MPXH_MAX_HOST);
    int i = 0;
    /* the reference reads every line (it does not stop at group_size) into a
       group_size-line block; here reading stops at the block's end */
    while (i < group_size && fgets(lines + (size_t)i * MPXH_MAX_HOST, MPXH_MAX_HOST, f)) i++;
    fclose(f);
    return lines;
}

/* mpi_perf.c:34-53 */
int mpxh_strnicmp(const char *s1, const char *s2, size_t n)
{
    for (size_t i = 0; i < n; i++) {
        const int c1 = tolower((unsigned char)s1[i]);
        const int c2 = tolower((unsigned char)s2[i]);
        if (c1 != c2) return c1 - c2;
        if (c1 == '\0') break;
    }
    return 0;
}

/* mpi_perf.c:437-444: name_len = strlen(name) chars compared per line */
int mpxh_in_group1(const char *name, const char *lines, int group_size)
{
    const size_t name_len = strlen(name);
    int g = 0;
    for (int i = 0; i < group_size; i++)
        if (mpxh_strnicmp(name, lines + (size_t)i * MPXH_MAX_HOST, name_len) == 0) g = 1;
    return g;
}

/* MPI_Comm_split(WORLD, group, world_rank) -> group_rank/group_size
   (mpi_perf.c:447-450); first other-group rank with equal group_rank
   (mpi_perf.c:225-233) */
void mpxh_pairing(int world, const int *group, int *group_rank, int *group_size, int *peer)
{
    int count[2] = {0, 0};
    for (int r = 0; r < world; ++r) group_rank[r] = count[group[r] ? 1 : 0]++;
    for (int r = 0; r < world; ++r) {
        group_size[r] = count[group[r] ? 1 : 0];
        peer[r] = -1;
        for (int i = 0; i < world; ++i)
            if (group[i] != group[r] && group_rank[i] == group_rank[r]) {
                peer[r] = i;
                break;
            }
    }
}

void mpxh_processor_name(char *out, const char *node, int rank, int ppn, const char *override_list)
{
    if (override_list && *override_list) {
        const char *p = override_list;
        for (int i = 0; i < rank && p; ++i) {
            p = strchr(p, ',');
            if (p) p++;
        }
        if (p) {
            size_t len = strcspn(p, ",");
            if (len >= MPXH_MAX_HOST) len = MPXH_MAX_HOST - 1;
            memcpy(out, p, len);
            out[len] = 0;
            return;
        }
    }
    snprintf(out, MPXH_MAX_HOST, "%s-%d", node, ppn > 0 ? rank / ppn : 0);
}

/* Round r of the circle method: position 0 fixed, positions 1..n-1 rotate
   by r; pair k joins positions k and n-1-k. */
int mpxh_round_pairs(int n, int r, int (*pairs)[2])
{
    if (n < 2 || (n & 1) || r < 0 || r >= n - 1) return -1;
    int pos[MPXH_MAX_RANKS];
    pos[0] = 0;
    for (int i = 1; i < n; ++i) pos[i] = 1 + ((i - 1 + (n - 1) - r) % (n - 1));
    for (int k = 0; k < n / 2; ++k) {
        pairs[k][0] = pos[k];
        pairs[k][1] = pos[n - 1 - k];
    }
    return n / 2;
}

int mpxh_round_role(int n, int r, int rank, int *group, int *peer)
{
    int pairs[MPXH_MAX_RANKS / 2][2];
    const int np = mpxh_round_pairs(n, r, pairs);
    for (int k = 0; k < np; ++k) {
        if (pairs[k][0] == rank) { *group = 1; *peer = pairs[k][1]; return 0; }
        if (pairs[k][1] == rank) { *group = 0; *peer = pairs[k][0]; return 0; }
    }
    return -1;
}

int mpxh_parse_gpu_list(const char *s, int *devs, int n)
{
    int k = 0;
    const char *p = s;
    while (*p) {
        char *end;
        const long v = strtol(p, &end, 10);
        if (end == p || v < 0 || k >= n) return -1;
        devs[k++] = (int)v;
        p = end;
        if (*p == ',') p++;
        else if (*p) return -1;
    }
    return k;
}

/* mpi_perf.c:341-353 */
void mpxh_format_time(char *buf, size_t cap, int for_kusto)
{
    time_t t;
    time(&t);
    struct tm tmv;
    localtime_r(&t, &tmv);
    strftime(buf, cap, for_kusto ? "%Y-%m-%d %H:%M:%S" : "%Y-%m-%d-%H-%M-%S", &tmv);
}

/* mpi_perf.c:550-554 (Timestamp,JobId,Rank,VMCount,LocalIP,RemoteIP,
   NumOfFlows,BufferSize,NumOfBuffers,TimeTakenms,RunId) */
int mpxh_format_record(char *out, size_t cap, const char *timestamp, const char *uuid, int world_rank,
                       int world_size, int ppn, const char *local_ip, const char *remote_ip, int buff_len,
                       int iters, double my_time_s, long long run_idx)
{
    return snprintf(out, cap, "%s,%s,%d,%d,%s,%s,%d,%d,%d,%.2lf,%lld\n", timestamp, uuid, world_rank,
                    world_size / ppn, local_ip, remote_ip, ppn, buff_len, iters, my_time_s * 1000.0, run_idx);
}

/* mpi_perf.c:494 */
int mpxh_log_name(char *out, size_t cap, const char *logfolder, const char *uuid, int world_rank,
                  const char *file_time)
{
    return snprintf(out, cap, "%s/tcp-%s-%d-%s.log", logfolder, uuid, world_rank, file_time);
}

/* mpi_perf.c:535-541 */
int mpxh_format_bandwidth(char *out, size_t cap, int world_rank, long long run_idx, int buff_len, int iters,
                          int uni_dir, double my_time_s)
{
    const long double gbits = 8.0 * buff_len * iters * ((uni_dir == 1) ? 1.0 : 2.0) * 1e-9;
    const long double bw = (gbits * 1.0) / my_time_s;
    return snprintf(out, cap, "[Rank: %d Run#: %lld]: Total Gbits: %Lf, Bandwidth: %.2Lf Gbps\n", world_rank,
                    run_idx, gbits, bw);
}

/* mpi_perf.c:564-568 */
int mpxh_format_summary(char *out, size_t cap, long long run_idx, double total_s, double min_s, double max_s,
                        double sum_s, int world)
{
    return snprintf(out, cap, "[Run#: %lld]: Total time: %.2lf ms, Min: %.2lf ms, Max: %.2lf ms, Avg: %.2lf ms\n",
                    run_idx, total_s * 1000.0, min_s * 1000.0, max_s * 1000.0, (sum_s * 1000) / world);
}

/* mpi_perf.c:460-461 */
int mpxh_format_info(char *out, size_t cap, const char *name, int rank, int world, int group, int group_size,
                     int group_rank, int peer, const char *my_ip, const char *peer_name, const char *peer_ip)
{
    return snprintf(out, cap,
                    "INFO: %s, rank %d out of %d ranks, my_group: %d, group_size: %d, group_rank: %d, my_peer: %d, "
                    "hostname: %s (%s), peer_host: %s (%s)\n",
                    name, rank, world, group, group_size, group_rank, peer, name, my_ip, peer_name, peer_ip);
}

/* mpi_perf.c:147-168 */
int mpxh_format_dotnet(char *out, size_t cap, int my_group, int my_rank, int peer_rank, const char *peer_ip,
                       const char *my_ip, int buff_len, int iters, int ppn)
{
    const int port = 40000; /* DEF_PORT */
    if (my_group == 1)
        return snprintf(out, cap,
                        "dotnet /mnt/anfvol/tepati/clientserverapp/bin/Release/net6.0/clientserverapp.dll server %s "
                        "%d 1 %d %d %d %d true\n",
                        my_ip, port + my_rank, ppn, buff_len, iters, 0);
    return snprintf(out, cap,
                    "dotnet /mnt/anfvol/tepati/clientserverapp/bin/Release/net6.0/clientserverapp.dll client %s %d "
                    "%d %d %d %d true\n",
                    peer_ip, port + peer_rank, ppn, buff_len, iters, 0);
}

void mpxh_uuid(char out[37])
{
    unsigned char b[16];
    int fd = open("/dev/urandom", O_RDONLY);
    ssize_t got = fd >= 0 ? read(fd, b, sizeof b) : -1;
    if (fd >= 0) close(fd);
    if (got != (ssize_t)sizeof b) {
        struct timespec ts;
        clock_gettime(CLOCK_REALTIME, &ts);
        uint64_t x = (uint64_t)ts.tv_nsec ^ ((uint64_t)ts.tv_sec << 20) ^ (uint64_t)getpid();
        for (int i = 0; i < 16; ++i) {
            x = x * 6364136223846793005ULL + 1442695040888963407ULL;
            b[i] = (unsigned char)(x >> 56);
        }
    }
    b[6] = (unsigned char)((b[6] & 0x0f) | 0x40); /* version 4 */
    b[8] = (unsigned char)((b[8] & 0x3f) | 0x80); /* RFC 4122 variant */
    snprintf(out, 37, "%02x%02x%02x%02x-%02x%02x-%02x%02x-%02x%02x-%02x%02x%02x%02x%02x%02x", b[0], b[1], b[2],
             b[3], b[4], b[5], b[6], b[7], b[8], b[9], b[10], b[11], b[12], b[13], b[14], b[15]);
}

/* mpi_perf.c:171-198: AF_INET, SOCK_STREAM; keeps the LAST address */
int mpxh_ipv4(const char *host, char *out, size_t cap)
{
    struct addrinfo hints, *res;
    memset(&hints, 0, sizeof hints);
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (!host || getaddrinfo(host, NULL, &hints, &res) != 0) return -1;
    char ip[INET_ADDRSTRLEN] = {0};
    for (struct addrinfo *p = res; p != NULL; p = p->ai_next)
        inet_ntop(p->ai_family, &((struct sockaddr_in *)p->ai_addr)->sin_addr, ip, sizeof ip);
    freeaddrinfo(res);
    snprintf(out, cap, "%s", ip);
    return 0;
}

/* ---- the Windows / MS-MPI variant (/root/reference/windows/mpi-perf.cpp) --
   Same record, log name and run loop as mpi_perf.c; a different front end:
   seven positional arguments, unidirectional only, groups keyed by IPv4
   address with a whole-string match, the peer is the last match. */

/* generate_uuid, windows/mpi-perf.cpp:175-184: the GUID is formatted with
   snprintf(guid_str, sizeof(guid_str), ...) where guid_str is a char *, so
   only sizeof(char *) - 1 = 7 characters survive: the first 7 hex digits of
   Data1.  Job ids and log names of the Windows variant carry exactly that. */
void mpxh_uuid_windows(char out[64])
{
    char full[37];
    mpxh_uuid(full);
    memset(out, 0, 64);
    memcpy(out, full, sizeof(char *) - 1); /* what snprintf(out, sizeof(char *), ...) keeps */
}

/* parse_args, windows/mpi-perf.cpp:187-197, over main's defaults (:226-230):
   argv[1..7] = group-1 address file, group size, ppn, iters, buffer size,
   runs, log folder.  A missing argument makes the reference pass argv[argc]
   (NULL) to strncpy / atoi: MPXH_PARSE_CRASH.  Arguments after the seven are
   ignored by the reference; here they may carry the MI355X extension flags
   (-w -g -e -a -c -S -t), never the reference's own letters. */
int mpxh_parse_args_windows(mpxh_options *o, int argc, char **argv)
{
    if (argc < 8) return MPXH_PARSE_CRASH;
    o->use_dotnet = 0; /* :226 */
    o->uni_dir = 1;    /* :228 */
    o->nonblocking = 0;
    strncpy(o->group1_hostfile, argv[1], MPXH_MAX_HOST - 1);
    o->group_size = atoi(argv[2]);
    o->ppn = atoi(argv[3]);
    o->iters = atoi(argv[4]);
    o->buff_sz = atoi(argv[5]);
    o->num_runs = atoi(argv[6]);
    strncpy(o->logfolder, argv[7], MPXH_MAX_HOST - 1);
    if (argc > 8) {
        for (int i = 8; i < argc; ++i)
            if (argv[i][0] == '-' && argv[i][1] && !argv[i][2] && strchr("fndpibuhrlx", argv[i][1]))
                return MPXH_PARSE_USAGE;
        mpxh_options x;
        mpxh_defaults(&x);
        const int st = mpxh_parse_args(&x, argc - 7, argv + 7);
        if (st != MPXH_PARSE_OK) return st;
        o->world = x.world;
        o->engine = x.engine;
        o->all_pairs = x.all_pairs;
        o->check = x.check;
        o->sweep_min = x.sweep_min;
        o->sweep_max = x.sweep_max;
        o->timeout_ms = x.timeout_ms;
        o->arm = x.arm;
        memcpy(o->gpus, x.gpus, sizeof o->gpus);
    }
    mpxh_uuid_windows(o->uuid); /* :196 */
    return MPXH_PARSE_OK;
}

/* windows/mpi-perf.cpp:249-261: fgets every line, newline cut off (:259) */
char *mpxh_read_group1_windows(const char *path, int group_size)
{
    char *lines = mpxh_read_group1(path, group_size);
    if (!lines) return NULL;
    for (int i = 0; i < (group_size > 0 ? group_size : 0); ++i) {
        char *ln = lines + (size_t)i * MPXH_MAX_HOST;
        ln[strcspn(ln, "\n")] = '\0';
    }
    return lines;
}

/* windows/mpi-perf.cpp:283-289: my_strnicmp(my_ipaddr, line, MAX_HOST_SZ),
   i.e. the whole address, case-insensitively (no prefix match) */
int mpxh_in_group1_windows(const char *addr, const char *lines, int group_size)
{
    int g = 0;
    for (int i = 0; i < group_size; i++)
        if (mpxh_strnicmp(addr, lines + (size_t)i * MPXH_MAX_HOST, MPXH_MAX_HOST) == 0) g = 1;
    return g;
}

/* MPI_Comm_split (windows/mpi-perf.cpp:292-295) and get_peer_info
   (:114-133): the loop has no break, so the LAST other-group rank with the
   same group rank wins.  With two groups and ranks numbered by world rank
   there is at most one, so the pairs equal mpxh_pairing's. */
void mpxh_pairing_windows(int world, const int *group, int *group_rank, int *group_size, int *peer)
{
    mpxh_pairing(world, group, group_rank, group_size, peer);
    for (int r = 0; r < world; ++r) {
        peer[r] = -1;
        for (int i = 0; i < world; ++i)
            if (group[i] != group[r] && group_rank[i] == group_rank[r]) peer[r] = i;
    }
}
