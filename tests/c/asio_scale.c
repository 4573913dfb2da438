/*
 * tests/c/asio_scale.c -- the netcache checksum call site at the reference's
 * own thread scale, as a plain-C program over the C ABI (test and
 * measurement infrastructure; not part of the product).
 *
 * netcache's ASIO pool runs 4-512 threads (asio_mgr.c:86, :91, started at
 * :205), and every one of them calls the block checksum on its completed
 * vector at once (asio_mgr.c:1050-1057); httpd runs 32 MHD workers by
 * default (httpd.c:8630) and chunk_size defaults to 128 KiB (httpd.c:8627).
 * Here T threads each submit a vector of B blocks of L bytes synchronously,
 * over and over, for S seconds:
 *   batcher  md5_batch_submit on ONE shared batcher (md5hip_batcher_create)
 *   pool     md5hip_pool_submit on a pool over device 0 listed twice
 *   host     MD5Init/MD5Update/MD5Final of the product library (md5_stream.c)
 *            per block on the calling thread -- the alternative the call
 *            site has, timed the same way
 * Each thread owns R vectors of distinct bytes and submits them in turn, R
 * chosen so that all threads' vectors together span at least 2 GiB: every
 * call's source is cold in the host caches whatever the thread count (with
 * one vector per thread, 8 threads' 8 MiB would stay in L3 and their
 * staging copies would look cheaper than 256 threads').  MODE pageable (the
 * default: the batcher copies the blocks into its pinned staging) or
 * registered (each thread's vectors md5hip_host_register'ed: zero-copy, the
 * device pulls them, no host copy -- what is left per call is the queue's
 * own cost).  Every call's digests are compared with the oracle's
 * (oracle/md5_oracle.c, linked in as the checker and computed once per
 * vector before timing).  Per call it records the wall
 * latency and the calling thread's CPU time (CLOCK_THREAD_CPUTIME_ID, the
 * clock of getrusage(RUSAGE_THREAD), around the call); the process CPU time
 * over the timed window (CLOCK_PROCESS_CPUTIME_ID, which includes the
 * batchers' progress threads and the HIP runtime's) is reported per call too.  Prints one JSON object.
 *
 * ASIO_FIXED_BG_MIB=M (batcher target): one more thread calls
 * md5hip_batch_host_fixed on an M MiB PAGEABLE array of 16 KiB chunks over
 * and over during the timed window (its H2D copy is synchronous from pageable
 * memory); its call times are reported as "bg_fixed" and its digests checked
 * -- the submitters' latency must not include that copy.
 *
 * ASIO_CRC=F: netcache's own CRC-32 (blk_make_crc, blk_io.c:354-430) with
 * fastcrc window F (0 = whole block) instead of MD5: the batcher / pool set
 * to MD5HIP_DIGEST_CRC32, the host leg the library's nc_crc32 over the same
 * windows, the checker oracle/crc32_oracle.c's blk_make_crc rule.
 *
 * usage: asio_scale TARGET THREADS BLOCKS BLOCK_BYTES SECS [MODE [SLICE_MIB NSLOTS]]
 * Exit 0 = every digest equal to the oracle's; 1 = a mismatch or error;
 * 77 = no usable HIP device.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/resource.h>
#include <time.h>

#include "md5.h"
#include "md5hip.h"
#include "nc_digest.h"

void oracle_md5(const void *data, uint64_t len, unsigned char digest[16]);
uint32_t oracle_blk_crc(const void *data, uint64_t remained, uint32_t fastcrc);
void oracle_xorshift_fill(void *dst, uint64_t nbytes, uint64_t seed);

enum target { T_BATCHER, T_POOL, T_HOST };

static enum target g_target;
static int g_threads, g_blocks;
static uint32_t g_len;
static double g_secs;
static md5hip_batcher *g_b;
static md5hip_pool *g_p;
static pthread_barrier_t g_start, g_warm, g_go;
static double g_t_end;          /* set between g_warm and g_go */
static int g_nvec = 1;          /* vectors per thread (R) */
static int g_register;          /* MODE registered */
static int g_crc = -1;          /* ASIO_CRC: fastcrc window of a CRC-32 run, -1 = MD5 */
static size_t g_dsz = 16;       /* digest bytes per block */

static double now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* user + system CPU of the calling thread / the process: the clocks behind
 * getrusage(RUSAGE_THREAD / RUSAGE_SELF), read at scheduler resolution
 * (getrusage rounds to the tick on kernels without precise accounting) */
static double cpu_clock(clockid_t id)
{
    struct timespec ts;
    clock_gettime(id, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}
static double thread_cpu(void) { return cpu_clock(CLOCK_THREAD_CPUTIME_ID); }
static double process_cpu(void) { return cpu_clock(CLOCK_PROCESS_CPUTIME_ID); }

struct job {
    int t, cur;                  /* cur: the vector of the next call */
    unsigned char *buf;          /* g_nvec vectors of BLOCKS x BLOCK_BYTES */
    const void **ptrs;           /* g_nvec x BLOCKS */
    uint32_t *lens;              /* BLOCKS (the same for every vector of a thread) */
    unsigned char *want, *got;   /* g_dsz-byte digests; want: g_nvec x BLOCKS */
    double *lat, *cpu;           /* per timed call */
    size_t ncalls, cap;
    int rc, bad;
};

static int one_call(struct job *j)
{
    const void **ptrs = j->ptrs + (size_t)j->cur * g_blocks;
    switch (g_target) {
    case T_BATCHER:
        return md5_batch_submit(g_b, ptrs, j->lens, (uint64_t)g_blocks, j->got);
    case T_POOL:
        return md5hip_pool_submit(g_p, ptrs, j->lens, (uint64_t)g_blocks, j->got);
    case T_HOST:
        for (int i = 0; i < g_blocks; i++) {
            if (g_crc >= 0) {               /* the library's host CRC-32 over the same windows */
                const unsigned char *p = ptrs[i];
                const uint32_t L = j->lens[i], F = (uint32_t)g_crc;
                const uint32_t c = !F || L <= F ? nc_crc32(p, L) : nc_crc32(p, F) ^ nc_crc32(p + L - F, F);
                memcpy(j->got + 4 * (size_t)i, &c, 4);
                continue;
            }
            struct MD5Context c;
            MD5Init(&c);
            MD5Update(&c, ptrs[i], j->lens[i]);
            MD5Final(j->got + 16 * (size_t)i, &c);
        }
        return 0;
    }
    return -EINVAL;
}

/* the call's digests against the oracle's for its vector; then the next vector */
static int check_next(struct job *j)
{
    const int bad = memcmp(j->got, j->want + (size_t)j->cur * g_blocks * g_dsz, g_dsz * (size_t)g_blocks) != 0;
    j->cur = (j->cur + 1) % g_nvec;
    return bad;
}

static void *worker(void *arg)
{
    struct job *j = arg;
    const size_t vec = (size_t)g_blocks * g_len;
    j->buf = malloc(vec * g_nvec + 64);
    j->ptrs = malloc(sizeof(void *) * g_blocks * g_nvec);
    j->lens = malloc(sizeof(uint32_t) * g_blocks);
    j->want = malloc(g_dsz * (size_t)g_blocks * g_nvec);
    j->got = malloc(g_dsz * (size_t)g_blocks);
    if (!j->buf || !j->ptrs || !j->lens || !j->want || !j->got) j->rc = -ENOMEM;
    if (!j->rc) {
        oracle_xorshift_fill(j->buf, vec * g_nvec + 64, 0x5A11ull + (uint64_t)j->t * 7919u);
        for (int i = 0; i < g_blocks; i++)   /* a short last block, as a vector's tail often is (blk_io.c:377) */
            j->lens[i] = i == g_blocks - 1 && g_blocks > 1 ? g_len - 1000u * (uint32_t)(1 + j->t % 7) : g_len;
        for (int v = 0; v < g_nvec; v++)
            for (int i = 0; i < g_blocks; i++) {
                const size_t k = (size_t)v * g_blocks + i;
                j->ptrs[k] = j->buf + v * vec + (size_t)i * g_len;
                if (g_crc >= 0) {
                    const uint32_t c = oracle_blk_crc(j->ptrs[k], j->lens[i], (uint32_t)g_crc);
                    memcpy(j->want + 4 * k, &c, 4);
                } else {
                    oracle_md5(j->ptrs[k], j->lens[i], j->want + 16 * k);
                }
            }
        if (g_register) j->rc = md5hip_host_register(j->buf, vec * g_nvec + 64);
    }
    pthread_barrier_wait(&g_start);
    for (int w = 0; w < 2 && !j->rc; w++) {               /* warm-up calls, checked */
        j->rc = one_call(j);
        if (!j->rc) j->bad += check_next(j);
    }
    pthread_barrier_wait(&g_warm);
    pthread_barrier_wait(&g_go);
    const double t_end = g_t_end;
    while (!j->rc && now() < t_end) {
        memset(j->got, 0, g_dsz * (size_t)g_blocks);
        const double c0 = thread_cpu(), t0 = now();
        const int rc = one_call(j);
        const double t1 = now(), c1 = thread_cpu();
        if (rc) {
            j->rc = rc;
            break;
        }
        j->bad += check_next(j);
        if (j->ncalls == j->cap) {
            j->cap = j->cap ? 2 * j->cap : 1024;
            j->lat = realloc(j->lat, sizeof(double) * j->cap);
            j->cpu = realloc(j->cpu, sizeof(double) * j->cap);
            if (!j->lat || !j->cpu) { j->rc = -ENOMEM; break; }
        }
        j->lat[j->ncalls] = (t1 - t0) * 1e6;
        j->cpu[j->ncalls] = (c1 - c0) * 1e6;
        j->ncalls++;
    }
    return NULL;
}

/* ASIO_FIXED_BG_MIB: host_fixed over a pageable array beside the callers */
struct bg {
    size_t bytes;
    unsigned char *buf;
    unsigned char (*want)[16], (*got)[16];
    double *lat;
    size_t ncalls, cap;
    int rc, bad;
};
static struct bg g_bg;

static void *bg_fixed(void *arg)
{
    struct bg *g = arg;
    const uint64_t n = g->bytes / 16384;
    pthread_barrier_wait(&g_go);
    const double t_end = g_t_end;
    while (!g->rc && now() < t_end) {
        memset(g->got, 0, 16 * n);
        const double t0 = now();
        const int rc = md5hip_batch_host_fixed(g_b, g->buf, n, 16384, 16384, &g->got[0][0]);
        const double t1 = now();
        if (rc) { g->rc = rc; break; }
        g->bad += memcmp(g->got, g->want, 16 * n) != 0;
        if (g->ncalls == g->cap) {
            g->cap = g->cap ? 2 * g->cap : 256;
            g->lat = realloc(g->lat, sizeof(double) * g->cap);
            if (!g->lat) { g->rc = -ENOMEM; break; }
        }
        g->lat[g->ncalls++] = (t1 - t0) * 1e6;
    }
    return NULL;
}

static int cmp_d(const void *a, const void *b)
{
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

static double pct(const double *v, size_t n, double p)
{
    if (!n) return 0;
    size_t k = (size_t)(p / 100.0 * (double)(n - 1) + 0.5);
    return v[k < n ? k : n - 1];
}

int main(int argc, char **argv)
{
    if (argc < 6) {
        fprintf(stderr, "usage: %s batcher|pool|host THREADS BLOCKS BLOCK_BYTES SECS [pageable|registered [SLICE_MIB NSLOTS]]\n",
                argv[0]);
        return 2;
    }
    g_target = !strcmp(argv[1], "pool") ? T_POOL : !strcmp(argv[1], "host") ? T_HOST : T_BATCHER;
    g_threads = atoi(argv[2]);
    g_blocks = atoi(argv[3]);
    g_len = (uint32_t)strtoul(argv[4], NULL, 0);
    g_secs = atof(argv[5]);
    g_register = argc > 6 && !strcmp(argv[6], "registered");
    const uint64_t slice = argc > 7 ? strtoull(argv[7], NULL, 0) << 20 : 0;
    const uint32_t nslots = argc > 8 ? (uint32_t)atoi(argv[8]) : 0;
    if (g_threads < 1 || g_threads > 1024 || g_blocks < 1 || g_len < 8000 || g_secs <= 0) return 2;
    {   /* all threads' vectors span >= 2 GiB (cold sources; ASIO_WS_MIB overrides) */
        const char *e = getenv("ASIO_WS_MIB");
        const double vec = (double)g_blocks * g_len, ws = (e ? atof(e) : 2048.0) * (1u << 20);
        g_nvec = (int)(ws / (vec * g_threads) + 0.999);
        if (g_nvec < 1) g_nvec = 1;
    }
    int rc = 0;
    {
        const char *e = getenv("ASIO_CRC");
        if (e && *e) {
            g_crc = atoi(e);
            g_dsz = 4;
        }
    }
    if (g_target == T_BATCHER) rc = md5hip_batcher_create(0, slice, nslots, &g_b);
    if (g_target == T_POOL) {
        const int devs[2] = {0, 0};
        rc = md5hip_pool_create(devs, 2, slice, nslots, &g_p);
    }
    if (rc == 0 && g_crc >= 0 && g_b) rc = md5hip_batcher_set_digest(g_b, MD5HIP_DIGEST_CRC32, (uint32_t)g_crc);
    if (rc == 0 && g_crc >= 0 && g_p) rc = md5hip_pool_set_digest(g_p, MD5HIP_DIGEST_CRC32, (uint32_t)g_crc);
    if (rc == -ENODEV) {
        printf("{\"error\": \"no usable HIP device\", \"rc\": %d}\n", rc);
        return 77;
    }
    if (rc) {
        printf("{\"error\": \"create\", \"rc\": %d}\n", rc);
        return 1;
    }
    {
        const char *e = getenv("ASIO_FIXED_BG_MIB");
        if (e && g_b && g_crc < 0) g_bg.bytes = (size_t)atoi(e) << 20;   /* MD5 runs only */
    }
    pthread_t bg_th;
    if (g_bg.bytes) {
        const uint64_t n = g_bg.bytes / 16384;
        g_bg.buf = malloc(g_bg.bytes);                     /* pageable */
        g_bg.want = malloc(16 * n);
        g_bg.got = malloc(16 * n);
        if (!g_bg.buf || !g_bg.want || !g_bg.got) return 1;
        oracle_xorshift_fill(g_bg.buf, g_bg.bytes, 0xB6ull);
        for (uint64_t i = 0; i < n; i++) oracle_md5(g_bg.buf + i * 16384, 16384, g_bg.want[i]);
    }
    const unsigned nbar = (unsigned)g_threads + 1 + (g_bg.bytes ? 1u : 0u);
    struct job *jobs = calloc((size_t)g_threads, sizeof *jobs);
    pthread_t *th = calloc((size_t)g_threads, sizeof *th);
    pthread_barrier_init(&g_start, NULL, (unsigned)g_threads + 1);
    pthread_barrier_init(&g_warm, NULL, (unsigned)g_threads + 1);
    pthread_barrier_init(&g_go, NULL, nbar);
    if (g_bg.bytes && pthread_create(&bg_th, NULL, bg_fixed, &g_bg)) return 1;
    pthread_attr_t at;
    pthread_attr_init(&at);
    pthread_attr_setstacksize(&at, 256u << 10);
    for (int t = 0; t < g_threads; t++) {
        jobs[t].t = t;
        if (pthread_create(&th[t], &at, worker, &jobs[t])) {
            printf("{\"error\": \"pthread_create\", \"thread\": %d}\n", t);
            return 1;
        }
    }
    pthread_barrier_wait(&g_start);               /* oracle digests done */
    pthread_barrier_wait(&g_warm);                /* warm-up calls done */
    struct rusage ru0, ru1;
    getrusage(RUSAGE_SELF, &ru0);
    const double p0 = process_cpu(), w0 = now();
    g_t_end = w0 + g_secs;
    pthread_barrier_wait(&g_go);                  /* (the barrier orders g_t_end) */
    for (int t = 0; t < g_threads; t++) pthread_join(th[t], NULL);
    if (g_bg.bytes) pthread_join(bg_th, NULL);
    const double wall = now() - w0, pcpu = process_cpu() - p0;
    getrusage(RUSAGE_SELF, &ru1);
    const double usr = (ru1.ru_utime.tv_sec - ru0.ru_utime.tv_sec) + (ru1.ru_utime.tv_usec - ru0.ru_utime.tv_usec) * 1e-6;
    const double sys = (ru1.ru_stime.tv_sec - ru0.ru_stime.tv_sec) + (ru1.ru_stime.tv_usec - ru0.ru_stime.tv_usec) * 1e-6;
    size_t total = 0;
    int bad = 0, err = 0;
    double bytes = 0;
    for (int t = 0; t < g_threads; t++) {
        total += jobs[t].ncalls;
        if (jobs[t].lens)
            for (int i = 0; i < g_blocks; i++) bytes += (double)jobs[t].ncalls * jobs[t].lens[i];
        bad += jobs[t].bad;
        if (jobs[t].rc && !err) err = jobs[t].rc;
    }
    double *lat = malloc(sizeof(double) * (total ? total : 1)), *cpu = malloc(sizeof(double) * (total ? total : 1));
    size_t k = 0;
    double cpu_sum = 0;
    for (int t = 0; t < g_threads; t++)
        for (size_t c = 0; c < jobs[t].ncalls; c++, k++) {
            lat[k] = jobs[t].lat[c];
            cpu[k] = jobs[t].cpu[c];
            cpu_sum += cpu[k];
        }
    qsort(lat, total, sizeof *lat, cmp_d);
    qsort(cpu, total, sizeof *cpu, cmp_d);
    struct md5hip_batcher_stats st = {0};
    if (g_b) md5hip_batcher_get_stats(g_b, &st);
    if (g_p) {
        struct md5hip_batcher_stats s2;
        for (uint32_t g = 0; g < 2; g++)
            if (md5hip_pool_device_stats(g_p, g, &s2) == 0) {
                st.launches += s2.launches;
                st.coalesced_launches += s2.coalesced_launches;
                if (s2.max_tickets_per_launch > st.max_tickets_per_launch)
                    st.max_tickets_per_launch = s2.max_tickets_per_launch;
            }
    }
    printf("{\"digest\": \"%s\", \"fastcrc\": %d, ", g_crc >= 0 ? "crc32" : "md5", g_crc >= 0 ? g_crc : 0);
    printf("\"target\": \"%s\", \"mode\": \"%s\", \"vectors_per_thread\": %d, \"threads\": %d, "
           "\"blocks\": %d, \"block_bytes\": %u, \"secs\": %.3f, "
           "\"calls\": %zu, \"lat_us\": {\"p50\": %.1f, \"p90\": %.1f, \"p99\": %.1f, \"max\": %.1f}, "
           "\"thread_cpu_us_per_call\": {\"mean\": %.2f, \"p50\": %.2f, \"p99\": %.2f}, "
           "\"process_cpu_us_per_call\": %.2f, \"process_cpu_cores\": %.2f, "
           "\"process_user_sys_us_per_call\": [%.2f, %.2f], \"gib_s\": %.3f, "
           "\"launches\": %llu, \"coalesced_launches\": %llu, \"max_tickets_per_launch\": %llu, "
           "\"mismatches\": %d, \"rc\": %d",
           argv[1], g_register ? "registered" : "pageable", g_nvec, g_threads, g_blocks, g_len, wall, total, pct(lat, total, 50), pct(lat, total, 90),
           pct(lat, total, 99), total ? lat[total - 1] : 0.0, total ? cpu_sum / (double)total : 0.0,
           pct(cpu, total, 50), pct(cpu, total, 99), total ? pcpu * 1e6 / (double)total : 0.0, pcpu / wall,
           total ? usr * 1e6 / (double)total : 0.0, total ? sys * 1e6 / (double)total : 0.0,
           bytes / wall / (double)(1u << 30), (unsigned long long)st.launches,
           (unsigned long long)st.coalesced_launches, (unsigned long long)st.max_tickets_per_launch, bad, err);
    if (g_bg.bytes) {
        qsort(g_bg.lat, g_bg.ncalls, sizeof *g_bg.lat, cmp_d);
        printf(", \"bg_fixed\": {\"mib\": %zu, \"calls\": %zu, \"lat_us\": {\"min\": %.1f, \"p50\": %.1f, "
               "\"max\": %.1f}, \"mismatches\": %d, \"rc\": %d}",
               g_bg.bytes >> 20, g_bg.ncalls, g_bg.ncalls ? g_bg.lat[0] : 0.0, pct(g_bg.lat, g_bg.ncalls, 50),
               g_bg.ncalls ? g_bg.lat[g_bg.ncalls - 1] : 0.0, g_bg.bad, g_bg.rc);
        bad += g_bg.bad;
        if (g_bg.rc && !err) err = g_bg.rc;
    }
    printf("}\n");
    if (g_b) md5hip_batcher_destroy(g_b);
    if (g_p) md5hip_pool_destroy(g_p);
    for (int t = 0; t < g_threads; t++) {
        if (g_register && jobs[t].buf) md5hip_host_unregister(jobs[t].buf);
        free(jobs[t].buf);
    }
    return bad || err || total == 0 ? 1 : 0;
}
