/*
 * oracle/cpu_baseline.c -- TEST/BENCH INFRASTRUCTURE ONLY.
 *
 * Times the host-core MD5 the way sproxy calls it (md5.h:41-51: one
 * MD5Init / MD5Update(len) / MD5Final per buffer, soluri2.c:711-713) over the
 * SURVEY.md §8(d) C1 workload: n x len bytes filled by xorshift64 (13/7/17)
 * from seed 0x9E3779B97F4A7C15, each u64 stored little-endian, contiguous.
 * Self-check: fold = fold*31 + byte over all digests (u32) -- 0x53a0a616 for
 * the full C1 set.
 *
 * Linked two ways by oracle/Makefile:
 *   _ref/md5_cpu_bench   against /root/reference/md5.c compiled in place
 *                        (cpu_baseline.kind = "reference")
 *   _build/md5_cpu_bench_port against oracle/md5_oracle.c ("port")
 * Only bench.py's cpu_baseline leg and the tests run these binaries.
 *
 * With -DCRC_MODE the same harness times netcache's block CRC-32 instead
 * (crc32_8bytes per chunk, crc32.c:186-240, as blk_make_crc calls it with
 * fastcrc = 0), 4-byte results, fold over those:
 *   _ref/crc32_cpu_bench        reference crc32.c compiled in place
 *   _build/crc32_cpu_bench_port oracle/crc32_oracle.c
 *
 * usage: md5_cpu_bench N LEN REPS THREADS   -> one JSON line on stdout
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#ifdef CRC_MODE
#include <stddef.h>
#ifdef USE_PORT
uint32_t oracle_crc32(const void *, uint64_t);
#define CRC_FN(p, n) oracle_crc32((p), (n))
#else
uint32_t crc32_8bytes(const void *data, size_t length);   /* reference crc32.c */
#define CRC_FN(p, n) crc32_8bytes((p), (n))
#endif
#define DSZ 4
#elif defined(USE_PORT)
struct oracle_md5_ctx { uint32_t s[4]; uint32_t b[2]; unsigned char in[64]; };
void oracle_md5_init(struct oracle_md5_ctx *);
void oracle_md5_update(struct oracle_md5_ctx *, const void *, unsigned);
void oracle_md5_final(unsigned char d[16], struct oracle_md5_ctx *);
#define CTX struct oracle_md5_ctx
#define H_INIT oracle_md5_init
#define H_UPDATE oracle_md5_update
#define H_FINAL oracle_md5_final
#define DSZ 16
#else
#include "md5.h"   /* /root/reference/md5.h via -I */
#define DSZ 16
#define CTX struct MD5Context
#define H_INIT MD5Init
#define H_UPDATE MD5Update
#define H_FINAL MD5Final
#endif

struct job { const unsigned char *data; unsigned char *dig; uint64_t lo, hi; unsigned len; };

static void *run_range(void *arg)
{
    struct job *j = (struct job *)arg;
    for (uint64_t i = j->lo; i < j->hi; i++) {
#ifdef CRC_MODE
        const uint32_t c = CRC_FN(j->data + i * (uint64_t)j->len, j->len);
        memcpy(j->dig + 4 * i, &c, 4);
#else
        CTX c;
        H_INIT(&c);
        H_UPDATE(&c, j->data + i * (uint64_t)j->len, j->len);
        H_FINAL(j->dig + 16 * i, &c);
#endif
    }
    return NULL;
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int cmp_d(const void *a, const void *b)
{
    double x = *(const double *)a, y = *(const double *)b;
    return (x > y) - (x < y);
}

int main(int argc, char **argv)
{
    uint64_t n = argc > 1 ? strtoull(argv[1], 0, 0) : 65536;
    unsigned len = argc > 2 ? (unsigned)strtoul(argv[2], 0, 0) : 16384;
    int reps = argc > 3 ? atoi(argv[3]) : 5;
    int threads = argc > 4 ? atoi(argv[4]) : 1;
    if (reps < 1) reps = 1;
    if (threads < 1) threads = 1;
    uint64_t bytes = n * (uint64_t)len;
    unsigned char *data = malloc(bytes + 8);
    unsigned char *dig = malloc(DSZ * n);
    double *t = malloc(sizeof(double) * reps);
    pthread_t *tid = malloc(sizeof(pthread_t) * threads);
    struct job *jobs = malloc(sizeof(struct job) * threads);
    if (!data || !dig || !t || !tid || !jobs) {
        fprintf(stderr, "oom\n");
        free(data); free(dig); free(t); free(tid); free(jobs);
        return 1;
    }
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (uint64_t off = 0; off < bytes; off += 8) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        for (int k = 0; k < 8; k++) data[off + k] = (unsigned char)(s >> (8 * k));
    }
    for (int r = 0; r < reps; r++) {
        double t0 = now_s();
        for (int k = 0; k < threads; k++) {
            jobs[k].data = data; jobs[k].dig = dig; jobs[k].len = len;
            jobs[k].lo = n * k / threads; jobs[k].hi = n * (k + 1) / threads;
            if (threads == 1) run_range(&jobs[k]);
            else pthread_create(&tid[k], NULL, run_range, &jobs[k]);
        }
        if (threads > 1)
            for (int k = 0; k < threads; k++) pthread_join(tid[k], NULL);
        t[r] = now_s() - t0;
    }
    uint32_t fold = 0;
    for (uint64_t i = 0; i < DSZ * n; i++) fold = fold * 31u + dig[i];
    qsort(t, reps, sizeof(double), cmp_d);
    double med = t[reps / 2];
    printf("{\"n\": %llu, \"len\": %u, \"reps\": %d, \"threads\": %d, "
           "\"median_s\": %.6f, \"min_s\": %.6f, \"gib_s\": %.6f, \"fold\": \"%08x\"}\n",
           (unsigned long long)n, len, reps, threads, med, t[0],
           (double)bytes / med / (double)(1ull << 30), fold);
    free(t); free(tid); free(jobs); free(data); free(dig);
    return 0;
}
