/* reserve_probe.c -- what the batcher's device-resident reserve pass
 * (md5_submit.c reserve_device) costs per chunk on the box's host, by how it
 * is run: one thread; parts on threads created per call (per-call calloc'd
 * histograms, as round 4's first try); parts on threads created per call with
 * preallocated histograms; parts handed to persistent helper threads.  The
 * destination is pinned coherent host memory (hipHostMallocCoherent) as in
 * the batcher, or plain malloc.  6 vectors of 79 K chunks of random C3-like
 * lengths (the c3q drained burst), median of 15 bursts.  Then one thread
 * writing into 4 slot-sized pinned regions in turn, as the batcher's slots
 * cycle (so the descriptor writes miss the caches), with ordinary and with
 * non-temporal stores.
 * usage: reserve_probe [threads]   (prints one JSON line) */
#include <hip/hip_runtime_api.h>
#include <immintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define KMAX (1u << 17)
enum { M = 78693, NV = 6, REPS = 15 };

static double now_ms(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec / 1e6;
}

struct part {
    const uint64_t *dp;
    const uint32_t *ln;
    uint64_t *ho;
    uint32_t *hl, *hh;
    uint64_t m, pay;
    uint32_t kmax;
};

static void *run(void *arg)
{
    struct part *p = arg;
    uint64_t pay = 0;
    uint32_t kmax = 0, last = UINT32_MAX;
    int uns = 0;
    for (uint64_t k = 0; k < p->m; k++) {
        const uint64_t q = p->dp[k];
        const uint32_t L = p->ln[k];
        p->ho[k] = q - 4096;
        p->hl[k] = L;
        pay += L;
        const uint32_t key = (L >> 6) + 1;
        uns |= key > last;
        last = key;
        if (key <= KMAX) {
            p->hh[key]++;
            if (key > kmax) kmax = key;
        }
    }
    p->pay = pay + (uint64_t)uns;
    p->kmax = kmax;
    return NULL;
}

static void *run_nt(void *arg)
{
    struct part *p = arg;
    uint64_t pay = 0;
    uint32_t kmax = 0, last = UINT32_MAX;
    int uns = 0;
    for (uint64_t k = 0; k < p->m; k++) {
        const uint64_t q = p->dp[k];
        const uint32_t L = p->ln[k];
        _mm_stream_si64((long long *)&p->ho[k], (long long)(q - 4096));
        _mm_stream_si32((int *)&p->hl[k], (int)L);
        pay += L;
        const uint32_t key = (L >> 6) + 1;
        uns |= key > last;
        last = key;
        if (key <= KMAX) {
            p->hh[key]++;
            if (key > kmax) kmax = key;
        }
    }
    _mm_sfence();
    p->pay = pay + (uint64_t)uns;
    p->kmax = kmax;
    return NULL;
}

/* persistent helpers */
static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t go = PTHREAD_COND_INITIALIZER, done = PTHREAD_COND_INITIALIZER;
static struct part *jobs[32];
static int gen_, ndone, quit;

static void *helper(void *arg)
{
    const int id = (int)(intptr_t)arg;
    int seen = 0;
    pthread_mutex_lock(&mu);
    for (;;) {
        while (gen_ == seen && !quit) pthread_cond_wait(&go, &mu);
        if (quit) break;
        seen = gen_;
        struct part *p = jobs[id];
        pthread_mutex_unlock(&mu);
        run(p);
        pthread_mutex_lock(&mu);
        if (++ndone == 0x7fffffff) ndone = 0;
        pthread_cond_signal(&done);
    }
    pthread_mutex_unlock(&mu);
    return NULL;
}

static int cmp(const void *a, const void *b)
{
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

int main(int argc, char **argv)
{
    const int T = argc > 1 ? atoi(argv[1]) : 4;
    uint64_t *dp = malloc(8 * (size_t)M);
    uint32_t *ln = malloc(4 * (size_t)M);
    uint64_t s = 88172645463325252ull, a = 1 << 20;
    for (int k = 0; k < M; k++) {
        s ^= s << 13, s ^= s >> 7, s ^= s << 17;
        const uint32_t L = 4096u << (s % 9);             /* 4 KiB .. 1 MiB */
        ln[k] = L - (uint32_t)((s >> 20) % 4096);
        dp[k] = a;
        a += (ln[k] + 15) & ~15ull;
    }
    uint64_t *ho_pin, *ho_mal = malloc(8 * (size_t)M * NV);
    uint32_t *hl_pin, *hl_mal = malloc(4 * (size_t)M * NV);
    if (hipHostMalloc((void **)&ho_pin, 8 * (size_t)M * NV, hipHostMallocCoherent) ||
        hipHostMalloc((void **)&hl_pin, 4 * (size_t)M * NV, hipHostMallocCoherent)) {
        printf("{\"error\": \"hipHostMalloc\"}\n");
        return 77;
    }
    uint32_t *hh = calloc(KMAX + 2, 4), *own[32];
    for (int t = 0; t < 32; t++) own[t] = calloc(KMAX + 2, 4);
    pthread_t hp[32];
    for (int t = 1; t < T; t++) pthread_create(&hp[t], NULL, helper, (void *)(intptr_t)t);
    const char *names[] = {"single", "create_calloc", "create_prealloc", "persistent"};
    printf("{\"chunks_per_vector\": %d, \"vectors\": %d, \"threads\": %d, \"ms_per_burst\": {", M, NV, T);
    for (int mem = 0; mem < 2; mem++) {
        uint64_t *HO = mem ? ho_mal : ho_pin;
        uint32_t *HL = mem ? hl_mal : hl_pin;
        for (int how = 0; how < 4; how++) {
            double ms[REPS];
            for (int r = 0; r < REPS; r++) {
                const double t0 = now_ms();
                for (int v = 0; v < NV; v++) {
                    struct part p[32];
                    pthread_t tid[32];
                    const int n = how ? T : 1;
                    for (int t = 0; t < n; t++) {
                        const uint64_t lo = (uint64_t)M * t / n, hi = (uint64_t)M * (t + 1) / n;
                        p[t] = (struct part){dp + lo, ln + lo, HO + (size_t)v * M + lo, HL + (size_t)v * M + lo,
                                             t ? own[t] : hh, hi - lo, 0, 0};
                        if (t && how == 1) p[t].hh = calloc(KMAX + 1, 4);
                        if (t && how <= 2) pthread_create(&tid[t], NULL, run, &p[t]);
                    }
                    if (how == 3) {
                        pthread_mutex_lock(&mu);
                        for (int t = 1; t < n; t++) jobs[t] = &p[t];
                        ndone = 0;
                        gen_++;
                        pthread_cond_broadcast(&go);
                        pthread_mutex_unlock(&mu);
                    }
                    run(&p[0]);
                    if (how == 3) {
                        pthread_mutex_lock(&mu);
                        while (ndone < n - 1) pthread_cond_wait(&done, &mu);
                        pthread_mutex_unlock(&mu);
                    }
                    for (int t = 1; t < n; t++) {
                        if (how <= 2) pthread_join(tid[t], NULL);
                        for (uint32_t k = 1; k <= p[t].kmax; k++) hh[k] += p[t].hh[k], p[t].hh[k] = 0;
                        if (how == 1) free(p[t].hh);
                    }
                }
                ms[r] = now_ms() - t0;
                memset(hh, 0, 4 * (KMAX + 2));
            }
            qsort(ms, REPS, sizeof(double), cmp);
            printf("%s\"%s_%s\": %.3f", mem || how ? ", " : "", mem ? "malloc" : "pinned", names[how], ms[REPS / 2]);
        }
    }
    /* 4 slot regions of NV * M descriptors, cycled per burst */
    uint64_t *cyc_o;
    uint32_t *cyc_l;
    if (hipHostMalloc((void **)&cyc_o, 8 * (size_t)M * NV * 4, hipHostMallocCoherent) ||
        hipHostMalloc((void **)&cyc_l, 4 * (size_t)M * NV * 4, hipHostMallocCoherent)) {
        printf("}}\n");
        return 77;
    }
    memset(cyc_o, 0, 8 * (size_t)M * NV * 4);
    memset(cyc_l, 0, 4 * (size_t)M * NV * 4);
    for (int nt = 0; nt < 2; nt++) {
        double ms[REPS];
        for (int r = 0; r < REPS; r++) {
            const size_t slot = (size_t)(r & 3) * M * NV;
            const double t0 = now_ms();
            for (int v = 0; v < NV; v++) {
                struct part p = {dp, ln, cyc_o + slot + (size_t)v * M, cyc_l + slot + (size_t)v * M, hh, M, 0, 0};
                if (nt) run_nt(&p);
                else run(&p);
            }
            ms[r] = now_ms() - t0;
            memset(hh, 0, 4 * (KMAX + 2));
        }
        qsort(ms, REPS, sizeof(double), cmp);
        printf(", \"pinned_4slots_%s\": %.3f", nt ? "nt" : "wb", ms[REPS / 2]);
    }
    printf("}}\n");
    pthread_mutex_lock(&mu);
    quit = 1;
    pthread_cond_broadcast(&go);
    pthread_mutex_unlock(&mu);
    for (int t = 1; t < T; t++) pthread_join(hp[t], NULL);
    return 0;
}
