/*
 * tools/fnptr_bench.c -- the unmodified LStore call pattern, in C, against liblstore_ec.so,
 * with the reference (vendor/jerasure via oracle/_ref) timed the same way beside it.
 *
 * T pthreads share one plan and each calls plan->encode_block(plan, ptr, C) (or
 * plan->decode_block with data shard 0 lost) on its own host buffers, one stripe per call,
 * exactly as segjerase_write_func / jerase_control_check do from the gop pool
 * (src/lio/segment/jerasure.c:1847, :245, :1937).  The threads live for the whole run, like
 * the pool's: a warm-up phase (per-thread streams, slots, device images, galois tables), then a
 * timed phase of fixed duration between two barriers.  Runs last long enough (default 2 s) that
 * a CPU quota enforced per scheduler period (the GPU box grants 16 CPUs of a larger machine)
 * is what the threads get, not a burst.  Prints per-call latency percentiles and the aggregate
 * user-data rate as one JSON line per implementation.  Also a compile-time proof that a C
 * caller needs nothing but include/lstore_ec.h and -llstore_ec.
 *
 * build: gcc -O2 -o build/fnptr_bench tools/fnptr_bench.c -Iinclude -Llstore_amd -llstore_ec \
 *            -Wl,-rpath,'$ORIGIN/../lstore_amd' -lpthread -ldl
 * run:   build/fnptr_bench <chunk> <threads> <seconds> [method] [encode|decode]
 *        FNPTR_PINNED=1  each thread's buffer is page-locked (hipHostMalloc, looked up at run time
 *                        from libamdhip64.so), as an LStore cache that pins its pages would hold it
 *        FNPTR_REF=path  also time the reference: oracle/_ref/libjerasure_ref.so (test
 *                        infrastructure: the real jerasure behind erasure_tools.c's dispatch)
 *        FNPTR_ONLY_REF=1  time the reference only
 *        FNPTR_SET_MB=n  the threads' buffers together hold n MiB of stripes, and each thread
 *                        walks its own stripes round-robin, one per call (default: 4x the last-level
 *                        caches of the CPUs this process may run on, so neither implementation works
 *                        on cache-resident chunks; 0 = one stripe per thread, reused every call)
 *        FNPTR_VERIFY=1  (with FNPTR_REF) every timed engine call is checked: the chunks it writes
 *                        are overwritten before the call, and after it must equal the reference's
 *                        (parity for encode, the lost data chunk 0 for decode); the JSON line then
 *                        carries "verified" and "mismatches", and the exit status is 2 on any
 *        FNPTR_LAT_OUT=path  every timed call's latency (us), one line per call in call order
 *                        ("thread latency"), for joining with LSEC_TRACE's per-call phases
 *        FNPTR_FREE_AFTER=1  LStore's buffer lifetime: every encode writes its parity into a buffer
 *                        malloc'd for that call and freed right after it (segjerase_write_func:
 *                        segment/jerasure.c:1689-1697, free at :1882); every decode works on a stripe
 *                        buffer malloc'd for the call, filled from the thread's stripes (the bytes
 *                        the depots returned) and freed after it (the read path, :1621).
 *                        =2: the same with glibc's mmap threshold fixed at 128 KiB (mallopt), so
 *                        every buffer is a fresh mmap and every free an munmap: the next call's
 *                        buffer often lands at the addresses just unmapped, the case a
 *                        registration outliving its call would get wrong.  With FNPTR_VERIFY every
 *                        call's output is checked before the free.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <malloc.h>
#include <sched.h>
#include <pthread.h>
#include <sys/resource.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "lstore_ec.h"

#define MAX_SAMPLES 200000  /* latency samples kept per thread */

static lio_erasure_plan_t *g_plan;
static void *g_ref;  /* ref_plan_t* of oracle/_ref */
static void (*g_ref_encode)(void *, char **, int);
static int (*g_ref_decode)(void *, char **, int, int *);
static int (*g_host_malloc)(void **, size_t, unsigned);
static int (*g_host_free)(void *);
static int g_chunk, g_decode, g_use_ref, g_verify, g_free_after, g_k = 6, g_m = 3;
static long g_nbuf = 1;  /* stripes per thread (FNPTR_SET_MB) */
static double g_set_mb;
static long g_verified, g_mismatch;  /* FNPTR_VERIFY counters (atomic adds) */
static double g_seconds;
static volatile double g_t_end;
static pthread_barrier_t g_bar;

typedef struct {
    long t;
    long calls;
    double *lat;
    long nlat;
} thread_rec_t;

static double now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void one_call(char **ptr, int *erasures)
{
    if (g_use_ref) {
        if (g_decode) g_ref_decode(g_ref, ptr, g_chunk, erasures);
        else g_ref_encode(g_ref, ptr, g_chunk);
    } else {
        if (g_decode) g_plan->decode_block(g_plan, ptr, g_chunk, erasures);   /* segment/jerasure.c:245 */
        else g_plan->encode_block(g_plan, ptr, g_chunk);                      /* segment/jerasure.c:1847 */
    }
}

static void *worker(void *arg)
{
    thread_rec_t *r = (thread_rec_t *)arg;
    int k = g_k, m = g_m;
    char *buf = NULL;
    const size_t stripe = (size_t)(k + m) * g_chunk;
    const long nbuf = g_nbuf;
    if (g_host_malloc) {
        if (g_host_malloc((void **)&buf, stripe * nbuf, 0) != 0) buf = NULL;
    } else {
        buf = malloc(stripe * nbuf);
    }
    char *ptr[256];
    long cur = 0;
    int erasures[2] = {0, -1};
    char *gold = NULL;  /* FNPTR_VERIFY: the stripe with the reference's parity */
    const size_t C = (size_t)g_chunk;
    if (buf) {
        for (size_t i = 0; i < stripe; i++) buf[i] = (char)(i * 131 + r->t);
        for (long b = 1; b < nbuf; b++) memcpy(buf + b * stripe, buf, stripe);  /* every page touched */
        for (int i = 0; i < k + m; i++) ptr[i] = buf + (size_t)i * g_chunk;
        if (g_use_ref || g_verify) g_ref_encode(g_ref, ptr, g_chunk);   /* consistent parity for the decodes */
        else g_plan->encode_block(g_plan, ptr, g_chunk);
        if (g_verify && !g_use_ref) {
            gold = malloc((size_t)(k + m) * C);
            if (gold) memcpy(gold, buf, (size_t)(k + m) * C);
        }
        for (int c = 0; c < 3; c++) one_call(ptr, erasures);  /* warm */
    }
    pthread_barrier_wait(&g_bar);  /* timed phase starts */
    while (buf) {
        if (nbuf > 1) {  /* the next stripe of this thread's set */
            cur = cur + 1 == nbuf ? 0 : cur + 1;
            for (int i = 0; i < k + m; i++) ptr[i] = buf + cur * stripe + (size_t)i * g_chunk;
        }
        if (gold) {  /* overwrite what the call must write */
            if (g_decode) memset(ptr[0], 0xA5, C);
            else memset(ptr[k], 0x5A, (size_t)m * C);
        }
        char *own = NULL;  /* FNPTR_FREE_AFTER: this call's buffer, freed after the call */
        char *cptr[256];
        char **p = ptr;
        if (g_free_after) {
            memcpy(cptr, ptr, sizeof(char *) * (size_t)(k + m));
            if (g_decode) {  /* the stripe as read from the depots, into a buffer of its own */
                own = malloc((size_t)(k + m) * C);
                if (own) {
                    for (int i = 0; i < k + m; i++) {
                        cptr[i] = own + (size_t)i * C;
                        memcpy(cptr[i], ptr[i], C);
                    }
                    memset(cptr[0], 0xA5, C);
                }
            } else {  /* the parity buffer of one write op */
                own = malloc((size_t)m * C);
                if (own) {
                    for (int r2 = 0; r2 < m; r2++) cptr[k + r2] = own + (size_t)r2 * C;
                    memset(own, 0x5A, (size_t)m * C);
                }
            }
            if (!own) break;
            p = cptr;
        }
        double t0 = now();
        one_call(p, erasures);
        double t1 = now();
        if (gold) {
            const int bad = g_decode ? memcmp(p[0], gold, C) != 0 : memcmp(p[k], gold + (size_t)k * C, (size_t)m * C) != 0;
            __atomic_add_fetch(&g_verified, 1, __ATOMIC_RELAXED);
            if (bad) __atomic_add_fetch(&g_mismatch, 1, __ATOMIC_RELAXED);
        }
        free(own);
        if (r->nlat < MAX_SAMPLES) r->lat[r->nlat++] = t1 - t0;
        r->calls++;
        if (t1 >= g_t_end) break;
    }
    pthread_barrier_wait(&g_bar);  /* timed phase ends */
    if (buf) {
        if (g_host_malloc) g_host_free(buf);
        else free(buf);
    }
    free(gold);
    return NULL;
}

/* total last-level cache of the CPUs this process may run on (distinct index3 domains), bytes */
static double llc_bytes(void)
{
    cpu_set_t set;
    char seen[64][256];
    int nseen = 0;
    double total = 0;
    if (sched_getaffinity(0, sizeof(set), &set) != 0) return 256.0 * (1 << 20);
    for (int c = 0; c < CPU_SETSIZE; c++) {
        if (!CPU_ISSET(c, &set)) continue;
        char path[128], dom[256] = {0}, size[64] = {0};
        snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list", c);
        FILE *f = fopen(path, "r");
        if (!f) continue;
        if (!fgets(dom, sizeof(dom), f)) dom[0] = 0;
        fclose(f);
        int dup = 0;
        for (int i = 0; i < nseen && !dup; i++) dup = strcmp(seen[i], dom) == 0;
        if (dup || nseen == 64) continue;
        strcpy(seen[nseen++], dom);
        snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/cache/index3/size", c);
        if ((f = fopen(path, "r"))) {
            if (fgets(size, sizeof(size), f)) {
                double v = atof(size);
                total += strchr(size, 'M') ? v * (1 << 20) : strchr(size, 'K') ? v * 1024 : v;
            }
            fclose(f);
        }
    }
    return total > 0 ? total : 256.0 * (1 << 20);
}

static int cmp(const void *a, const void *b)
{
    double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

static double cpu_seconds(void)
{
    struct rusage ru;
    getrusage(RUSAGE_SELF, &ru);
    return ru.ru_utime.tv_sec + ru.ru_stime.tv_sec + 1e-6 * (ru.ru_utime.tv_usec + ru.ru_stime.tv_usec);
}

/* the cgroup's CPU throttling so far (cpu.stat throttled_usec; 0 without cgroup v2) */
static double throttled_seconds(void)
{
    FILE *f = fopen("/sys/fs/cgroup/cpu.stat", "r");
    char key[64];
    long long v;
    double t = 0;
    if (!f) return 0;
    while (fscanf(f, "%63s %lld", key, &v) == 2)
        if (strcmp(key, "throttled_usec") == 0) t = v * 1e-6;
    fclose(f);
    return t;
}

static void run(int T, const char *impl, const char *method)
{
    pthread_t th[1024];
    thread_rec_t rec[1024];
    const double stripe = (double)(g_k + g_m) * g_chunk;
    g_nbuf = g_verify ? 1 : (long)(g_set_mb * (1 << 20) / (T * stripe));
    if (g_nbuf < 1) g_nbuf = 1;
    pthread_barrier_init(&g_bar, NULL, T + 1);
    for (long t = 0; t < T; t++) {
        rec[t].t = t;
        rec[t].calls = 0;
        rec[t].nlat = 0;
        rec[t].lat = malloc(sizeof(double) * MAX_SAMPLES);
        pthread_create(&th[t], NULL, worker, &rec[t]);
    }
    g_t_end = now() + 1e9;
    pthread_barrier_wait(&g_bar);  /* every thread warmed up */
    double t0 = now(), c0 = cpu_seconds(), th0 = throttled_seconds();
    g_t_end = t0 + g_seconds;
    pthread_barrier_wait(&g_bar);  /* every thread done */
    double wall = now() - t0, cpu = cpu_seconds() - c0, thr = throttled_seconds() - th0;
    long calls = 0, n = 0;
    for (int t = 0; t < T; t++) {
        pthread_join(th[t], NULL);
        calls += rec[t].calls;
        n += rec[t].nlat;
    }
    const char *lat_out = getenv("FNPTR_LAT_OUT");
    if (lat_out && *lat_out) {  /* in call order, before the sort */
        FILE *f = fopen(lat_out, "w");
        if (f) {
            for (int t = 0; t < T; t++)
                for (long i = 0; i < rec[t].nlat; i++) fprintf(f, "%d %.2f\n", t, rec[t].lat[i] * 1e6);
            fclose(f);
        }
    }
    double *lat = malloc(sizeof(double) * (n ? n : 1));
    long o = 0;
    for (int t = 0; t < T; t++) {
        memcpy(lat + o, rec[t].lat, sizeof(double) * rec[t].nlat);
        o += rec[t].nlat;
        free(rec[t].lat);
    }
    qsort(lat, n, sizeof(double), cmp);
    double sum = 0;
    for (long i = 0; i < n; i++) sum += lat[i];
    pthread_barrier_destroy(&g_bar);
    printf("{\"impl\": \"%s\", \"op\": \"%s\", \"chunk\": %d, \"threads\": %d, \"calls\": %ld, \"seconds\": %.3f, "
           "\"method\": \"%s\", \"pinned\": %d, \"per_call_us_p50\": %.1f, "
           "\"per_call_us_p99\": %.1f, \"per_call_us_p999\": %.1f, \"per_call_us_max\": %.1f, \"per_call_us_mean\": %.1f, "
           "\"gibps\": %.3f, \"cpu_util\": %.2f, \"cpu_us_per_call\": %.1f, \"cgroup_throttled_ms\": %.1f, "
           "\"verified\": %ld, \"mismatches\": %ld, \"stripes_per_thread\": %ld, \"set_mib\": %.0f, \"free_after\": %d}\n",
           impl, g_decode ? "decode" : "encode", g_chunk, T, calls, wall, method, g_host_malloc != NULL,
           n ? lat[n / 2] * 1e6 : 0.0, n ? lat[(size_t)(n * 0.99)] * 1e6 : 0.0, n ? lat[(size_t)(n * 0.999)] * 1e6 : 0.0,
           n ? lat[n - 1] * 1e6 : 0.0, n ? sum / n * 1e6 : 0.0, calls * (double)g_k * g_chunk / wall / (1 << 30),
           cpu / wall, calls ? cpu / calls * 1e6 : 0.0, thr * 1e3, g_verified, g_mismatch, g_nbuf,
           g_nbuf * (double)T * stripe / (1 << 20), g_free_after);
    fflush(stdout);
    free(lat);
}

int main(int argc, char **argv)
{
    if (getenv("FNPTR_PINNED") && atoi(getenv("FNPTR_PINNED"))) {
        void *h = dlopen("libamdhip64.so", RTLD_NOW | RTLD_GLOBAL);
        if (h) {
            g_host_malloc = (int (*)(void **, size_t, unsigned))dlsym(h, "hipHostMalloc");
            g_host_free = (int (*)(void *))dlsym(h, "hipHostFree");
        }
        if (!g_host_malloc || !g_host_free) {
            fprintf(stderr, "FNPTR_PINNED: hipHostMalloc not found\n");
            return 1;
        }
    }
    g_chunk = argc > 1 ? atoi(argv[1]) : 16384;
    int T = argc > 2 ? atoi(argv[2]) : 8;
    g_seconds = argc > 3 ? atof(argv[3]) : 2.0;
    int method = argc > 4 ? et_method_type(argv[4]) : CAUCHY_GOOD;
    g_decode = argc > 5 && strcmp(argv[5], "decode") == 0;
    const char *set_mb = getenv("FNPTR_SET_MB");
    g_set_mb = set_mb ? atof(set_mb) : 4 * llc_bytes() / (1 << 20);
    if (T > 1024) T = 1024;
    if (T < 1) T = 1;
    g_plan = et_generate_plan((long long)g_k * g_chunk, method, g_k, g_m, -1, -1, -1);   /* :2237 */
    if (!g_plan || g_plan->form_encoding_matrix(g_plan) || g_plan->form_decoding_matrix(g_plan)) {
        fprintf(stderr, "plan: %s\n", lsec_last_error());
        return 1;
    }
    const char *only_ref = getenv("FNPTR_ONLY_REF");
    const char *ref_so = getenv("FNPTR_REF");
    g_verify = getenv("FNPTR_VERIFY") && atoi(getenv("FNPTR_VERIFY"));
    g_free_after = getenv("FNPTR_FREE_AFTER") ? atoi(getenv("FNPTR_FREE_AFTER")) : 0;
    if (g_free_after == 2) mallopt(M_MMAP_THRESHOLD, 128 * 1024);  /* fixed: every buffer is mmap'd */
    if (ref_so && *ref_so) {
        void *h = dlopen(ref_so, RTLD_NOW | RTLD_LOCAL);
        void *(*ref_new)(int, int, int, int, int) = h ? (void *(*)(int, int, int, int, int))dlsym(h, "ref_plan_new") : NULL;
        g_ref_encode = h ? (void (*)(void *, char **, int))dlsym(h, "ref_plan_encode") : NULL;
        g_ref_decode = h ? (int (*)(void *, char **, int, int *))dlsym(h, "ref_plan_decode") : NULL;
        if (!ref_new || !g_ref_encode || !g_ref_decode) {
            fprintf(stderr, "FNPTR_REF: cannot load %s\n", ref_so);
            return 1;
        }
        g_ref = ref_new(method, g_k, g_m, g_plan->w, g_plan->packet_size);
    } else if (g_verify) {
        fprintf(stderr, "FNPTR_VERIFY needs FNPTR_REF\n");
        return 1;
    }
    if (!(only_ref && atoi(only_ref))) run(T, "engine", JE_method[method]);
    const int bad = g_verify && (g_mismatch > 0 || g_verified == 0);
    if (g_ref && !g_verify) {
        g_use_ref = 1;
        run(T, "reference", JE_method[method]);
    }
    et_destroy_plan(g_plan);
    return bad ? 2 : 0;
}
