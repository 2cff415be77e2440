/*
 * tools/fnptr_bench.c -- the unmodified LStore call pattern, in C, against liblstore_ec.so.
 *
 * T pthreads share one plan and each calls plan->encode_block(plan, ptr, C) on its own
 * host buffers, one stripe per call, exactly as segjerase_write_func does from the gop pool
 * (src/lio/segment/jerasure.c:1847, :1937).  Prints per-call latency percentiles and the
 * aggregate user-data rate.  Also a compile-time proof that a C caller needs nothing but
 * include/lstore_ec.h and -llstore_ec.
 *
 * build: gcc -O2 -o build/fnptr_bench tools/fnptr_bench.c -Iinclude -Llstore_amd -llstore_ec \
 *            -Wl,-rpath,'$ORIGIN/../lstore_amd' -lpthread
 * run:   build/fnptr_bench <chunk> <threads> <calls_per_thread> [method]
 *        FNPTR_PINNED=1: each thread's buffer is page-locked (hipHostMalloc, looked up at run
 *        time from libamdhip64.so), as an LStore cache that pins its pages would hold it
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "lstore_ec.h"

static lio_erasure_plan_t *g_plan;
static int (*g_host_malloc)(void **, size_t, unsigned);
static int (*g_host_free)(void *);
static int g_chunk, g_calls;
static double *g_lat;

static double now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void *worker(void *arg)
{
    long t = (long)arg;
    int k = g_plan->data_strips, m = g_plan->parity_strips;
    char *buf = NULL;
    if (g_host_malloc) {
        if (g_host_malloc((void **)&buf, (size_t)(k + m) * g_chunk, 0) != 0) buf = NULL;
    } else {
        buf = malloc((size_t)(k + m) * g_chunk);
    }
    if (!buf) return NULL;
    char *ptr[64];
    for (size_t i = 0; i < (size_t)(k + m) * g_chunk; i++) buf[i] = (char)(i * 131 + t);
    for (int i = 0; i < k + m; i++) ptr[i] = buf + (size_t)i * g_chunk;
    for (int c = 0; c < g_calls; c++) {
        double t0 = now();
        g_plan->encode_block(g_plan, ptr, g_chunk);     /* segment/jerasure.c:1847 */
        g_lat[t * g_calls + c] = now() - t0;
    }
    if (g_host_malloc) g_host_free(buf);
    else free(buf);
    return NULL;
}

static int cmp(const void *a, const void *b)
{
    double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
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
    g_calls = argc > 3 ? atoi(argv[3]) : 200;
    int method = argc > 4 ? et_method_type(argv[4]) : CAUCHY_GOOD;
    int k = 6, m = 3;
    g_plan = et_generate_plan((long long)k * g_chunk, method, k, m, -1, -1, -1);   /* :2237 */
    if (!g_plan || g_plan->form_encoding_matrix(g_plan) || g_plan->form_decoding_matrix(g_plan)) {
        fprintf(stderr, "plan: %s\n", lsec_last_error());
        return 1;
    }
    g_lat = calloc((size_t)T * g_calls, sizeof(double));
    pthread_t th[1024];
    { /* warm: staging, dispatcher, device images */
        g_calls = 2;
        for (long t = 0; t < T; t++) pthread_create(&th[t], NULL, worker, (void *)t);
        for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
        g_calls = argc > 3 ? atoi(argv[3]) : 200;
    }
    double t0 = now();
    for (long t = 0; t < T; t++) pthread_create(&th[t], NULL, worker, (void *)t);
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    double wall = now() - t0;
    size_t n = (size_t)T * g_calls;
    qsort(g_lat, n, sizeof(double), cmp);
    const char *kc = getenv("LSEC_KERNEL_COPY");
    printf("{\"chunk\": %d, \"threads\": %d, \"calls\": %zu, \"method\": \"%s\", \"pinned\": %d, \"kernel_copy\": \"%s\", "
           "\"per_call_us_p50\": %.1f, \"per_call_us_p99\": %.1f, \"gibps\": %.3f}\n", g_chunk, T, n, JE_method[method],
           g_host_malloc != NULL, kc ? kc : "default",
           g_lat[n / 2] * 1e6, g_lat[(size_t)(n * 0.99)] * 1e6, n * (double)k * g_chunk / wall / (1 << 30));
    et_destroy_plan(g_plan);
    free(g_lat);
    return 0;
}
