/* Development probe: per-stripe calls of two sizes in one process, as an LStore process serving
 * segments with different chunk sizes does.  S threads keep making 16 KiB Cauchy-good(6+3) decodes
 * (the stripe server's route: a persistent kernel on the device) for `secs` seconds; L threads
 * make 1 MiB decodes (pinned in place and DMA'd, released with hipHostUnregister, which waits
 * until the device is idle) over the same window.  Prints one JSON line: per size, calls and the
 * p50 / p99 / max call time.  The S threads stop at `secs`, so a release that waits for the
 * server to retire ends then at the latest.
 * Build: gcc -O2 -o build/mixed_sizes_probe tools/probes/mixed_sizes_probe.c -Iinclude -Llstore_amd -llstore_ec
 *        -Wl,-rpath,$ORIGIN/../lstore_amd -lpthread
 * Run:   build/mixed_sizes_probe [S threads] [L threads] [secs] */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "lstore_ec.h"

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

typedef struct {
  lio_erasure_plan_t *p;
  double t_end;
  double *lat;
  long n, cap;
  int bad;
} worker_t;

static void *run(void *arg) {
  worker_t *w = arg;
  const int k = w->p->data_strips, m = w->p->parity_strips;
  const size_t C = (size_t)w->p->strip_size;
  enum { NBUF = 8 };
  char *buf = malloc(NBUF * (k + m) * C);
  for (size_t i = 0; i < NBUF * (k + m) * C; ++i) buf[i] = (char)(i * 131 + 7);
  char *ptr[32];
  int er[2] = {0, -1};
  for (int b = 0; b < NBUF; ++b) {
    for (int i = 0; i < k + m; ++i) ptr[i] = buf + ((size_t)b * (k + m) + i) * C;
    w->p->encode_block(w->p, ptr, (int)C);
  }
  char *keep = malloc(C);
  for (long it = 0; now() < w->t_end; ++it) {
    const int b = (int)(it % NBUF);
    for (int i = 0; i < k + m; ++i) ptr[i] = buf + ((size_t)b * (k + m) + i) * C;
    memcpy(keep, ptr[0], C);
    memset(ptr[0], 0xA5, C);
    const double t0 = now();
    if (w->p->decode_block(w->p, ptr, (int)C, er) != 0) w->bad++;
    const double t1 = now();
    if (memcmp(keep, ptr[0], C) != 0) w->bad++;
    if (w->n < w->cap) w->lat[w->n++] = (t1 - t0) * 1e6;
  }
  free(keep);
  free(buf);
  return NULL;
}

static int cmp(const void *a, const void *b) {
  const double x = *(const double *)a, y = *(const double *)b;
  return x < y ? -1 : x > y;
}

static void report(const char *name, worker_t *w, int n) {
  long tot = 0, bad = 0;
  for (int i = 0; i < n; ++i) tot += w[i].n, bad += w[i].bad;
  double *all = malloc(sizeof(double) * (tot ? tot : 1));
  long j = 0;
  for (int i = 0; i < n; ++i)
    for (long c = 0; c < w[i].n; ++c) all[j++] = w[i].lat[c];
  qsort(all, tot, sizeof(double), cmp);
  printf("\"%s\": {\"threads\": %d, \"calls\": %ld, \"bad\": %ld, \"p50_us\": %.0f, \"p99_us\": %.0f, \"max_us\": %.0f}", name, n,
         tot, bad, tot ? all[tot / 2] : 0, tot ? all[(long)(0.99 * (tot - 1))] : 0, tot ? all[tot - 1] : 0);
  free(all);
}

int main(int argc, char **argv) {
  const int ns = argc > 1 ? atoi(argv[1]) : 4, nl = argc > 2 ? atoi(argv[2]) : 1;
  const double secs = argc > 3 ? atof(argv[3]) : 4.0;
  lio_erasure_plan_t *ps = et_generate_plan(6 * 16384, CAUCHY_GOOD, 6, 3, -1, -1, -1);
  lio_erasure_plan_t *pl = et_generate_plan(6 << 20, CAUCHY_GOOD, 6, 3, -1, -1, -1);
  if (!ps || !pl) {
    fprintf(stderr, "plan: %s\n", lsec_last_error());
    return 1;
  }
  ps->form_encoding_matrix(ps), ps->form_decoding_matrix(ps);
  pl->form_encoding_matrix(pl), pl->form_decoding_matrix(pl);
  worker_t ws[64], wl[64];
  pthread_t ts[64], tl[64];
  const double t_end = now() + secs;
  for (int i = 0; i < ns; ++i) {
    ws[i] = (worker_t){ps, t_end, malloc(sizeof(double) * 2000000), 0, 2000000, 0};
    pthread_create(&ts[i], NULL, run, &ws[i]);
  }
  for (int i = 0; i < nl; ++i) {
    wl[i] = (worker_t){pl, t_end, malloc(sizeof(double) * 200000), 0, 200000, 0};
    pthread_create(&tl[i], NULL, run, &wl[i]);
  }
  for (int i = 0; i < ns; ++i) pthread_join(ts[i], NULL);
  for (int i = 0; i < nl; ++i) pthread_join(tl[i], NULL);
  printf("{\"secs\": %.1f, ", secs);
  report("small_16k", ws, ns);
  printf(", ");
  report("large_1m", wl, nl);
  printf("}\n");
  return 0;
}
