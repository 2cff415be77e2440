/*
 * host_san.c -- driver for the host-sanitizer build of liblstore_ec.so (tools/host_san.sh).
 *
 * The engine's host code (plan service, routes, pinning, staging, waits, segment read / write /
 * inspect, the network compiler's queue) built with -fsanitize=address,undefined on the host side
 * only (the GPU code objects are the ordinary ones: GPU sanitizers are not available on gfx950
 * boxes here), driven from C the way LStore drives it:
 *   CPU part (any host): method names, plan generation for every method incl. refused shapes,
 *     the self-tests behind the CPU test suite (waits, copies, bit-decode planner, DMA lattices,
 *     pinned budget, in-place stall guard), scatter-list straddle sizes.
 *   GPU part (when a device is visible): T threads per configuration calling the plan's
 *     encode_block / decode_block per stripe with the parity buffer malloc'd and freed around
 *     every call (segjerase_write_func, segment/jerasure.c:1689-1697, :1882), batched
 *     et_*_stripes, and a segment write -> read (a device missing, a corrupted record) ->
 *     inspect-and-fix round trip.  Checks are round trips (encode, erase, decode, compare); the
 *     parity itself is checked against the reference by the GPU suite, not here.
 * Prints one JSON line per part; exit status 0 only if every check held.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/uio.h>
#include <time.h>
#include <unistd.h>

#include "lstore_ec.h"

/* test hooks of the library (not in include/) */
int lsec_selftest_waits(int threads, int iters);
int lsec_selftest_copies(int cases, unsigned seed);
int lsec_selftest_bit_decode(int method, int k, int w);
int lsec_test_inplace_guard(int op, unsigned long long bytes, double drain_ms);
long long lsec_test_pinned_budget(int ndev, long long budget_mb, long long slot_mb, long long *server_mb);
int lsec_test_lattices(const uint64_t *dst, const uint64_t *src, const uint64_t *bytes, int n, int64_t *out,
                       int out_cap);
int lsec_test_jit_compile(int shape, int R, int K, int w, int packet, unsigned seed);

static int g_checks, g_fails;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;

#define CHECK(cond, ...)                                                         \
  do {                                                                           \
    pthread_mutex_lock(&g_mu);                                                   \
    ++g_checks;                                                                  \
    if (!(cond)) {                                                               \
      ++g_fails;                                                                 \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);                       \
      fprintf(stderr, __VA_ARGS__);                                              \
      fprintf(stderr, " (last error: %s)\n", lsec_last_error());                 \
    }                                                                            \
    pthread_mutex_unlock(&g_mu);                                                 \
  } while (0)

static uint64_t mix(uint64_t *s) { /* splitmix64 */
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static void fill(char *p, size_t n, uint64_t seed) {
  uint64_t s = seed;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t v = mix(&s);
    memcpy(p + i, &v, 8);
  }
  for (; i < n; ++i) p[i] = (char)mix(&s);
}

/* ------------------------------------------------------------------ CPU part */
static void cpu_part(void) {
  CHECK(et_method_type("reed_sol_van") == REED_SOL_VAN, "reed_sol_van");
  CHECK(et_method_type("CAUCHY_GOOD") == CAUCHY_GOOD, "case-insensitive name");
  CHECK(et_method_type("no_such_code") == -1, "unknown name");
  CHECK(nearest_prime(8, 0) > 0, "nearest_prime");

  static const int km[][2] = {{2, 1}, {4, 2}, {6, 3}, {10, 4}, {20, 6}, {40, 8}};
  int made = 0, refused = 0; /* refused: shapes the reference refuses too (w search fails) */
  for (int meth = 0; meth < N_JE_METHODS; ++meth)
    for (size_t i = 0; i < sizeof km / sizeof km[0]; ++i)
      for (long long C = 4096; C <= (4ll << 20); C *= 16) {
        const int k = km[i][0];
        const int m = meth == RAID4 ? 1 : meth == REED_SOL_R6_OP ? 2 : km[i][1];
        lio_erasure_plan_t *p = et_generate_plan((long long)k * C, meth, k, m, -1, -1, -1);
        if (!p) {
          ++refused;
          continue;
        }
        ++made;
        CHECK(p->form_encoding_matrix(p) == 0, "form_encoding_matrix %s(%d+%d)", JE_method[meth], k, m);
        CHECK(p->form_decoding_matrix(p) == 0, "form_decoding_matrix %s(%d+%d)", JE_method[meth], k, m);
        CHECK(p->data_strips == k && p->parity_strips == m, "plan shape");
        et_destroy_plan(p);
      }
  CHECK(made > 60, "plans made %d (refused %d)", made, refused);
  /* bad shapes: et_new_plan stores them as the reference does (erasure_tools.c:606-685), and
     form_encoding_matrix refuses them with a message instead of exiting */
  static const int bad[][4] = {{REED_SOL_VAN, 0, 3, 8}, {REED_SOL_VAN, 6, -1, 8}, {REED_SOL_VAN, 300, 3, 8},
                               {CAUCHY_GOOD, 6, 3, 3},  {LIBER8TION, 9, 2, 8}};
  for (size_t i = 0; i < sizeof bad / sizeof bad[0]; ++i) {
    lio_erasure_plan_t *p = et_new_plan(bad[i][0], 1 << 20, bad[i][1], bad[i][2], bad[i][3], 1024, 8);
    CHECK(p && p->form_encoding_matrix(p) != 0, "bad shape %d refused at form time", (int)i);
    et_destroy_plan(p);
  }

  CHECK(lsec_selftest_waits(1, 200) == 0, "waits 1");
  CHECK(lsec_selftest_waits(16, 100) == 0, "waits 16");
  CHECK(lsec_selftest_waits(128, 20) == 0, "waits 128");
  CHECK(lsec_selftest_waits(0, 1) == -1, "waits bad arguments");
  for (unsigned seed = 1; seed <= 3; ++seed) CHECK(lsec_selftest_copies(150, seed) == 0, "copies seed %u", seed);
  CHECK(lsec_selftest_bit_decode(LIBERATION, 7, 7) == 45, "liberation 7/7");
  CHECK(lsec_selftest_bit_decode(BLAUM_ROTH, 10, 10) == 78, "blaum-roth 10/10");
  CHECK(lsec_selftest_bit_decode(LIBER8TION, 8, 8) == 55, "liber8tion 8");
  CHECK(lsec_selftest_bit_decode(LIBERATION, 8, 7) == -1, "liberation k > w refused");

  { /* DMA lattices over a few runs at one stride */
    uint64_t dst[6], src[6], bytes[6];
    int64_t out[5 * 8]; /* five words per group */
    for (int i = 0; i < 6; ++i) {
      dst[i] = 0x100000 + (uint64_t)i * 0x20000;
      src[i] = 0x900000 + (uint64_t)i * 0x20000;
      bytes[i] = 0x10000;
    }
    CHECK(lsec_test_lattices(dst, src, bytes, 6, out, 8) == 1 && out[2] == 6, "lattices: one group of six rows");
  }
  {
    long long srv = 0;
    CHECK(lsec_test_pinned_budget(2, 1024, 9, &srv) >= 0, "pinned budget");
    CHECK(lsec_test_pinned_budget(0, 1024, 1, NULL) == -1, "pinned budget bad arguments");
  }
  { /* in-place stall guard: three stalls in a window suspend it, a reset lifts it */
    CHECK(lsec_test_inplace_guard(0, 0, 0) == 0, "guard reset");
    for (int i = 0; i < 3; ++i) lsec_test_inplace_guard(1, 8ull << 20, 40.0);
    CHECK(lsec_test_inplace_guard(2, 0, 0) == 1, "guard suspended");
    lsec_test_inplace_guard(0, 0, 0);
    CHECK(lsec_test_inplace_guard(2, 0, 0) == 0, "guard lifted");
  }
  { /* scatter-list straddles: pieces that cut stripes, an error page */
    lio_erasure_plan_t *p = et_generate_plan(6ll * 65536, REED_SOL_VAN, 6, 3, -1, -1, -1);
    CHECK(p != NULL, "plan for straddles");
    if (p) {
      const long long C = p->strip_size;
      char *a = malloc(6 * C * 3);
      struct iovec iov[4] = {{a, (size_t)(6 * C + 100)}, {NULL, (size_t)(3 * C)}, {a, (size_t)(3 * C - 100)},
                             {a, (size_t)(6 * C * 2)}};
      const long long st = lsec_segment_straddle_bytes(p, iov, 4, 3, (int)C);
      CHECK(st == 6 * C, "straddle bytes %lld", st); /* stripe 1 only */
      free(a);
      et_destroy_plan(p);
    }
  }
  if (getenv("LSEC_JITC")) { /* the network compiler's child and its queue, one shape per generator */
    CHECK(lsec_test_jit_compile(0, 6, 20, 8, 0, 7) == 0, "jit w=8");
    CHECK(lsec_test_jit_compile(3, 4, 10, 16, 32, 7) == 0, "jit cauchy w=16 packet");
    CHECK(lsec_test_jit_compile(9, 4, 10, 32, 0, 1) == -1, "jit bad shape");
  }
}

/* ------------------------------------------------------------------ GPU part */
typedef struct {
  int method, k, m, w;
  long long C;
  int packet; /* > 0: et_new_plan with this packet size (the bitmatrix codes), else et_generate_plan */
} config_t;

typedef struct {
  lio_erasure_plan_t *p;
  int id, iters;
  long long calls;
} worker_t;

static void erasure_set(int k, int m, int id, int *er) {
  int n = 0;
  er[n++] = id % k; /* a data shard */
  if (m > 1) er[n++] = k + (id % m); /* and a parity shard */
  er[n] = -1;
}

/* per-stripe calls as segjerase_write_func / jerase_control_check make them */
static void *worker(void *arg) {
  worker_t *w = arg;
  lio_erasure_plan_t *p = w->p;
  const int k = p->data_strips, m = p->parity_strips;
  const long long C = p->strip_size;
  char **ptr = calloc(k + m, sizeof(char *));
  char *data = malloc((size_t)k * C), *keep = malloc((size_t)(k + m) * C);
  for (int it = 0; it < w->iters; ++it) {
    fill(data, (size_t)k * C, (uint64_t)w->id * 1000003u + it);
    char *parity = malloc((size_t)m * C); /* the reference's per-op parity buffer */
    for (int i = 0; i < k; ++i) ptr[i] = data + (size_t)i * C;
    for (int r = 0; r < m; ++r) ptr[k + r] = parity + (size_t)r * C;
    p->encode_block(p, ptr, (int)C);
    memcpy(keep, data, (size_t)k * C);
    memcpy(keep + (size_t)k * C, parity, (size_t)m * C);
    int er[4];
    erasure_set(k, m, w->id + it, er);
    for (int e = 0; er[e] >= 0; ++e) memset(ptr[er[e]], 0xA5, (size_t)C);
    const int rc = p->decode_block(p, ptr, (int)C, er);
    CHECK(rc == 0, "decode_block rc %d", rc);
    int ok = 1;
    for (int e = 0; er[e] >= 0; ++e) ok &= memcmp(ptr[er[e]], keep + (size_t)er[e] * C, (size_t)C) == 0;
    CHECK(ok, "%s(%d+%d) C=%lld thread %d call %d: decode differs", JE_method[p->method], k, m, C, w->id, it);
    free(parity); /* freed right after the op, :1882 */
    ++w->calls;
  }
  free(ptr);
  free(data);
  free(keep);
  return NULL;
}

static long long batched(lio_erasure_plan_t *p, int nstripes) {
  const int k = p->data_strips, m = p->parity_strips, n = k + m;
  const long long C = p->strip_size;
  char *buf = malloc((size_t)nstripes * n * C), *keep = malloc((size_t)nstripes * n * C);
  char **ptrs = malloc(sizeof(char *) * nstripes * n);
  fill(buf, (size_t)nstripes * n * C, 99);
  for (int s = 0; s < nstripes; ++s)
    for (int i = 0; i < n; ++i) ptrs[s * n + i] = buf + ((size_t)s * n + i) * C;
  CHECK(et_encode_stripes(p, ptrs, nstripes, (int)C) == 0, "et_encode_stripes");
  char *magic = malloc(4 * (size_t)nstripes), *magic2 = malloc(4 * (size_t)nstripes);
  CHECK(et_encode_stripes_magic(p, ptrs, nstripes, (int)C, magic) == 0, "et_encode_stripes_magic");
  CHECK(et_stripes_magic(p, ptrs, nstripes, (int)C, magic2) == 0, "et_stripes_magic");
  CHECK(memcmp(magic, magic2, 4 * (size_t)nstripes) == 0, "magics agree");
  memcpy(keep, buf, (size_t)nstripes * n * C);
  int er[4];
  erasure_set(k, m, 1, er);
  for (int s = 0; s < nstripes; ++s)
    for (int e = 0; er[e] >= 0; ++e) memset(ptrs[s * n + er[e]], 0, (size_t)C);
  CHECK(et_decode_stripes(p, ptrs, nstripes, (int)C, er) == 0, "et_decode_stripes");
  CHECK(memcmp(buf, keep, (size_t)nstripes * n * C) == 0, "batched round trip %s(%d+%d)", JE_method[p->method], k, m);
  free(buf);
  free(keep);
  free(ptrs);
  free(magic);
  free(magic2);
  return nstripes;
}

static void segment_round_trip(lio_erasure_plan_t *p, int N) {
  const int k = p->data_strips, m = p->parity_strips, n = k + m;
  const int C = (int)p->strip_size;
  const size_t rec = (size_t)C + 4;
  char *data = malloc((size_t)N * k * C), *out = malloc((size_t)N * k * C);
  char **dev = malloc(sizeof(char *) * n);
  fill(data, (size_t)N * k * C, 7);
  for (int i = 0; i < n; ++i) dev[i] = calloc(N, rec);
  CHECK(lsec_segment_write(p, data, N, C, 1, 0, dev) == 0, "segment_write");
  int *status = calloc(N, sizeof(int));
  CHECK(lsec_segment_read(p, dev, N, C, 1, 0, 0, out, status) == 0, "segment_read clean");
  CHECK(memcmp(out, data, (size_t)N * k * C) == 0, "segment read back");
  char *lost = dev[0]; /* a device missing */
  dev[0] = NULL;
  memset(out, 0, (size_t)N * k * C);
  const int bad = lsec_segment_read(p, dev, N, C, 1, 0, 0, out, status);
  CHECK(bad == 0, "%s(%d+%d) w=%d C=%d: segment_read with device 0 missing: %d unrecoverable, status %d %d %d %d",
        JE_method[p->method], k, m, p->w, C, bad, status[0], status[1], status[2], status[N - 1]);
  CHECK(memcmp(out, data, (size_t)N * k * C) == 0, "%s(%d+%d): segment rebuilt without device 0",
        JE_method[p->method], k, m);
  dev[0] = lost;
  dev[1][4 + 17] ^= 0x40; /* silent corruption in stripe 0's record on device 1 */
  CHECK(lsec_segment_read(p, dev, N, C, 1, 0, LSEC_READ_PARANOID, out, status) == 0, "paranoid read");
  CHECK(memcmp(out, data, (size_t)N * k * C) == 0, "paranoid read repairs");
  /* inspect-and-fix over the stripe-major logical records (the LUN view: logical chunk j of
     stripe s on device (j - s) mod n at n_shift 1) */
  char *buf = malloc((size_t)N * n * rec);
  for (int s = 0; s < N; ++s)
    for (int j = 0; j < n; ++j) memcpy(buf + ((size_t)s * n + j) * rec, dev[((j - s) % n + n) % n] + (size_t)s * rec, rec);
  int *st = calloc(N, sizeof(int));
  unsigned char *badmap = calloc((size_t)N * n, 1), *rewrite = calloc((size_t)N * n, 1);
  lsec_inspect_state_t state;
  memset(&state, 0, sizeof state);
  CHECK(lsec_segment_inspect(p, buf, N, C, LSEC_INSPECT_FIX, st, badmap, rewrite, &state) == 0, "inspect");
  CHECK(st[0] != LSEC_STRIPE_OK && st[1] == LSEC_STRIPE_OK, "inspect finds stripe 0 (%d, %d)", st[0], st[1]);
  memset(&state, 0, sizeof state);
  CHECK(lsec_segment_inspect(p, buf, N, C, 0, st, badmap, rewrite, &state) == 0, "inspect after fix");
  int clean = 1;
  for (int s = 0; s < N; ++s) clean &= st[s] == LSEC_STRIPE_OK;
  CHECK(clean, "fixed records inspect clean");
  for (int i = 0; i < n; ++i) free(dev[i]);
  free(dev);
  free(data);
  free(out);
  free(status);
  free(buf);
  free(st);
  free(badmap);
  free(rewrite);
}

/* the scatter-list writes (segjerase_write_func's tbuf, :1786-1858): pieces cut at odd offsets,
   equal to the contiguous write; the hand-off form's parity and magics equal the images' records */
static void scatter_writes(lio_erasure_plan_t *p, int N) {
  const int k = p->data_strips, m = p->parity_strips, n = k + m;
  const int C = (int)p->strip_size;
  const size_t rec = (size_t)C + 4, total = (size_t)N * k * C;
  char *data = malloc(total);
  fill(data, total, 11);
  char **dev = malloc(sizeof(char *) * n), **dev2 = malloc(sizeof(char *) * n);
  for (int i = 0; i < n; ++i) {
    dev[i] = calloc(N, rec);
    dev2[i] = calloc(N, rec);
  }
  CHECK(lsec_segment_write(p, data, N, C, 0, 0, dev) == 0, "segment_write for the scatter check");
  struct iovec iov[8];
  const size_t cut[8] = {0, 1, (size_t)C - 3, (size_t)C * k + 5, (size_t)C * k + 4096, total / 2 + 7, total - 9, total};
  int niov = 0;
  for (int i = 0; i + 1 < 8; ++i)
    if (cut[i + 1] > cut[i]) iov[niov++] = (struct iovec){data + cut[i], cut[i + 1] - cut[i]};
  CHECK(lsec_segment_write_iov(p, iov, niov, N, C, 0, 0, dev2) == 0, "segment_write_iov");
  int same = 1;
  for (int i = 0; i < n; ++i) same &= memcmp(dev[i], dev2[i], (size_t)N * rec) == 0;
  CHECK(same, "%s(%d+%d): scatter write equals the contiguous write", JE_method[p->method], k, m);
  const long long sb = lsec_segment_straddle_bytes(p, iov, niov, N, C);
  char *parity = malloc((size_t)N * m * C), *magic = malloc(4 * (size_t)N), *straddle = malloc(sb > 0 ? sb : 1);
  struct iovec *out = malloc(sizeof(struct iovec) * 2 * n * N);
  const int got = lsec_segment_encode_iov(p, iov, niov, N, C, parity, magic, straddle, sb, out, 2 * n * N);
  CHECK(got == 2 * n * N, "segment_encode_iov returned %d", got);
  int ok = got == 2 * n * N;
  for (int s = 0; ok && s < N; ++s) {
    ok &= memcmp(magic + 4 * s, dev[0] + s * rec, 4) == 0;
    for (int r = 0; r < m; ++r) ok &= memcmp(parity + ((size_t)s * m + r) * C, dev[k + r] + s * rec + 4, C) == 0;
    for (int j = 0; j < n; ++j) /* [magic | chunk] iovecs in logical order */
      ok &= out[2 * (s * n + j)].iov_len == 4 && out[2 * (s * n + j) + 1].iov_len == (size_t)C &&
            memcmp(out[2 * (s * n + j) + 1].iov_base, dev[j] + s * rec + 4, C) == 0;
  }
  CHECK(ok, "%s(%d+%d): hand-off parity, magics and iovecs", JE_method[p->method], k, m);
  for (int i = 0; i < n; ++i) {
    free(dev[i]);
    free(dev2[i]);
  }
  free(dev);
  free(dev2);
  free(data);
  free(parity);
  free(magic);
  free(straddle);
  free(out);
}

/* et_encode / et_decode over files (erasure_tools.c:339-600) */
static void file_tools(lio_erasure_plan_t *p) {
  const int k = p->data_strips, m = p->parity_strips;
  const long long strip = p->strip_size, fsize = k * strip - 13, foff = 100, poff = 7;
  const char *tmp = getenv("TMPDIR") ? getenv("TMPDIR") : "/tmp";
  char dname[512], pname[512];
  snprintf(dname, sizeof dname, "%s/host_san_%d.data", tmp, (int)getpid());
  snprintf(pname, sizeof pname, "%s/host_san_%d.parity", tmp, (int)getpid());
  char *buf = malloc(foff + k * strip);
  memset(buf, '0', foff + k * strip);
  fill(buf + foff, fsize, 5);
  FILE *f = fopen(dname, "w");
  CHECK(f && fwrite(buf, 1, foff + fsize, f) == (size_t)(foff + fsize), "write %s", dname);
  if (f) fclose(f);
  remove(pname);
  CHECK(et_encode(p, dname, foff, pname, poff, 1 << 20) == 0, "et_encode");
  f = fopen(dname, "r+");
  if (f) { /* lose data strip 1 */
    fseek(f, foff + strip, SEEK_SET);
    for (long long i = 0; i < strip; ++i) fputc(0xEE, f);
    fclose(f);
  }
  int er[3] = {1, m > 1 ? k : -1, -1};
  CHECK(et_decode(p, foff + fsize, dname, foff, pname, poff, 1 << 20, er) == 0, "et_decode");
  char *back = malloc(foff + fsize);
  f = fopen(dname, "r");
  CHECK(f && fread(back, 1, foff + fsize, f) == (size_t)(foff + fsize), "read back");
  if (f) fclose(f);
  CHECK(memcmp(back + foff, buf + foff, fsize) == 0, "%s(%d+%d): file tools round trip", JE_method[p->method], k, m);
  remove(dname);
  remove(pname);
  free(buf);
  free(back);
}

/* small and large per-stripe calls side by side (the stripe server running while calls pinned in
   place release their registrations: servers_yield_begin / _end) */
typedef struct {
  lio_erasure_plan_t *p;
  double t_end;
  long calls;
} mixed_t;
static double now_s(void);
static void *mixed_worker(void *arg) {
  mixed_t *w = arg;
  lio_erasure_plan_t *p = w->p;
  const int k = p->data_strips, m = p->parity_strips;
  const size_t C = (size_t)p->strip_size;
  char *buf = malloc((size_t)(k + m) * C), *keep = malloc(C);
  char *ptr[32];
  fill(buf, (size_t)k * C, C + 3);
  for (int i = 0; i < k + m; ++i) ptr[i] = buf + (size_t)i * C;
  p->encode_block(p, ptr, (int)C);
  memcpy(keep, ptr[0], C);
  int er[2] = {0, -1};
  while (now_s() < w->t_end) {
    memset(ptr[0], 0x5C, C);
    const int rc = p->decode_block(p, ptr, (int)C, er);
    CHECK(rc == 0 && memcmp(ptr[0], keep, C) == 0, "mixed sizes: C=%zu decode", C);
    ++w->calls;
  }
  free(buf);
  free(keep);
  return NULL;
}
static void mixed_sizes(double secs) {
  lio_erasure_plan_t *ps = et_generate_plan(6 * 16384, CAUCHY_GOOD, 6, 3, -1, -1, -1);
  lio_erasure_plan_t *pl = et_generate_plan(6 << 20, CAUCHY_GOOD, 6, 3, -1, -1, -1);
  ps->form_encoding_matrix(ps), ps->form_decoding_matrix(ps);
  pl->form_encoding_matrix(pl), pl->form_decoding_matrix(pl);
  mixed_t w[4];
  pthread_t th[4];
  const double t_end = now_s() + secs;
  for (int i = 0; i < 4; ++i) {
    w[i] = (mixed_t){i < 2 ? ps : pl, t_end, 0};
    pthread_create(&th[i], NULL, mixed_worker, &w[i]);
  }
  for (int i = 0; i < 4; ++i) pthread_join(th[i], NULL);
  CHECK(w[0].calls + w[1].calls > 100 && w[2].calls + w[3].calls > 10, "mixed sizes progress: %ld small, %ld large",
        w[0].calls + w[1].calls, w[2].calls + w[3].calls);
  printf("{\"part\": \"mixed sizes\", \"small_calls\": %ld, \"large_calls\": %ld}\n", w[0].calls + w[1].calls,
         w[2].calls + w[3].calls);
  et_destroy_plan(ps);
  et_destroy_plan(pl);
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

static void gpu_part(int threads, int iters) {
  static const config_t cfg[] = {
      {REED_SOL_VAN, 6, 3, -1, 16384},   {REED_SOL_VAN, 6, 3, -1, 1 << 20}, {CAUCHY_GOOD, 6, 3, -1, 65536},
      {CAUCHY_GOOD, 10, 4, -1, 1 << 20}, {REED_SOL_R6_OP, 6, 2, -1, 65536}, {RAID4, 6, 1, -1, 65536},
      {LIBERATION, 6, 2, 7, 7 * 32 * 64, 32}, {BLAUM_ROTH, 6, 2, 6, 6 * 24 * 64, 24}, {LIBER8TION, 6, 2, -1, 65536},
      {CAUCHY_ORIG, 8, 4, -1, 65536},
      {REED_SOL_VAN, 10, 4, 16, 262144}, {CAUCHY_GOOD, 20, 6, -1, 262144}, {REED_SOL_VAN, 6, 3, -1, 4 << 20},
      {REED_SOL_VAN, 20, 6, -1, 262144}, /* a compiled w = 8 network once it is ready */
      {REED_SOL_VAN, 10, 4, 32, 262144}, {CAUCHY_GOOD, 10, 4, 16, 262144},
  };
  long long calls = 0, stripes = 0;
  const double t0 = now_s();
  for (size_t c = 0; c < sizeof cfg / sizeof cfg[0]; ++c) {
    const config_t *f = &cfg[c];
    lio_erasure_plan_t *p = f->packet > 0 ? et_new_plan(f->method, f->C, f->k, f->m, f->w, f->packet, 8)
                                          : et_generate_plan(f->k * f->C, f->method, f->k, f->m, f->w, -1, -1);
    CHECK(p != NULL, "plan %s(%d+%d) C=%lld", JE_method[f->method], f->k, f->m, f->C);
    if (!p) continue;
    p->form_encoding_matrix(p);
    p->form_decoding_matrix(p);
    CHECK(lsec_prepare_encode(p) == 0, "prepare_encode"); /* waits for a compiled network where one is made */
    pthread_t th[64];
    worker_t wk[64];
    const int T = threads < 64 ? threads : 64;
    const int its = f->C >= (1 << 20) ? (iters + 3) / 4 : iters;
    for (int t = 0; t < T; ++t) {
      wk[t] = (worker_t){p, t, its, 0};
      pthread_create(&th[t], NULL, worker, &wk[t]);
    }
    for (int t = 0; t < T; ++t) {
      pthread_join(th[t], NULL);
      calls += wk[t].calls;
    }
    stripes += batched(p, f->C >= (1 << 20) ? 8 : 64);
    if (f->k + f->m <= 32 && f->C <= (1 << 20)) {
      segment_round_trip(p, 9);
      scatter_writes(p, 5);
    }
    if (f->C <= (1 << 20)) file_tools(p);
    et_destroy_plan(p);
  }
  { /* one batched shape through every tile-dealing mode and a two-entry host device set */
    lio_erasure_plan_t *p = et_generate_plan(6ll << 20, REED_SOL_VAN, 6, 3, -1, -1, -1);
    p->form_encoding_matrix(p);
    p->form_decoding_matrix(p);
    const int mode0 = lsec_tile_sharing();
    for (int mode = 0; mode < 3; ++mode) {
      lsec_set_tile_sharing(mode);
      stripes += batched(p, 24);
    }
    lsec_set_tile_sharing(mode0);
    const int devs[2] = {0, 0};
    CHECK(lsec_set_host_devices(devs, 2) == 0, "host device set");
    stripes += batched(p, 48);
    CHECK(lsec_set_host_devices(NULL, 0) == 0, "host device set cleared");
    et_destroy_plan(p);
  }
  printf("{\"part\": \"gpu\", \"threads\": %d, \"per_stripe_calls\": %lld, \"batched_stripes\": %lld, "
         "\"seconds\": %.1f, \"checks\": %d, \"fails\": %d}\n",
         threads, calls, stripes, now_s() - t0, g_checks, g_fails);
  fflush(stdout);
}

int main(int argc, char **argv) {
  const int threads = argc > 1 ? atoi(argv[1]) : 4, iters = argc > 2 ? atoi(argv[2]) : 40;
  cpu_part();
  printf("{\"part\": \"cpu\", \"checks\": %d, \"fails\": %d}\n", g_checks, g_fails);
  fflush(stdout);
  if (lsec_device_count() > 0) {
    gpu_part(threads, iters);
    mixed_sizes(3.0);
    lsec_host_unpin_drain();
  }
  return g_fails ? 1 : 0;
}
