/*
 * oracle/ref_harness.c -- TEST INFRASTRUCTURE ONLY (never linked into the engine).
 *
 * A thin driver that is compiled together with the UNMODIFIED reference sources
 * under /root/reference/vendor/jerasure/src/{jerasure,galois,reed_sol,cauchy,liberation}.c
 * and /root/reference/src/lio/raid4.c into oracle/_ref/libjerasure_ref.so
 * (recipe: oracle/Makefile, target `ref`).  Nothing from the reference is
 * copied here; this file only *calls* the reference the way LStore's plan
 * service does.
 *
 * src/lio/erasure_tools.c itself cannot be built in this image: it includes
 * tbx/log.h -> tbx/iniparse.h -> apr_time.h and APR is not installed
 * (SURVEY.md §8c).  So the per-method dispatch of erasure_tools.c is
 * restated below (a handful of lines, each citing the line it mirrors), and
 * the packet-size search of et_generate_plan (erasure_tools.c:733-908) lives
 * in the oracle restatement (oracle/ec_oracle.c: eco_generate_plan) instead.
 *
 * Exports (all prefixed ref_):
 *   ref_plan_new / ref_plan_free          et_new_plan + form_encoding_matrix + form_decoding_matrix
 *   ref_plan_matrix / _bitmatrix / _schedule   read back what the reference built
 *   ref_plan_encode / ref_plan_decode     plan->encode_block / plan->decode_block
 *   ref_plan_encode_many / _decode_many   same over N stripes on T pthreads (CPU baseline)
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include "jerasure.h"
#include "galois.h"
#include "reed_sol.h"
#include "cauchy.h"
#include "liberation.h"
#include "raid4.h"

/* method ids: src/lio/erasure_tools.h:37-45 */
enum { M_RS_VAN = 0, M_RS_R6 = 1, M_CAUCHY_ORIG = 2, M_CAUCHY_GOOD = 3,
       M_BLAUM_ROTH = 4, M_LIBERATION = 5, M_LIBER8TION = 6, M_RAID4 = 7 };

typedef struct {
    int method, k, m, w, packet;
    int *matrix;      /* m*k, or NULL      */
    int *bitmatrix;   /* (m*w)*(k*w), or NULL */
    int **schedule;   /* -1 terminated op list, or NULL */
} ref_plan_t;

/* form_encoding_matrix followed by form_decoding_matrix, in that order, as
 * segment/jerasure.c:2242-2243 does.  Per-method builders:
 *   RS_VAN      erasure_tools.c:120-130  reed_sol_vandermonde_coding_matrix
 *   RS_R6       erasure_tools.c:108-116  reed_sol_r6_coding_matrix
 *   CAUCHY_*    erasure_tools.c:134-162, :210-244  matrix -> bitmatrix -> smart schedule
 *   liberation family  erasure_tools.c:166-204, :248-292
 *   RAID4       erasure_tools.c:101-104 (dummy) */
ref_plan_t *ref_plan_new(int method, int k, int m, int w, int packet)
{
    ref_plan_t *p = (ref_plan_t *)calloc(1, sizeof(*p));
    p->method = method; p->k = k; p->m = m; p->w = w; p->packet = packet;
    switch (method) {
    case M_RS_VAN:
        p->matrix = reed_sol_vandermonde_coding_matrix(k, m, w);
        break;
    case M_RS_R6:
        p->matrix = reed_sol_r6_coding_matrix(k, w);
        break;
    case M_CAUCHY_ORIG:
        p->matrix = cauchy_original_coding_matrix(k, m, w);
        p->bitmatrix = jerasure_matrix_to_bitmatrix(k, m, w, p->matrix);
        p->schedule = jerasure_smart_bitmatrix_to_schedule(k, m, w, p->bitmatrix);
        break;
    case M_CAUCHY_GOOD:
        p->matrix = cauchy_good_general_coding_matrix(k, m, w);
        p->bitmatrix = jerasure_matrix_to_bitmatrix(k, m, w, p->matrix);
        p->schedule = jerasure_smart_bitmatrix_to_schedule(k, m, w, p->bitmatrix);
        break;
    case M_BLAUM_ROTH:
        p->bitmatrix = blaum_roth_coding_bitmatrix(k, w);
        p->schedule = jerasure_smart_bitmatrix_to_schedule(k, m, w, p->bitmatrix);
        break;
    case M_LIBERATION:
        p->bitmatrix = liberation_coding_bitmatrix(k, w);
        p->schedule = jerasure_smart_bitmatrix_to_schedule(k, m, w, p->bitmatrix);
        break;
    case M_LIBER8TION:
        p->bitmatrix = liber8tion_coding_bitmatrix(k);
        p->schedule = jerasure_smart_bitmatrix_to_schedule(k, m, w, p->bitmatrix);
        break;
    case M_RAID4:
        break;
    default:
        free(p);
        return NULL;
    }
    return p;
}

void ref_plan_free(ref_plan_t *p)
{
    if (!p) return;
    free(p->matrix);
    free(p->bitmatrix);
    if (p->schedule) jerasure_free_schedule(p->schedule);
    free(p);
}

/* copy helpers: return element count, or -1 when the plan has no such object */
int ref_plan_matrix(ref_plan_t *p, int *out)
{
    if (!p->matrix) return -1;
    int n = p->k * p->m;
    if (p->method == M_RS_R6) n = 2 * p->k;
    memcpy(out, p->matrix, sizeof(int) * n);
    return n;
}

int ref_plan_bitmatrix(ref_plan_t *p, int *out)
{
    if (!p->bitmatrix) return -1;
    int n = p->k * p->m * p->w * p->w;
    memcpy(out, p->bitmatrix, sizeof(int) * n);
    return n;
}

/* schedule as a flat int[5*nops] array; returns nops (out may be NULL to count) */
int ref_plan_schedule(ref_plan_t *p, int *out)
{
    if (!p->schedule) return -1;
    int n = 0;
    for (; p->schedule[n][0] >= 0; n++)
        if (out) memcpy(out + 5 * n, p->schedule[n], 5 * sizeof(int));
    return n;
}

/* plan->encode_block dispatch: erasure_tools.c:299-326 + et_new_plan's table :627-675 */
void ref_plan_encode(ref_plan_t *p, char **ptr, int size)
{
    switch (p->method) {
    case M_RS_VAN:
        jerasure_matrix_encode(p->k, p->m, p->w, p->matrix, ptr, ptr + p->k, size);
        break;
    case M_RS_R6:
        reed_sol_r6_encode(p->k, p->w, ptr, ptr + p->k, size);
        break;
    case M_RAID4:
        raid4_encode(p->k, ptr, ptr + p->k, size);
        break;
    default:
        jerasure_schedule_encode(p->k, p->m, p->w, p->schedule, ptr, ptr + p->k, size, p->packet);
        break;
    }
}

/* plan->decode_block dispatch: erasure_tools.c:439-458 */
int ref_plan_decode(ref_plan_t *p, char **ptr, int size, int *erasures)
{
    switch (p->method) {
    case M_RS_VAN:
    case M_RS_R6:
        return jerasure_matrix_decode(p->k, p->m, p->w, p->matrix, 1, erasures, ptr, ptr + p->k, size);
    case M_RAID4:
        return raid4_decode(p->k, erasures, ptr, ptr + p->k, size);
    default:
        return jerasure_schedule_decode_lazy(p->k, p->m, p->w, p->bitmatrix, erasures,
                                             ptr, ptr + p->k, size, p->packet, 1);
    }
}

/* ---- multi-stripe driver for the CPU baseline: each thread owns a contiguous
 * stripe range, as the gop pool's per-op stripe ranges do (segment/jerasure.c:1937). */
typedef struct {
    ref_plan_t *p;
    char **ptrs;          /* nstripes*(k+m) pointers, stripe-major */
    int s0, s1, size, decode;
    int *erasures;
    int rc;
} ref_job_t;

static void *ref_worker(void *arg)
{
    ref_job_t *j = (ref_job_t *)arg;
    int km = j->p->k + j->p->m;
    j->rc = 0;
    for (int s = j->s0; s < j->s1; s++) {
        char **ptr = j->ptrs + (size_t)s * km;
        if (j->decode) {
            if (ref_plan_decode(j->p, ptr, j->size, j->erasures) != 0) j->rc = -1;
        } else {
            ref_plan_encode(j->p, ptr, j->size);
        }
    }
    return NULL;
}

static int ref_many(ref_plan_t *p, char **ptrs, int nstripes, int size, int nthreads,
                    int decode, int *erasures)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > nstripes) nthreads = nstripes;
    galois_create_mult_tables(p->w <= 8 ? 8 : p->w);  /* warm the lazily built tables */
    pthread_t *th = (pthread_t *)calloc(nthreads, sizeof(pthread_t));
    ref_job_t *jobs = (ref_job_t *)calloc(nthreads, sizeof(ref_job_t));
    int rc = 0;
    for (int t = 0; t < nthreads; t++) {
        jobs[t].p = p; jobs[t].ptrs = ptrs; jobs[t].size = size;
        jobs[t].decode = decode; jobs[t].erasures = erasures;
        jobs[t].s0 = (int)((long long)nstripes * t / nthreads);
        jobs[t].s1 = (int)((long long)nstripes * (t + 1) / nthreads);
        pthread_create(&th[t], NULL, ref_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        if (jobs[t].rc) rc = -1;
    }
    free(th);
    free(jobs);
    return rc;
}

int ref_plan_encode_many(ref_plan_t *p, char **ptrs, int nstripes, int size, int nthreads)
{
    return ref_many(p, ptrs, nstripes, size, nthreads, 0, NULL);
}

int ref_plan_decode_many(ref_plan_t *p, char **ptrs, int nstripes, int size, int nthreads,
                         int *erasures)
{
    return ref_many(p, ptrs, nstripes, size, nthreads, 1, erasures);
}

/* ---- config c1 plumbing: the per-stripe work of segjerase_write_func for a whole-stripe
 * aligned write (src/lio/segment/jerasure.c:1782-1855), restated without gop/tbx/IBP:
 *   ptr[0..k) -> user data, ptr[k..k+m) -> parity buffer   (:1809-1844)
 *   plan->encode_block(plan, ptr, C)                        (:1847)  -- real jerasure
 *   je_cksum_calc(magic, ptr, k+m, C): zlib adler32 over the k+m chunks, 4 bytes LE (:169-182)
 * and the LUN child's placement of the 2(k+m) [magic | chunk] iovecs: physical device i
 * stores logical chunk (i + s*n_shift) % (k+m) of stripe s at offset s*(C+4)
 * (lun_row_decompose, lun.c:1140-1246).  dev[i] holds nstripes*(C+4) bytes. */
void ref_segment_write(ref_plan_t *p, const char *data, int nstripes, int chunk, int n_shift,
                       long long first_stripe, char **dev)
{
    int k = p->k, m = p->m, n = k + m;
    size_t C = (size_t)chunk, lchunk = C + 4;
    char **ptr = (char **)malloc(sizeof(char *) * n);
    char *parity = (char *)malloc(C * m);
    for (int s = 0; s < nstripes; s++) {
        for (int j = 0; j < k; j++) ptr[j] = (char *)data + ((size_t)s * k + j) * C;
        for (int r = 0; r < m; r++) ptr[k + r] = parity + (size_t)r * C;
        ref_plan_encode(p, ptr, chunk);
        unsigned long ck = adler32(0L, Z_NULL, 0);
        for (int i = 0; i < n; i++) ck = adler32(ck, (unsigned char *)ptr[i], chunk);
        unsigned char magic[4];
        for (int i = 0; i < 4; i++) { magic[i] = ck & 255; ck >>= 8; }
        long long ss = first_stripe + s;
        for (int i = 0; i < n; i++) {
            int j = (int)((i + ss * n_shift) % n);
            char *slot = dev[i] + (size_t)s * lchunk;
            memcpy(slot, magic, 4);
            memcpy(slot + 4, ptr[j], C);
        }
    }
    free(parity);
    free(ptr);
}
