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

/* segjerase_write_func's user-buffer handling (segment/jerasure.c:1786-1825) restated: the
 * data arrives as a scatter list of n_iov pieces (the cache pages of the tbuf; base NULL = an
 * error page).  For each stripe of k*C bytes, as tbx_tbuf_next sees it:
 *   - inside one piece (tbv.n_iov == 1): the data chunk pointers point into it (:1818-1819);
 *   - straddling pieces: the bytes are first copied into a contiguous buffer (:1795-1811) and
 *     the chunk pointers point into that copy (:1820-1821);
 *   - a stripe whose first piece is an error page: every data chunk pointer is a zero chunk
 *     (:1816, :1823-1831) -- zeros are encoded and written.
 * Error pages inside a straddling stripe (after its first piece) read as zeros here: the
 * reference's tbx_tbuf_copy would read through the NULL base. */
void ref_segment_write_iov(ref_plan_t *p, char **iov_base, const long long *iov_len, int n_iov, int nstripes,
                           int chunk, int n_shift, long long first_stripe, char **dev)
{
    int k = p->k, m = p->m, n = k + m;
    size_t C = (size_t)chunk, lchunk = C + 4, dsize = (size_t)k * C;
    char **ptr = (char **)malloc(sizeof(char *) * n);
    char *parity = (char *)malloc(C * m);
    char *straddle = (char *)malloc(dsize);
    char *empty = (char *)calloc(1, C);
    int pi = 0;              /* piece holding byte `off` */
    long long pstart = 0;    /* offset of piece pi */
    for (int s = 0; s < nstripes; s++) {
        long long off = (long long)s * (long long)dsize;
        while (pi < n_iov && pstart + iov_len[pi] <= off) pstart += iov_len[pi++];
        if (pi >= n_iov) break;  /* scatter list shorter than the stripes: nothing more to write */
        char *base;
        if (iov_base[pi] == NULL) {
            for (int j = 0; j < k; j++) ptr[j] = empty;
        } else {
            if (pstart + iov_len[pi] >= off + (long long)dsize) {
                base = iov_base[pi] + (off - pstart);
            } else {
                size_t got = 0;
                int q = pi;
                long long qs = pstart;
                while (got < dsize && q < n_iov) {
                    long long from = off + (long long)got - qs;
                    size_t take = (size_t)(iov_len[q] - from);
                    if (take > dsize - got) take = dsize - got;
                    if (iov_base[q]) memcpy(straddle + got, iov_base[q] + from, take);
                    else memset(straddle + got, 0, take);
                    got += take;
                    qs += iov_len[q++];
                }
                if (got < dsize) memset(straddle + got, 0, dsize - got);
                base = straddle;
            }
            for (int j = 0; j < k; j++) ptr[j] = base + (size_t)j * C;
        }
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
    free(empty);
    free(straddle);
    free(parity);
    free(ptr);
}

/* ---------------------------------------------------------------- verification / repair
 * The segment's verification helpers, restated over the real jerasure decode (ref_plan_decode)
 * and zlib, since segment/jerasure.c cannot be built here:
 *   h_cksum / h_cksum_cmp   je_cksum_calc / je_cksum_compare   (segment/jerasure.c:169-194)
 *   h_control_check         jerase_control_check               (:202-269)
 *   h_brute_recurse         jerase_brute_recurse               (:271-314)
 *   h_brute_recovery        jerase_brute_recovery              (:321-339)
 * ptr / eptr / pwork have the reference's roles: decode_block rebuilds the erased devices
 * through eptr, which aliases ptr (the stripe buffer) except for control chunks and the
 * brute-force work buffers. */
static void h_cksum(unsigned char *magic, char **ptr, int n, int C)
{
    unsigned long ck = adler32(0L, Z_NULL, 0);
    for (int i = 0; i < n; i++) ck = adler32(ck, (unsigned char *)ptr[i], C);
    for (int i = 0; i < 4; i++) { magic[i] = ck & 255; ck >>= 8; }
}

static int h_cksum_cmp(const unsigned char *magic, char **ptr, int n, int C)
{
    unsigned char calc[4];
    h_cksum(calc, ptr, n, C);
    return memcmp(magic, calc, 4) == 0 ? 0 : 1;
}

static int h_control_check(ref_plan_t *p, int C, int n, int m, int *badmap, char **ptr, char **eptr, char **pwork,
                           const unsigned char *magic)
{
    int erasures[n + 1], control[m + 1];
    int nbad = 0;
    for (int i = 0; i < n; i++) nbad += badmap[i];
    if (magic && nbad == 0) return h_cksum_cmp(magic, ptr, n, C);   /* nothing to rebuild */
    int n_ctl_max = magic ? 0 : m - nbad;
    int control_index = -1, errors = 0;
    do {
        memcpy(eptr, ptr, sizeof(char *) * n);
        int nc = 0, ne = 0;
        for (int i = 0; i < n; i++) {
            int take_ctl = !badmap[i] && nc < n_ctl_max && i > control_index;
            if (!take_ctl && !badmap[i]) continue;
            erasures[ne++] = i;
            if (take_ctl) { control[nc] = i; eptr[i] = pwork[nc]; nc++; control_index = i; }
        }
        erasures[ne] = -1;
        ref_plan_decode(p, eptr, C, erasures);
        if (magic) return h_cksum_cmp(magic, eptr, n, C);
        if (nc <= 0) {
            if (n_ctl_max > 0) control_index = n - 1;
            else return 0;                           /* m devices bad: nothing to compare */
        }
        for (int i = 0; i < nc; i++)
            if (memcmp(ptr[control[i]], eptr[control[i]], C) != 0) return ++errors;
    } while (control_index < n - 1);
    return errors;
}

static int h_brute_recurse(int level, int *index, ref_plan_t *p, int C, int n, int m, int nbad, int *badmap, char **ptr,
                           char **eptr, char **pwork, const unsigned char *magic)
{
    if (level == nbad) {   /* the combination is complete: swap in work buffers and check */
        char *saved[m + 1];
        memset(badmap, 0, sizeof(int) * n);
        for (int i = 0; i < nbad; i++) { saved[i] = ptr[index[i]]; ptr[index[i]] = pwork[i]; badmap[index[i]] = 1; }
        int r = h_control_check(p, C, n, m, badmap, ptr, eptr, pwork + nbad, magic);
        for (int i = 0; i < nbad; i++) ptr[index[i]] = saved[i];
        return r;
    }
    for (int i = level == 0 ? 0 : index[level - 1] + 1; i < n; i++) {
        index[level] = i;
        if (h_brute_recurse(level + 1, index, p, C, n, m, nbad, badmap, ptr, eptr, pwork, magic) == 0) return 0;
    }
    return 1;
}

static int h_brute_recovery(ref_plan_t *p, int C, int n, int m, int *badmap, char **ptr, char **eptr, char **pwork,
                            const unsigned char *magic)
{
    int index[m + 1];
    if (h_control_check(p, C, n, m, badmap, ptr, eptr, pwork, magic) == 0) return 0;   /* the given badmap */
    memset(badmap, 0, sizeof(int) * n);
    int ncheck = magic ? m + 1 : m;   /* with magic no control chunk is needed */
    for (int e = 1; e < ncheck; e++) {
        memset(index, 0, sizeof(index));
        if (h_brute_recurse(0, index, p, C, n, m, e, badmap, ptr, eptr, pwork, magic) == 0) return 0;
    }
    return 1;
}

/* majority vote over the n magics at mag[j] (first group with the largest count wins):
 * fills badmap with the devices outside the quorum, returns the quorum's count */
static int h_quorum(int n, unsigned char **mag, int *badmap, unsigned char *qmagic)
{
    int group[n], count[n], ng = 0;
    unsigned char *key[n];
    for (int j = 0; j < n; j++) {
        int g = 0;
        while (g < ng && memcmp(key[g], mag[j], 4) != 0) g++;
        if (g == ng) { key[ng] = mag[j]; count[ng] = 0; ng++; }
        count[g]++;
        group[j] = g;
    }
    int best = 0;
    for (int g = 1; g < ng; g++) if (count[g] > count[best]) best = g;
    for (int j = 0; j < n; j++) badmap[j] = group[j] != best;
    memcpy(qmagic, key[best], 4);
    return count[best];
}

static int h_nonzero(const char *b, int C) { for (int i = 0; i < C; i++) if (b[i]) return 1; return 0; }

/* segjerase_inspect_full_func's per-stripe loop (segment/jerasure.c:473-660) over one
 * buffer: nstripes x (k+m) records of [4-byte magic | chunk].  status[s] uses the engine's
 * LSEC_STRIPE_* numbering (0 ok, 1 empty, 2 bad magic, 3 repaired, 4 lost: magic,
 * 5 lost: mismatch); badmap_out / rewrite as lsec_segment_inspect documents.
 * counters[4] += bad_count, unrecoverable_count, erasure_errors, n_empty;
 * brute[0] / brute[1..n] = bm_brute_used / badmap_brute, carried between calls. */
void ref_segment_inspect(ref_plan_t *p, char *buf, int nstripes, int chunk, int magic_cksum, int do_fix, int *status,
                         unsigned char *badmap_out, unsigned char *rewrite, long long *counters, int *brute)
{
    int k = p->k, m = p->m, n = k + m, C = chunk;
    size_t rec = (size_t)C + 4;
    int badmap[n];
    char *ptr[n], *eptr[n], *pwork[m];
    unsigned char *mag[n], qmagic[4], zero[4] = {0, 0, 0, 0};
    char *parity = (char *)malloc((size_t)m * C);
    for (int i = 0; i < m; i++) pwork[i] = parity + (size_t)i * C;
    memset(rewrite, do_fix && !magic_cksum ? 1 : 0, (size_t)nstripes * n);   /* legacy: whole range (:464-470) */
    for (int s = 0; s < nstripes; s++) {
        char *b = buf + (size_t)s * n * rec;
        for (int j = 0; j < n; j++) { mag[j] = (unsigned char *)(b + j * rec); ptr[j] = b + j * rec + 4; }
        int count = h_quorum(n, mag, badmap, qmagic);
        int good_magic = memcmp(zero, qmagic, 4) != 0, skip = 0, st;
        if (!good_magic) {
            int nz = 0;
            for (int j = 0; j < n && !nz; j++) nz = h_nonzero(ptr[j], C);
            if (nz) good_magic = 1;
            else if (count == n) { counters[3]++; status[s] = 1;
                                   for (int j = 0; j < n; j++) badmap_out[(size_t)s * n + j] = badmap[j]; continue; }
        }
        const unsigned char *check_magic = magic_cksum ? qmagic : NULL;
        if ((!good_magic && count != n) || count < k) {
            counters[1]++; counters[0]++;
            st = 4;
        } else {
            if (h_control_check(p, C, n, m, badmap, ptr, eptr, pwork, check_magic) != 0) {
                counters[0]++; counters[2]++;
                if (brute[0]) for (int j = 0; j < n; j++) badmap[j] = brute[1 + j];
                if (h_brute_recovery(p, C, n, m, badmap, ptr, eptr, pwork, check_magic) == 0) {
                    brute[0] = 1;
                    for (int j = 0; j < n; j++) brute[1 + j] = badmap[j];
                    st = 3;
                } else {
                    st = 5; skip = 1; counters[1]++;
                }
            } else if (count != n) {
                counters[0]++; st = 2;
            } else {
                st = 0;
                if (magic_cksum) skip = 1;
            }
            if (!skip && do_fix) {
                unsigned char newmagic[4];
                const unsigned char *wm = qmagic;
                if (!magic_cksum) { h_cksum(newmagic, eptr, n, C); wm = newmagic; }
                for (int j = 0; j < n; j++) {
                    if (!badmap[j] && magic_cksum) continue;
                    memcpy(b + j * rec, wm, 4);
                    if (eptr[j] != ptr[j]) memcpy(ptr[j], eptr[j], C);
                    if (magic_cksum) rewrite[(size_t)s * n + j] = 1;
                }
            }
        }
        status[s] = st;
        for (int j = 0; j < n; j++) badmap_out[(size_t)s * n + j] = badmap[j];
    }
    free(parity);
}

/* segjerase_read_func's per-stripe verification (segment/jerasure.c:1378-1505) over device
 * images laid out as ref_segment_write makes them (every device readable).  status[s] =
 * 0 ok, 1 recovered, 2 blank, -1 unrecoverable, as lsec_segment_read reports; returns the
 * number of unrecoverable stripes. */
int ref_segment_read(ref_plan_t *p, char **dev, int nstripes, int chunk, int n_shift, long long first_stripe,
                     int paranoid, int magic_cksum, char *data_out, int *status)
{
    int k = p->k, m = p->m, n = k + m, C = chunk, bad = 0, brute_used = 0;
    size_t rec = (size_t)C + 4;
    int badmap[n], badmap_brute[n];
    char *ptr[n], *eptr[n], *pwork[m];
    unsigned char *mag[n], qmagic[4], zero[4] = {0, 0, 0, 0};
    char *work = (char *)malloc((size_t)n * C), *parity = (char *)malloc((size_t)m * C);
    for (int i = 0; i < m; i++) pwork[i] = parity + (size_t)i * C;
    for (int s = 0; s < nstripes; s++) {
        long long ss = first_stripe + s;
        for (int j = 0; j < n; j++) {   /* logical chunk j from device (j - ss*n_shift) mod n (lun.c:1178-1223) */
            int d = (int)(((j - ss * n_shift) % n + n) % n);
            char *r = dev[d] + (size_t)s * rec;
            mag[j] = (unsigned char *)r;
            ptr[j] = work + (size_t)j * C;
            memcpy(ptr[j], r + 4, C);
        }
        int count = h_quorum(n, mag, badmap, qmagic), data_ok = 1, st = 0;
        if (count != n) {
            int nd = 0;
            for (int j = 0; j < n; j++) nd += !badmap[j] && j < k;
            if (nd != k) data_ok = 0;
        } else if (memcmp(zero, qmagic, 4) == 0) {
            int nz = 0;
            for (int j = 0; j < n && !nz; j++) nz = h_nonzero(ptr[j], C);
            data_ok = nz ? 1 : 2;
        }
        int recover = 0;
        if (data_ok == 1) recover = paranoid;
        else if (data_ok == 2) { memset(work, 0, (size_t)k * C); st = 2; }
        else if (count < k) st = -1;
        else recover = 1;
        if (recover) {
            const unsigned char *cm = magic_cksum ? qmagic : NULL;
            if (h_control_check(p, C, n, m, badmap, ptr, eptr, pwork, cm) != 0) {
                if (brute_used) memcpy(badmap, badmap_brute, sizeof(badmap));
                if (h_brute_recovery(p, C, n, m, badmap, ptr, eptr, pwork, cm) == 0) {
                    brute_used = 1;
                    memcpy(badmap_brute, badmap, sizeof(badmap));
                    for (int j = 0; j < k; j++) if (eptr[j] != ptr[j]) memcpy(ptr[j], eptr[j], C);
                    for (int j = 0; j < k; j++) if (badmap[j]) st = 1;   /* user data rebuilt */
                } else {
                    st = -1;
                }
            } else {
                for (int j = 0; j < k; j++) if (badmap[j]) st = 1;
            }
        }
        status[s] = st;
        if (st == -1) bad++;
        else memcpy(data_out + (size_t)s * k * C, work, (size_t)k * C);
    }
    free(work);
    free(parity);
    return bad;
}
