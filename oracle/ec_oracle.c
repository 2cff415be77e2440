/*
 * oracle/ec_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Independent CPU restatement of LStore's erasure plan service
 * (src/lio/erasure_tools.c) over Jerasure 1.2A (vendor/jerasure/src), used
 * solely as the checker by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg.  It is never linked into, loaded by, or called from the
 * engine (lstore_amd/liblstore_ec.so).
 *
 * Pinning: this restatement is checked against fixtures produced by the real
 * reference (oracle/_ref/libjerasure_ref.so built from the unmodified
 * /root/reference sources by oracle/Makefile; fixtures in tests/golden/,
 * generator tests/golden/make_golden.py) and against the known-answer anchors
 * recorded in SURVEY.md §8c.
 *
 * Scope: w = 8, 16 and 32 (what erasure_tools.c:806-811 accepts) for all
 * matrix methods (reed_sol_van, reed_sol_r6_op, cauchy_orig, cauchy_good,
 * raid4), and generic bitmatrix encode/decode (any w) for the bitmatrix
 * methods.  Clarity over speed: plain element loops.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "ec_oracle.h"

/* ---------------- GF(2^8) over x^8+x^4+x^3+x^2+1 (galois.c:75, prim_poly[8] = 0435) */
static uint8_t g_exp[512];
static int g_log[256];
static int g_ready;

void eco_init(void)
{
    if (g_ready) return;
    int b = 1;
    /* log/antilog construction: galois.c:169-213 */
    for (int j = 0; j < 255; j++) {
        g_log[b] = j;
        g_exp[j] = (uint8_t)b;
        g_exp[j + 255] = (uint8_t)b;
        b <<= 1;
        if (b & 0x100) b ^= 0x11D;
    }
    g_log[0] = -1;
    g_ready = 1;
}

int eco_mul(int a, int b)
{
    if (a == 0 || b == 0) return 0;
    return g_exp[g_log[a] + g_log[b]];
}

int eco_div(int a, int b)
{
    if (b == 0) return -1;
    if (a == 0) return 0;
    return g_exp[g_log[a] + 255 - g_log[b]];
}

/* GF(2^w) for w = 16 and 32: shift-and-add multiply modulo Jerasure's primitive
 * polynomials (galois.c:65-98: prim_poly[16] = 0210013, prim_poly[32] = 020000007
 * with the x^32 term implied), as galois_shift_multiply (galois.c:343-371) does.
 * Multiplication in a field is unique, so this equals the log tables (w = 16,
 * galois.c:169-213) and the split-w8 tables (w = 32, galois.c:817-880). */
static uint32_t poly_w(int w) { return w == 16 ? 0x1100Bu : w == 32 ? 0x00400007u : 0x11Du; }

uint32_t eco_mulw(uint32_t a, uint32_t b, int w)
{
    if (w == 8) return (uint32_t)eco_mul((int)a, (int)b);
    uint32_t prod = 0, top = 1u << (w - 1), mask = w == 32 ? 0xFFFFFFFFu : (1u << w) - 1;
    for (int i = 0; i < w; i++) {
        if (a & (1u << i)) prod ^= b;
        b = (b & top) ? ((b << 1) ^ poly_w(w)) & mask : (b << 1) & mask;
    }
    return prod;
}

/* a^(2^w - 2) = a^-1 (any correct inverse equals galois_shift_inverse / the log tables) */
uint32_t eco_invw(uint32_t a, int w)
{
    if (w == 8) return (uint32_t)eco_div(1, (int)a);
    uint32_t r = 1, base = a;
    for (int i = 1; i < w; i++) {      /* exponent bits 1..w-1 are set, bit 0 is clear */
        base = eco_mulw(base, base, w);
        r = eco_mulw(r, base, w);
    }
    return r;
}


/* ---------------- coding matrices ---------------------------------------- */
/* Matrices are int arrays as in Jerasure; for w = 32 an element is the int's bit pattern. */
#define U(x) ((uint32_t)(x))

/* reed_sol_vandermonde_coding_matrix (reed_sol.c:79-99) via the systematic
 * distribution matrix (reed_sol.c:242-367): column-reduce an extended
 * Vandermonde matrix to [I;C], normalise row k to ones, then every later row's
 * first column to one. */
static int rs_vandermonde(int k, int m, int w, int *out)
{
    int rows = k + m, cols = k;
    if ((w < 30 && (1 << w) < rows) || cols >= rows) return -1;   /* reed_sol.c:247-248 */
    uint32_t *d = (uint32_t *)calloc((size_t)rows * cols, sizeof(uint32_t));
    d[0] = 1;                                  /* row 0 = e_0          */
    d[(rows - 1) * cols + cols - 1] = 1;       /* last row = e_{k-1}   */
    for (int i = 1; i < rows - 1; i++) {       /* row i = (1, i, i^2, ...) */
        uint32_t v = 1;
        for (int j = 0; j < cols; j++) { d[i * cols + j] = v; v = eco_mulw(v, U(i), w); }
    }
    for (int i = 1; i < cols; i++) {
        int r = i;
        while (r < rows && d[r * cols + i] == 0) r++;
        if (r >= rows) { free(d); return -1; }
        if (r != i)
            for (int c = 0; c < cols; c++) {
                uint32_t t = d[r * cols + c]; d[r * cols + c] = d[i * cols + c]; d[i * cols + c] = t;
            }
        if (d[i * cols + i] != 1) {
            uint32_t inv = eco_invw(d[i * cols + i], w);
            for (int rr = 0; rr < rows; rr++) d[rr * cols + i] = eco_mulw(inv, d[rr * cols + i], w);
        }
        for (int j = 0; j < cols; j++) {
            uint32_t e = d[i * cols + j];
            if (j == i || e == 0) continue;
            for (int rr = 0; rr < rows; rr++) d[rr * cols + j] ^= eco_mulw(e, d[rr * cols + i], w);
        }
    }
    for (int j = 0; j < cols; j++) {           /* row k -> all ones */
        uint32_t e = d[cols * cols + j];
        if (e == 1) continue;
        uint32_t inv = eco_invw(e, w);
        for (int rr = cols; rr < rows; rr++) d[rr * cols + j] = eco_mulw(inv, d[rr * cols + j], w);
    }
    for (int rr = cols + 1; rr < rows; rr++) { /* column 0 -> all ones */
        uint32_t e = d[rr * cols];
        if (e == 1) continue;
        uint32_t inv = eco_invw(e, w);
        for (int j = 0; j < cols; j++) d[rr * cols + j] = eco_mulw(d[rr * cols + j], inv, w);
    }
    for (int i = 0; i < m * k; i++) out[i] = (int)d[cols * cols + i];
    free(d);
    return 0;
}

/* number of ones in the w x w bit-block of n (what cauchy_n_ones, cauchy.c:92-132, counts) */
static int n_ones(uint32_t n, int w)
{
    int total = 0;
    for (int x = 0; x < w; x++) {
        total += __builtin_popcount(n);
        n = eco_mulw(n, 2, w);
    }
    return total;
}

/* cauchy_original_coding_matrix (cauchy.c:134-150): M[i][j] = 1/(i xor (m+j)) */
static int cauchy_orig(int k, int m, int w, int *out)
{
    if (w < 31 && k + m > (1 << w)) return -1;
    for (int i = 0; i < m; i++)
        for (int j = 0; j < k; j++) out[i * k + j] = (int)eco_invw(U(i ^ (m + j)), w);
    return 0;
}

/* cauchy_improve_coding_matrix (cauchy.c:169-210) */
static void cauchy_improve(int k, int m, int w, int *M)
{
    for (int j = 0; j < k; j++) {
        if (M[j] == 1) continue;
        uint32_t inv = eco_invw(U(M[j]), w);
        for (int i = 0; i < m; i++) M[i * k + j] = (int)eco_mulw(U(M[i * k + j]), inv, w);
    }
    for (int i = 1; i < m; i++) {
        int *row = M + i * k;
        int best = 0, best_j = -1;
        for (int j = 0; j < k; j++) best += n_ones(U(row[j]), w);
        for (int j = 0; j < k; j++) {
            if (row[j] == 1) continue;
            uint32_t inv = eco_invw(U(row[j]), w);
            int tot = 0;
            for (int x = 0; x < k; x++) tot += n_ones(eco_mulw(U(row[x]), inv, w), w);
            if (tot < best) { best = tot; best_j = j; }
        }
        if (best_j >= 0) {
            uint32_t inv = eco_invw(U(row[best_j]), w);
            for (int j = 0; j < k; j++) row[j] = (int)eco_mulw(U(row[j]), inv, w);
        }
    }
}

/* Second row of the best m=2 Cauchy matrices for w=8 (cauchy.c:262-274, data). */
static const uint8_t CBEST8[255] = {
    1, 2, 142, 4, 71, 8, 70, 173, 3, 35, 143, 16, 17, 67, 134, 140, 172, 6, 34, 69, 201, 216, 5, 33,
    86, 12, 65, 138, 158, 159, 175, 10, 32, 43, 66, 108, 130, 193, 234, 9, 24, 25, 50, 68, 79, 100,
    132, 174, 200, 217, 20, 21, 42, 48, 87, 169, 41, 54, 64, 84, 96, 117, 154, 155, 165, 226, 77, 82,
    135, 136, 141, 168, 192, 218, 238, 7, 18, 19, 39, 40, 78, 113, 116, 128, 164, 180, 195, 205, 220,
    232, 14, 26, 27, 58, 109, 156, 157, 203, 235, 13, 28, 29, 38, 51, 56, 75, 85, 90, 101, 110, 112,
    139, 171, 11, 37, 49, 52, 76, 83, 102, 119, 131, 150, 151, 167, 182, 184, 188, 197, 219, 224, 45,
    55, 80, 94, 97, 133, 170, 194, 204, 221, 227, 236, 36, 47, 73, 92, 98, 104, 118, 152, 153, 166,
    202, 207, 239, 251, 22, 23, 44, 74, 91, 148, 149, 161, 181, 190, 233, 46, 59, 88, 137, 146, 147,
    163, 196, 208, 212, 222, 250, 57, 81, 95, 106, 111, 129, 160, 176, 199, 243, 249, 15, 53, 72, 93,
    103, 115, 125, 162, 183, 185, 189, 206, 225, 255, 186, 210, 230, 237, 242, 248, 30, 31, 62, 89,
    99, 105, 114, 121, 124, 178, 209, 213, 223, 228, 241, 254, 60, 191, 198, 247, 120, 240, 107, 127,
    144, 145, 177, 211, 214, 246, 245, 123, 126, 187, 231, 253, 63, 179, 229, 244, 61, 122, 215, 252};

/* cauchy_good_general_coding_matrix (cauchy.c:212-241); cbest tables exist for
 * w <= 11 only (cbest_max_k, cauchy.c:81-83), so w = 16/32 always improves. */
static int cauchy_good(int k, int m, int w, int *out)
{
    if (w == 8 && m == 2 && k <= 255) {
        for (int j = 0; j < k; j++) { out[j] = 1; out[k + j] = CBEST8[j]; }
        return 0;
    }
    if (cauchy_orig(k, m, w, out)) return -1;
    cauchy_improve(k, m, w, out);
    return 0;
}

int eco_coding_matrix(int method, int k, int m, int w, int *out)
{
    eco_init();
    if (w != 8 && w != 16 && w != 32) return -1;
    switch (method) {
    case ECO_REED_SOL_VAN: return rs_vandermonde(k, m, w, out);
    case ECO_REED_SOL_R6_OP: {             /* reed_sol_r6_coding_matrix, reed_sol.c:59-77 */
        if (m != 2) return -1;
        uint32_t v = 1;
        for (int j = 0; j < k; j++) { out[j] = 1; out[k + j] = (int)v; v = eco_mulw(v, 2, w); }
        return 0;
    }
    case ECO_CAUCHY_ORIG: return cauchy_orig(k, m, w, out);
    case ECO_CAUCHY_GOOD: return cauchy_good(k, m, w, out);
    case ECO_RAID4:
        if (m != 1) return -1;
        for (int j = 0; j < k; j++) out[j] = 1;
        return 0;
    default: return -1;
    }
}

/* jerasure_matrix_to_bitmatrix (jerasure.c:273-299):
 * bit[(i*w+l)][(j*w+x)] = bit l of (M[i][j] * 2^x) */
int eco_matrix_to_bitmatrix(int k, int m, int w, const int *M, int *out)
{
    eco_init();
    if (w != 8 && w != 16 && w != 32) return -1;
    int cols = k * w;
    for (int i = 0; i < m; i++)
        for (int j = 0; j < k; j++) {
            uint32_t e = U(M[i * k + j]);
            for (int x = 0; x < w; x++) {
                for (int l = 0; l < w; l++) out[(i * w + l) * cols + j * w + x] = (e >> l) & 1;
                e = eco_mulw(e, 2, w);
            }
        }
    return 0;
}

/* ---------------- plan geometry: et_generate_plan (erasure_tools.c:733-908) */
static int nearest_prime_up(int n)
{
    for (int p = n > 2 ? n : 2;; p++) {
        int ok = 1;
        for (int d = 2; d * d <= p; d++) if (p % d == 0) { ok = 0; break; }
        if (ok) return p;
    }
}

int eco_generate_plan(long long file_size, int method, int k, int m, int w, int plow, int phigh,
                      int *w_out, int *packet_out, long long *strip_out, int *base_out)
{
    int base = 8;
    if (w == -1) {
        switch (method) {
        case ECO_REED_SOL_VAN: case ECO_REED_SOL_R6_OP:
        case ECO_CAUCHY_ORIG: case ECO_CAUCHY_GOOD: case ECO_LIBER8TION:
            w = 8; break;
        case ECO_BLAUM_ROTH: w = nearest_prime_up(k + 1) - 1; break;
        case ECO_LIBERATION: w = nearest_prime_up(k); break;
        case ECO_RAID4: w = 8; base = 1; break;
        default: return -1;
        }
    }
    long long approx = file_size / ((long long)w * base * k);
    int lo = approx < 4096 ? (int)(approx / 4) : 512;
    int hi = approx < 4096 ? (int)approx : 4096;
    if (plow < 0) plow = lo;
    if (phigh < 0) phigh = hi;
    if (plow > phigh) return -1;
    plow = (plow / base) * base;
    phigh = (phigh / base) * base;
    switch (method) {
    case ECO_REED_SOL_R6_OP: if (m != 2) return -1; /* fallthrough */
    case ECO_REED_SOL_VAN: case ECO_CAUCHY_ORIG: case ECO_CAUCHY_GOOD:
        if (w != 8 && w != 16 && w != 32) return -1;
        break;
    case ECO_RAID4:
        if (m != 1) return -1;
        base = 1; plow = 0; phigh = 1;
        break;
    default:
        break;   /* bitmatrix-family validation is not on the configs */
    }
    /* search downward from phigh for the packet with the least padding;
     * ties go to the smaller packet; stop once padding < 1% */
    long long best_excess = 10 * file_size, best_size = 0;
    int best_p = -1;
    for (int p = phigh; p > plow; p -= base) {
        long long unit = (long long)k * w * p * base;
        long long sz = file_size, rem = sz % unit;
        if (rem > 0) sz += unit - rem;
        int excess = (int)(sz - file_size);          /* int as in the reference */
        if (excess <= best_excess) {
            best_excess = excess; best_p = p; best_size = sz;
            float pct = (float)((1.0 * excess) / file_size * 100);  /* double, stored to float (:893-894) */
            if (pct < 1) break;
        }
    }
    *w_out = w;
    *packet_out = best_p;
    *strip_out = best_size / k;
    *base_out = base;
    return 0;
}

/* ---------------- encode ------------------------------------------------- */

/* jerasure_matrix_encode semantics (jerasure.c:301-315, :579-639):
 * coding[i][t] = XOR_j M[i][j] * data[j][t] over elements t of w bits, stored as
 * native little-endian bytes / uint16 / uint32 (galois_w{08,16,32}_region_multiply,
 * galois.c:471-525, :527-604, :730-810).  size is in bytes. */
void eco_matrix_encode(int k, int m, int w, const int *M, char **data, char **coding, int size)
{
    eco_init();
    int n = size / (w / 8);
    for (int i = 0; i < m; i++) {
        memset(coding[i], 0, size);
        for (int j = 0; j < k; j++) {
            uint32_t c = U(M[i * k + j]);
            if (c == 0) continue;
            if (w == 8) {
                uint8_t *o = (uint8_t *)coding[i], tab[256];
                const uint8_t *src = (const uint8_t *)data[j];
                for (int v = 0; v < 256; v++) tab[v] = (uint8_t)eco_mul((int)c, v);
                for (int t = 0; t < n; t++) o[t] ^= tab[src[t]];
            } else if (w == 16) {
                uint16_t *o = (uint16_t *)coding[i];
                const uint16_t *src = (const uint16_t *)data[j];
                for (int t = 0; t < n; t++) o[t] ^= (uint16_t)eco_mulw(c, src[t], 16);
            } else {
                uint32_t *o = (uint32_t *)coding[i];
                const uint32_t *src = (const uint32_t *)data[j];
                for (int t = 0; t < n; t++) o[t] ^= eco_mulw(c, src[t], 32);
            }
        }
    }
}

/* jerasure_bitmatrix_encode semantics (jerasure.c:1362-1382, :317-362): per
 * super-packet of w*P bytes, coding[i] packet l = XOR of data[j] packets x
 * with bit[(i*w+l)][(j*w+x)] == 1.  Requires size % (w*P) == 0. */
int eco_bitmatrix_encode(int k, int m, int w, const int *B, char **data, char **coding, int size,
                         int packet)
{
    if (packet <= 0 || size % (w * packet) != 0) return -1;
    int cols = k * w;
    for (int s = 0; s < size; s += w * packet)
        for (int r = 0; r < m * w; r++) {
            uint8_t *o = (uint8_t *)coding[r / w] + s + (r % w) * packet;
            memset(o, 0, packet);
            for (int c = 0; c < cols; c++) {
                if (!B[r * cols + c]) continue;
                const uint8_t *src = (const uint8_t *)data[c / w] + s + (c % w) * packet;
                for (int b = 0; b < packet; b++) o[b] ^= src[b];
            }
        }
    return 0;
}

/* ---------------- decode ------------------------------------------------- */

/* erasures: -1 terminated ids (0..k-1 data, k..k+m-1 coding); fills erased[k+m];
 * returns -1 when fewer than k devices survive (jerasure_erasures_to_erased, jerasure.c:524-549) */
static int to_erased(int k, int m, const int *erasures, int *erased)
{
    int alive = k + m;
    memset(erased, 0, sizeof(int) * (k + m));
    for (int i = 0; erasures[i] != -1; i++) {
        int e = erasures[i];
        if (e < 0 || e >= k + m) return -1;
        if (!erased[e]) { erased[e] = 1; if (--alive < k) return -1; }
    }
    return 0;
}

/* Gauss-Jordan inverse over GF(2^w); returns -1 if singular */
static int gf_invert(int n, int w, uint32_t *a, uint32_t *inv)
{
    for (int i = 0; i < n * n; i++) inv[i] = 0;
    for (int i = 0; i < n; i++) inv[i * n + i] = 1;
    for (int c = 0; c < n; c++) {
        int p = c;
        while (p < n && a[p * n + c] == 0) p++;
        if (p == n) return -1;
        if (p != c)
            for (int x = 0; x < n; x++) {
                uint32_t t = a[p * n + x]; a[p * n + x] = a[c * n + x]; a[c * n + x] = t;
                t = inv[p * n + x]; inv[p * n + x] = inv[c * n + x]; inv[c * n + x] = t;
            }
        uint32_t s = eco_invw(a[c * n + c], w);
        for (int x = 0; x < n; x++) { a[c * n + x] = eco_mulw(a[c * n + x], s, w); inv[c * n + x] = eco_mulw(inv[c * n + x], s, w); }
        for (int r = 0; r < n; r++) {
            uint32_t f = a[r * n + c];
            if (r == c || f == 0) continue;
            for (int x = 0; x < n; x++) { a[r * n + x] ^= eco_mulw(f, a[c * n + x], w); inv[r * n + x] ^= eco_mulw(f, inv[c * n + x], w); }
        }
    }
    return 0;
}

/* Recover erased devices from the first k survivors (the choice made by
 * jerasure_make_decoding_matrix, jerasure.c:100-128).  Because the code is MDS
 * the recovered bytes are unique, so any correct decode equals jerasure's. */
int eco_matrix_decode(int k, int m, int w, const int *M, const int *erasures, char **ptrs, int size)
{
    eco_init();
    int erased[2048], ids[2048];
    if (k + m > 2048 || to_erased(k, m, erasures, erased)) return -1;
    int n = 0;
    for (int i = 0; n < k; i++) if (!erased[i]) ids[n++] = i;
    uint32_t *a = (uint32_t *)malloc(sizeof(uint32_t) * k * k), *inv = (uint32_t *)malloc(sizeof(uint32_t) * k * k);
    int *row = (int *)malloc(sizeof(int) * k);
    for (int r = 0; r < k; r++)
        for (int c = 0; c < k; c++)
            a[r * k + c] = ids[r] < k ? (uint32_t)(ids[r] == c) : U(M[(ids[r] - k) * k + c]);
    if (gf_invert(k, w, a, inv)) { free(a); free(inv); free(row); return -1; }
    char **surv = (char **)malloc(sizeof(char *) * k);
    for (int j = 0; j < k; j++) surv[j] = ptrs[ids[j]];
    for (int i = 0; i < k; i++) {
        if (!erased[i]) continue;
        char *out = ptrs[i];
        for (int j = 0; j < k; j++) row[j] = (int)inv[i * k + j];
        eco_matrix_encode(k, 1, w, row, surv, &out, size);
    }
    for (int i = 0; i < m; i++)
        if (erased[k + i]) eco_matrix_encode(k, 1, w, M + i * k, ptrs, &ptrs[k + i], size);
    free(surv); free(a); free(inv); free(row);
    return 0;
}

/* GF(2) inverse of an n x n 0/1 matrix */
static int gf2_invert(int n, int *a, int *inv)
{
    for (int i = 0; i < n * n; i++) inv[i] = 0;
    for (int i = 0; i < n; i++) inv[i * n + i] = 1;
    for (int c = 0; c < n; c++) {
        int p = c;
        while (p < n && a[p * n + c] == 0) p++;
        if (p == n) return -1;
        if (p != c)
            for (int x = 0; x < n; x++) {
                int t = a[p * n + x]; a[p * n + x] = a[c * n + x]; a[c * n + x] = t;
                t = inv[p * n + x]; inv[p * n + x] = inv[c * n + x]; inv[c * n + x] = t;
            }
        for (int r = 0; r < n; r++) {
            if (r == c || !a[r * n + c]) continue;
            for (int x = 0; x < n; x++) { a[r * n + x] ^= a[c * n + x]; inv[r * n + x] ^= inv[c * n + x]; }
        }
    }
    return 0;
}

/* Bitmatrix decode (the job of jerasure_schedule_decode_lazy, jerasure.c:953-979):
 * invert the (k*w)^2 survivor bitmatrix over GF(2), rebuild erased data,
 * then re-encode erased coding devices. */
int eco_bitmatrix_decode(int k, int m, int w, const int *B, const int *erasures, char **ptrs,
                         int size, int packet)
{
    int erased[2048], ids[2048];
    if (k + m > 2048 || to_erased(k, m, erasures, erased)) return -1;
    if (packet <= 0 || size % (w * packet) != 0) return -1;
    int n = 0;
    for (int i = 0; n < k; i++) if (!erased[i]) ids[n++] = i;
    int kw = k * w;
    int *a = (int *)calloc((size_t)kw * kw, sizeof(int)), *inv = (int *)malloc(sizeof(int) * kw * kw);
    for (int r = 0; r < k; r++)
        for (int l = 0; l < w; l++) {
            int *row = a + (r * w + l) * kw;
            if (ids[r] < k) row[ids[r] * w + l] = 1;
            else memcpy(row, B + ((ids[r] - k) * w + l) * kw, sizeof(int) * kw);
        }
    if (gf2_invert(kw, a, inv)) { free(a); free(inv); return -1; }
    char **surv = (char **)malloc(sizeof(char *) * k);
    for (int j = 0; j < k; j++) surv[j] = ptrs[ids[j]];
    for (int i = 0; i < k; i++) {
        if (!erased[i]) continue;
        char *out = ptrs[i];
        eco_bitmatrix_encode(k, 1, w, inv + i * w * kw, surv, &out, size, packet);
    }
    for (int i = 0; i < m; i++)
        if (erased[k + i]) eco_bitmatrix_encode(k, 1, w, B + i * w * kw, ptrs, &ptrs[k + i], size, packet);
    free(surv); free(a); free(inv);
    return 0;
}

/* ---------------- adler32 (RFC 1950), as zlib computes it for je_cksum_calc
 * (segment/jerasure.c:169-182).  zlib is a system dependency, not vendored:
 * parity unpinned by the reference; pinned against the container's zlib. */
unsigned int eco_adler32(unsigned int adler, const unsigned char *buf, long long len)
{
    unsigned long a = adler & 0xffff, b = (adler >> 16) & 0xffff;
    for (long long i = 0; i < len; i++) {
        a += buf[i];
        if (a >= 65521) a -= 65521;
        b += a;
        if (b >= 65521) b -= 65521;
    }
    return (unsigned int)((b << 16) | a);
}
