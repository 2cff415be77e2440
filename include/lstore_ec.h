/*
 * lstore_ec.h -- C ABI of liblstore_ec.so, the MI355X (gfx950) erasure-coding engine that
 * drops in behind LStore's erasure plan service.
 *
 * Part 1 is the reference interface, declaration for declaration: the plan struct layout,
 * method ids and et_* entry points of src/lio/erasure_tools.h:28-75.  LStore's segment
 * driver dereferences the struct's fields and function pointers directly
 * (src/lio/segment/jerasure.c:1231-1232, :1847, :2242-2243, :245), so the layout below IS
 * the ABI and must not change.  A binary built against the reference header links against
 * this library unchanged (INTEGRATION.md shows the build-line change).
 *
 * Part 2 adds batched and device-resident entry points (prefix lsec_ / et_*_stripes) that
 * the reference does not have; they let a caller hand over many stripes per call, which is
 * what a GPU needs (SURVEY.md §8b "recommended extension").
 *
 * Errors: every call that can fail returns a status (0 = success, negative = failure) and
 * records a message for lsec_last_error().  The two void fn-pointers inherited from the
 * reference (encode_block) cannot return a status; on failure they print the reason to
 * stderr and abort() -- the engine never silently skips or falls back to a CPU path.
 */
#ifndef LSTORE_EC_H
#define LSTORE_EC_H

#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ===================================================================== Part 1: reference ABI */

typedef struct lio_erasure_plan_t lio_erasure_plan_t;   /* src/lio/lio/erasure_tools.h:31 */

/* method ids -- src/lio/erasure_tools.h:37-45 */
#define REED_SOL_VAN    0
#define REED_SOL_R6_OP  1
#define CAUCHY_ORIG     2
#define CAUCHY_GOOD     3
#define BLAUM_ROTH      4
#define LIBERATION      5
#define LIBER8TION      6
#define RAID4           7
#define N_JE_METHODS    8

/* method names -- src/lio/erasure_tools.c:35 */
extern const char *JE_method[N_JE_METHODS];

/* src/lio/erasure_tools.h:50-65 (layout-identical) */
struct lio_erasure_plan_t {
    long long int strip_size;   /* size of each data strip */
    int method;                 /* encoding/decoding method */
    int data_strips;            /* k */
    int parity_strips;          /* m */
    int w;                      /* word size */
    int packet_size;            /* bitmatrix packet size */
    int base_unit;              /* register size in bytes */
    int *encode_matrix;         /* m x k coding matrix (matrix / Cauchy methods) */
    int *encode_bitmatrix;      /* (m*w) x (k*w) 0/1 bitmatrix (bitmatrix methods) */
    int **encode_schedule;      /* smart XOR schedule, -1 terminated (bitmatrix methods) */
    int (*form_encoding_matrix)(lio_erasure_plan_t *plan);
    int (*form_decoding_matrix)(lio_erasure_plan_t *plan);
    void (*encode_block)(lio_erasure_plan_t *plan, char **ptr, int block_size);
    int (*decode_block)(lio_erasure_plan_t *plan, char **ptr, int block_size, int *erasures);
};

/* replaces nearest_prime, erasure_tools.c:50-77 */
int nearest_prime(int w, int which);
/* replaces et_method_type, erasure_tools.c:716-725 (case-insensitive name -> id, -1 if unknown) */
int et_method_type(char *meth);
/* replaces et_new_plan, erasure_tools.c:606-685 */
lio_erasure_plan_t *et_new_plan(int method, long long int strip_size,
                                int data_strips, int parity_strips, int w, int packet_size, int base_unit);
/* replaces et_generate_plan, erasure_tools.c:733-908 (same w / packet-size search) */
lio_erasure_plan_t *et_generate_plan(long long int file_size, int method,
                                     int data_strips, int parity_strips, int w, int packet_low, int packet_high);
/* replaces et_destroy_plan, erasure_tools.c:691-710 */
void et_destroy_plan(lio_erasure_plan_t *plan);
/* replace the file tools et_encode / et_decode, erasure_tools.c:339-436 / :476-600 */
int et_encode(lio_erasure_plan_t *plan, const char *fname, long long int foffset, const char *pname,
              long long int poffset, int buffer_size);
int et_decode(lio_erasure_plan_t *plan, long long int fsize, const char *fname, long long int foffset,
              const char *pname, long long int poffset, int buffer_size, int *erasures);

/*
 * Semantics of the plan's fn-pointers (unchanged from the reference):
 *   encode_block(plan, ptr, C)   ptr[0..k) data chunks, ptr[k..k+m) parity chunks, C bytes each;
 *                                writes only ptr[k..k+m).   (segment/jerasure.c:1847)
 *   decode_block(plan, ptr, C, erasures)  erasures = -1 terminated ids; rebuilds only the
 *                                erased slots; 0 on success, -1 if unrecoverable.  (:245)
 * ptr may hold host pointers (staged over PCIe) or device pointers (used in place).
 * C must be a multiple of 8 (matrix methods) or of w*packet_size (bitmatrix methods).
 */

/* ===================================================================== Part 2: extensions */

#define LSEC_ABI_VERSION 2

/* Stripe-batched host-memory calls.  ptrs holds nstripes*(k+m) pointers laid out exactly
 * like segjerase_write_func's ptr[] array (segment/jerasure.c:1647, :1812-1836): stripe s
 * uses ptrs[s*(k+m) .. s*(k+m)+k+m).  One erasure pattern for all stripes. */
int et_encode_stripes(lio_erasure_plan_t *plan, char **ptrs, int nstripes, int block_size);
int et_decode_stripes(lio_erasure_plan_t *plan, char **ptrs, int nstripes, int block_size, int *erasures);

/* Device-resident calls.  Shard i (0..k+m-1) of stripe s lives at
 *   (char *)shards[i].base + s * shards[i].stride        (device memory)
 * e.g. LStore's layout: data base = page + i*C, stride = k*C; parity base = par + i*C,
 * stride = m*C.  Work is enqueued on `stream` (a hipStream_t; NULL = legacy default stream)
 * and the call returns without synchronising. */
typedef struct {
    void *base;
    long long stride;
} lsec_shard_t;

int lsec_encode_dev(lio_erasure_plan_t *plan, const lsec_shard_t *shards, int nstripes,
                    long long block_size, void *stream);
int lsec_decode_dev(lio_erasure_plan_t *plan, const lsec_shard_t *shards, int nstripes,
                    long long block_size, const int *erasures, void *stream);

/* Per-stripe "magic": the 4-byte little-endian zlib adler32 over the concatenation of a
 * stripe's k+m chunks that LStore's erasure segment stores in front of every chunk
 * (je_cksum_calc, src/lio/segment/jerasure.c:169-182; checked by je_cksum_compare, :188-194).
 * Computed on the GPU.  magic receives 4*nstripes bytes (host memory for et_*, device memory
 * for lsec_*_dev).  The *_encode_* forms encode first and checksum data + fresh parity,
 * which is what segjerase_write_func does per stripe (:1847-1850). */
int et_encode_stripes_magic(lio_erasure_plan_t *plan, char **ptrs, int nstripes, int block_size, char *magic);
int et_stripes_magic(lio_erasure_plan_t *plan, char **ptrs, int nstripes, int block_size, char *magic);
int lsec_encode_magic_dev(lio_erasure_plan_t *plan, const lsec_shard_t *shards, int nstripes,
                          long long block_size, void *magic, void *stream);
int lsec_stripe_magic_dev(lio_erasure_plan_t *plan, const lsec_shard_t *shards, int nstripes,
                          long long block_size, void *magic, void *stream);

/* Batched write side of LStore's erasure segment (segjerase_write_func,
 * src/lio/segment/jerasure.c:1640-1895, for whole-stripe-aligned writes) including the LUN
 * child's placement (lun_row_decompose, src/lio/segment/lun.c:1140-1246).
 * data: nstripes*k*C user bytes (host memory, stripe-major, as the cache page holds them).
 * dev[i] (i = 0..k+m-1, host memory, nstripes*(C+4) bytes each) receives, at offset
 * s*(C+4), the LUN chunk [4-byte stripe magic | chunk j] with
 * j = (i + (first_stripe + s)*n_shift) % (k+m) -- data chunk j for j < k, parity j-k else.
 * Parity and magics are computed on the GPU.  0 / -1. */
int lsec_segment_write(lio_erasure_plan_t *plan, const char *data, int nstripes, int chunk, int n_shift,
                       long long first_stripe, char **dev);
/* The same with the user data as a scatter list (the tbuf's iovecs, segment/jerasure.c:1786-1825):
 * stripe s covers bytes [s*k*C, (s+1)*k*C) of the concatenated pieces.  A stripe inside one
 * piece is read in place; a stripe straddling pieces is gathered into a contiguous copy first
 * (:1795-1811); a stripe whose first piece is an error page (iov_base NULL) is encoded and
 * written as zero data chunks (:1816, :1823-1831).  Error pages inside a straddling stripe read
 * as zeros (the reference would read through the NULL base).  0 / -1 (fewer than nstripes*k*C
 * bytes listed is an error). */
struct iovec;
int lsec_segment_write_iov(lio_erasure_plan_t *plan, const struct iovec *iov, int n_iov, int nstripes, int chunk,
                           int n_shift, long long first_stripe, char **dev);
/* segjerase_write_func's own hand-off, with no data copy (segment/jerasure.c:1780-1858): for
 * nstripes stripes of the scatter list `iov` (as lsec_segment_write_iov reads it), the parity
 * goes to `parity` (caller memory, nstripes*m*C bytes, stripe-major: parity chunk r of stripe s
 * at (s*m + r)*C, the reference's per-op parity buffer) and the stripe magics to `magic`
 * (nstripes*4 bytes), both computed on the GPU; `out` receives 2*(k+m)*nstripes iovecs
 * [4-byte magic | chunk] in logical chunk order (data 0..k-1 then parity 0..m-1 per stripe):
 * the tbuf the reference hands its LUN child (:1852-1853).  Data iovecs point into the caller's
 * pages; a stripe straddling scatter pieces is gathered into `straddle` (k*C bytes per such
 * stripe, lsec_segment_straddle_bytes tells how many bytes); a stripe starting in an error page
 * points at an engine-owned zero chunk.  Returns the number of iovecs, or -1. */
int lsec_segment_encode_iov(lio_erasure_plan_t *plan, const struct iovec *iov, int n_iov, int nstripes, int chunk,
                            char *parity, char *magic, char *straddle, long long straddle_bytes, struct iovec *out,
                            int out_cap);
long long lsec_segment_straddle_bytes(lio_erasure_plan_t *plan, const struct iovec *iov, int n_iov, int nstripes,
                                      int chunk);

/* Flags of the read / inspect entry points */
#define LSEC_READ_PARANOID 1   /* verify every stripe, not only those with bad chunks */
#define LSEC_MAGIC_LEGACY  2   /* segment magic_cksum == 0: magics are not adler32 sums, so
                                  stripes are verified with control chunks (jerasure.c:218-266) */
#define LSEC_INSPECT_FIX   4   /* inspect: repair in place (INSPECT_{QUICK,SCAN,FULL}_REPAIR) */
#define LSEC_MAX_DEVS      256  /* k + m of the segment paths, of w = 8 and of the bitmatrix codes;
                                  the GF(2^16) / GF(2^32) matrix codes (RS, r6, Cauchy) take up
                                  to LSEC_MAX_DEVS_WIDE through the et_* / lsec_*_dev calls */
#define LSEC_MAX_DEVS_WIDE 1024

/* Batched read side for whole stripes (segjerase_read_func, segment/jerasure.c:1255-1631):
 * dev[i] are device images laid out as lsec_segment_write writes them (NULL = device
 * unreadable).  Per stripe: majority vote over the stored magics (:1383-1438); stripes with
 * chunks outside the quorum are rebuilt (decode) and verified (jerase_control_check,
 * :202-269: against the quorum magic, or with control chunks under LSEC_MAGIC_LEGACY),
 * falling back to the brute-force search over erasure combinations (jerase_brute_recovery,
 * :321-339); with LSEC_READ_PARANOID every stripe is verified.  Checks and rebuilds run as
 * GPU batches.  User data (nstripes*k*C) goes to data_out; status[s] (optional) = 0 ok,
 * 1 recovered (a data chunk was rebuilt), 2 blank (zero-filled), -1 unrecoverable.  Returns the number of
 * unrecoverable stripes, or -1 on error. */
int lsec_segment_read(lio_erasure_plan_t *plan, char **dev, int nstripes, int chunk, int n_shift,
                      long long first_stripe, int flags, char *data_out, int *status);

/* Full byte-level inspection and optional repair (segjerase_inspect_full_func,
 * segment/jerasure.c:347-732).  buf holds nstripes stripes as the inspection reads them from
 * the LUN child: stripe-major, k+m records of [4-byte magic | chunk] each
 * (stripe_size_with_magic = (k+m)*(C+4)).  Every stripe is classified as the reference does:
 * stripe_status[s] = LSEC_STRIPE_*; badmap[s*(k+m)+j] = 1 for the devices the reference's
 * badmap holds after the stripe (what [DEVMAP] prints).  With LSEC_INSPECT_FIX the repaired
 * chunks and magics are written into buf and rewrite[s*(k+m)+j] = 1 marks every record the
 * reference writes back (all of them under LSEC_MAGIC_LEGACY, which converts the stripe to
 * adler32 magics).  `state` carries the counters and the brute-force guess between
 * consecutive calls of one inspection (zero it first).  Returns 0, or -1 on error. */
enum {
  LSEC_STRIPE_OK = 0,            /* every magic agrees and the stripe verifies */
  LSEC_STRIPE_EMPTY = 1,         /* never written: zero magics, zero data (skipped) */
  LSEC_STRIPE_BAD_MAGIC = 2,     /* some magics disagree; the rebuild of those devices verifies */
  LSEC_STRIPE_REPAIRED = 3,      /* silent corruption found by the brute-force search ("r-mismatch") */
  LSEC_STRIPE_LOST_MAGIC = 4,    /* too few matching magics to rebuild ("magic") */
  LSEC_STRIPE_LOST_MISMATCH = 5  /* data and parity disagree beyond repair ("u-mismatch") */
};
typedef struct {
  long long bad_stripes;      /* sf->bad_stripes (bad_count) */
  long long unrecoverable;    /* unrecoverable_count */
  long long silent_errors;    /* erasure_errors: stripes whose check failed */
  long long empty_stripes;    /* n_empty */
  int brute_used;             /* bm_brute_used */
  unsigned char brute_badmap[LSEC_MAX_DEVS];  /* badmap_brute */
} lsec_inspect_state_t;
int lsec_segment_inspect(lio_erasure_plan_t *plan, char *buf, int nstripes, int chunk, int flags,
                         int *stripe_status, unsigned char *badmap, unsigned char *rewrite,
                         lsec_inspect_state_t *state);

/* Pre-build (and cache on the current device) the decode matrix for one erasure pattern,
 * so the first lsec_decode_dev of that pattern does no host work.  0 / -1. */
int lsec_prepare_decode(lio_erasure_plan_t *plan, const int *erasures);
/* The same for the encode image.  For wide matrix codes (R*K >= 96 at w = 8) both also wait
 * for the plan's run-time compiled XOR network (ec_jit.cpp); until it is ready the table
 * kernel serves.  0 / -1. */
int lsec_prepare_encode(lio_erasure_plan_t *plan);
/* 1 when the encode (erasures == NULL) or the decode of that erasure pattern runs on a
 * compiled network on the current device (wide GF(2^8) RS codes; RS / r6 at w = 16 / 32; the
 * packet networks of the liberation family and of Cauchy at w = 16 / 32, and at w = 8 with more
 * than four outputs -- at the plan's strip_size), 0 otherwise. */
int lsec_plan_jit(lio_erasure_plan_t *plan, const int *erasures);

/* Devices that serve host-memory calls (et_*_stripes, et_*_magic, the plan's fn-pointers,
 * lsec_segment_write).  n = 0 (the default): the calling thread's current HIP device.  With a
 * set, a batch larger than the coalescing limit is split into contiguous stripe ranges, one
 * per listed device, each staged and computed on its own device and PCIe link in parallel;
 * smaller calls go to the listed devices in turn.  A device may be listed more than once.
 * 0 / -1 (unknown device). */
int lsec_set_host_devices(const int *devices, int n);
/* Host NUMA placement of device `dev`: its node (-1 if unknown) in *node and up
 * to max_cpus of that node's CPUs this process may use in cpus[].  The engine pins a device's
 * dispatcher thread, the threads running its share of a split host batch and the copy pool that
 * packs its page-locked staging to these CPUs (LSEC_NUMA=0: no pinning).  A caller that owns a
 * device (one process per GPU) can pin itself there before it allocates its host buffers.
 * Returns the number of CPUs (0: no placement known), or -1 (no such device). */
int lsec_device_numa(int dev, int *node, int *cpus, int max_cpus);

/* Engine information / control */
int lsec_abi_version(void);
int lsec_device_count(void);                 /* visible HIP devices, 0 if none */
const char *lsec_last_error(void);           /* thread-local message of the last failure */
/* kernel that applies the plan: 1 = bytewise GF(2^8) (RS, r6, raid4), 2 = bit-sliced GF(2^8)
 * (Cauchy w = 8), 3 = GF(2) bitmatrix (liberation family), 4 = wordwise GF(2^16) / GF(2^32)
 * (RS, r6 at w = 16/32), 5 = bit-sliced GF(2^16) / GF(2^32) (Cauchy at w = 16/32),
 * 0 = no GPU kernel (calls fail with -1) */
int lsec_plan_kernel(lio_erasure_plan_t *plan);
void lsec_set_kernel_variant(int bytewise_variant, int bitsliced_variant);  /* tuning experiments */
/* How the streaming kernels deal their tiles to the 8 XCDs (LSEC_TILES=static|shared|tail picks
 * the start value; default tail): 0 = each XCD its static eighth; 1 = persistent grid, each XCD
 * takes tiles from its own eighth through an atomic counter and then helps the others; 2 = the
 * first 7/8 of each eighth static, the rest shared.  For A/B runs; results are identical in every
 * mode. */
void lsec_set_tile_sharing(int mode);
int lsec_tile_sharing(void);
/* Pageable host chunks a call pins in place (hipHostRegister) are unregistered before the call
 * returns.  Opt-in (LSEC_DEFER_UNPIN_MB > 0, for a process where this library is the only HIP
 * user): while other calls hold registrations of their own, a background thread does it instead,
 * shortly after the call returns (hipHostUnregister waits until the whole device is idle).  With
 * that on, a caller that registers host memory with HIP itself, or hands memory it may have freed
 * and reallocated to another HIP user, calls this first: it returns when nothing is pending.  0. */
int lsec_host_unpin_drain(void);
/* Measurement probe, not part of the coding path: enqueue a streaming device copy dst <- src
 * (bytes a multiple of 16, 16-byte aligned device pointers) on `stream` with the coding kernels'
 * memory shape; bench.py times it as the box's practical HBM ceiling.  0 / -1. */
int lsec_hbm_copy_dev(void *dst, const void *src, unsigned long long bytes, void *stream);
/* Measurement probe: for every stripe, shards[k+r] <- XOR of shards[0..k) (r < m <= 16), with
 * the RS encode kernel's tiles: the encode's k-read : m-write HBM traffic without its GF
 * arithmetic, which bench.py times beside the encode.  0 / -1. */
int lsec_hbm_mix_dev(const lsec_shard_t *shards, int k, int m, int nstripes, long long block_size, void *stream);

/* Measurement probe: for every stripe, shards[k] <- XOR of shards[0..k), in a kernel that shares
 * no code with the coding kernels: the single-erasure decode's k-read : 1-write HBM traffic with
 * the plainest streaming code.  variant = IT | G << 4 | REMAP << 8: IT (1, 2, 4) 16-byte steps
 * per lane, G (1, 2, 4) tiles of 4096 * IT bytes per workgroup, REMAP 1 = XCD-contiguous grabs;
 * block_size a multiple of 4096 * IT.  bench.py times every variant beside the decode.  0 / -1. */
int lsec_hbm_decode_shape_dev(const lsec_shard_t *shards, int k, int nstripes, long long block_size, int variant,
                              void *stream);
#ifdef __cplusplus
}
#endif

#endif /* LSTORE_EC_H */
