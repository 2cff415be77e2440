"""Segment adapter: the write side of LStore's erasure segment.

The reference image format -- per physical device, per stripe, [4-byte adler32 magic |
chunk] with LUN rotation -- comes from oracle/_ref (real jerasure + zlib, driven by the
restated segjerase_write_func loop); the engine's lsec_segment_write must produce the same
bytes.  The CPU test pins the harness's layout against an independent Python restatement.
"""
import zlib

import numpy as np
import pytest

import lstore_amd as L
import oracle as O
from patterns import stripe
from test_verify import OTHER_CODES, other_plan


def py_segment_images(method, data, m, chunk, n_shift, first, packet=0):
    """segment/jerasure.c:1809-1850 + lun.c:1178-1223, restated in numpy + zlib."""
    n_str, k, _ = data.shape
    n = k + m
    dev = np.zeros((n, n_str * (chunk + 4)), dtype=np.uint8)
    for s in range(n_str):
        full = np.vstack([data[s], O.encode(method, data[s], m, packet)])
        a = 1
        for row in full:
            a = zlib.adler32(row.tobytes(), a)
        magic = np.frombuffer(np.uint32(a).tobytes(), np.uint8)
        for i in range(n):
            j = (i + (first + s) * n_shift) % n
            dev[i, s * (chunk + 4): s * (chunk + 4) + 4] = magic
            dev[i, s * (chunk + 4) + 4: (s + 1) * (chunk + 4)] = full[j]
    return dev


def test_reference_plumbing_layout(built):
    if not O.ref_available():
        pytest.skip("oracle/_ref not built")
    data = np.stack([stripe(6, 4096, s) for s in range(7)])
    rp = O.RefPlan(O.REED_SOL_VAN, 6, 3)
    for n_shift, first in ((1, 0), (1, 5), (2, 3), (0, 0)):
        assert np.array_equal(rp.segment_write(data, 7, 4096, n_shift, first),
                              py_segment_images(O.REED_SOL_VAN, data, 3, 4096, n_shift, first))


@pytest.mark.gpu
@pytest.mark.parametrize("method,k,m,chunk,n_shift,first", [
    (L.REED_SOL_VAN, 6, 3, 65536, 1, 17),     # config c1 geometry
    (L.CAUCHY_GOOD, 6, 3, 16384, 1, 0),       # cjerase_16k.ex3 (sample_exnodes)
    (L.CAUCHY_GOOD, 10, 4, 262144, 3, 2),
    (L.REED_SOL_VAN, 20, 6, 1 << 20, 1, 0),   # column-block staging
    (L.REED_SOL_VAN, 100, 28, 4096, 1, 0),    # k + m = 128: input groups, magic in 80-shard launches
    (L.CAUCHY_GOOD, 70, 2, 8192, 2, 1),
])
def test_segment_write_matches_reference(cuda, method, k, m, chunk, n_shift, first):
    n_str = 12 if chunk <= 262144 else 3
    data = np.stack([stripe(k, chunk, s) for s in range(n_str)])
    with L.Plan.for_chunk(method, k, m, chunk) as p:
        ours = p.segment_write(data, n_shift, first)
        rp = O.RefPlan(method, k, m, 8, p.packet_size)
        ref = rp.segment_write(data, n_str, chunk, n_shift, first)
        assert np.array_equal(ours, ref)


@pytest.mark.gpu
def test_segment_read_quorum_repair_and_brute_force(cuda):
    k, m, C, N, shift = 6, 3, 16384, 16, 1
    data = np.stack([stripe(k, C, s) for s in range(N)])
    lc = C + 4
    with L.Plan.for_chunk(L.CAUCHY_GOOD, k, m, C) as p:
        img = p.segment_write(data, shift, 0)
        out, status, bad = p.segment_read(img, N, C, shift, 0)
        assert bad == 0 and (status == 0).all() and np.array_equal(out, data)

        def phys(s, j):
            return (j - s * shift) % (k + m)

        dmg = img.copy()
        # s0: silent data corruption in data chunk 2 (magic intact) -> only paranoid finds it (brute force)
        dmg[phys(0, 2), 0 * lc + 4 + 100] ^= 0x5A
        # s1: bad magic on data chunk 4 -> quorum marks it, rebuild + verify
        dmg[phys(1, 4), 1 * lc] ^= 1
        # s2: bad magic on a parity chunk -> data quorum intact, returned as is
        dmg[phys(2, k + 1), 2 * lc + 1] ^= 1
        # s3: silent corruption of two chunks -> brute force over pairs
        dmg[phys(3, 0), 3 * lc + 4 + 7] ^= 0xFF
        dmg[phys(3, k), 3 * lc + 4 + 9] ^= 0xFF
        # s4: blank stripe (all magics zero, all data zero)
        dmg[:, 4 * lc: 5 * lc] = 0
        # s5: four bad magics -> unrecoverable (count < k)
        for j in range(4):
            dmg[phys(5, j), 5 * lc + 2] ^= (j + 1)
        out, status, bad = p.segment_read(dmg, N, C, shift, 0, paranoid=True)
        assert status[0] == 1 and status[1] == 1 and status[2] == 0 and status[3] == 1
        assert status[4] == 2 and status[5] == -1 and bad == 1
        keep = [s for s in range(N) if s not in (4, 5)]
        assert np.array_equal(out[keep], data[keep])
        assert not out[4].any()
        # without paranoid mode the silently corrupted stripes pass through unchecked (reference behaviour)
        out, status, bad = p.segment_read(dmg, N, C, shift, 0, paranoid=False)
        assert status[0] == 0 and not np.array_equal(out[0], data[0])
        assert status[1] == 1 and np.array_equal(out[1], data[1])
        # an unreadable device: every stripe rebuilds through decode
        out, status, bad = p.segment_read(img, N, C, shift, 0, missing=(3,))
        assert bad == 0 and np.array_equal(out, data)


@pytest.mark.gpu
@pytest.mark.parametrize("method,k,m,C", [(L.REED_SOL_VAN, 100, 28, 4096), (L.CAUCHY_GOOD, 70, 2, 8192)])
def test_wide_segment_read_repairs(cuda, method, k, m, C):
    """Wide segments (k + m = 128 / 72): a stale magic on up to m devices of a stripe is voted
    out, the stripe rebuilt from the others and checked against its magic."""
    N, shift = 6, 1
    n = k + m
    data = np.stack([stripe(k, C, s + 40) for s in range(N)])
    lc = C + 4
    with L.Plan.for_chunk(method, k, m, C) as p:
        img = p.segment_write(data, shift, 0)
        rng = np.random.default_rng(k)
        for s in range(N):
            for d in rng.permutation(n)[: min(m, 1 + s % 3)]:
                img[d, s * lc] ^= 0x11
        out, status, bad = p.segment_read(img, N, C, shift, 0)
        assert bad == 0 and np.array_equal(out, data)


# ---------------------------------------------------------------- scatter lists (tbuf pieces)
def scatter(data, cuts, error_pieces):
    """Split the flat user bytes at `cuts`; pieces whose index is in `error_pieces` become error
    pages (ints: their length)."""
    flat = data.reshape(-1)
    bounds = [0] + sorted(cuts) + [flat.size]
    pieces = []
    for i in range(len(bounds) - 1):
        pc = flat[bounds[i]:bounds[i + 1]]
        pieces.append(int(pc.size) if i in error_pieces else pc.copy())
    return pieces


def flatten_like_reference(pieces, n_str, k, chunk):
    """What segjerase_write_func encodes for each stripe of a scatter list (segment/jerasure.c:
    1786-1831): the stripe's bytes, except a stripe whose first piece is an error page is all
    zeros; error pages inside a straddling stripe read as zeros."""
    flat = np.concatenate([np.zeros(pc, np.uint8) if isinstance(pc, int) else pc for pc in pieces])
    starts = np.cumsum([0] + [pc if isinstance(pc, int) else pc.size for pc in pieces])
    out = flat[: n_str * k * chunk].reshape(n_str, k, chunk).copy()
    for s in range(n_str):
        p = int(np.searchsorted(starts, s * k * chunk, side="right")) - 1
        if isinstance(pieces[p], int):
            out[s] = 0
    return out


SCATTER_CASES = [
    # (cuts as fractions of a stripe, error pieces)
    ([], set()),                          # one piece: in place
    ([0.5, 1.0, 2.25, 2.75], set()),      # straddles at half / quarter stripes
    ([1.0, 2.0, 3.5], {1}),               # stripe 1 starts in an error page -> zeros
    ([0.3, 0.6, 4.0], {1}),               # error page inside a straddling stripe
    ([2.0, 2.002], {1}),                  # a small error page at a stripe start
]


def _cut_points(k, chunk, fracs):
    dsize = k * chunk
    return [int(round(f * dsize)) // 8 * 8 for f in fracs]


def test_scatter_write_restatement(built):
    """The harness's scatter-list write (ref_segment_write_iov) equals the contiguous reference
    write of the bytes segjerase_write_func encodes (CPU only)."""
    if not O.ref_available():
        pytest.skip("oracle/_ref not built")
    k, m, C, N = 6, 3, 1024, 6
    data = np.stack([stripe(k, C, s + 3) for s in range(N)])
    rp = O.RefPlan(O.REED_SOL_VAN, k, m)
    for fracs, errs in SCATTER_CASES:
        pieces = scatter(data, _cut_points(k, C, fracs), errs)
        got = rp.segment_write_iov(pieces, N, C, 1, 2)
        want = rp.segment_write(flatten_like_reference(pieces, N, k, C), N, C, 1, 2)
        assert np.array_equal(got, want), (fracs, errs)


@pytest.mark.gpu
@pytest.mark.parametrize("method,k,m,chunk", [(L.REED_SOL_VAN, 6, 3, 4096), (L.CAUCHY_GOOD, 6, 3, 16384),
                                              (L.REED_SOL_VAN, 10, 4, 65536)])
def test_segment_write_iov_matches_reference(cuda, method, k, m, chunk):
    """lsec_segment_write_iov vs the restated segjerase_write_func over the real jerasure on
    scatter lists with straddling stripes and error pages: identical device images."""
    N = 6
    data = np.stack([stripe(k, chunk, s + 11) for s in range(N)])
    with L.Plan.for_chunk(method, k, m, chunk) as p:
        rp = O.RefPlan(method, k, m, 8, p.packet_size)
        for fracs, errs in SCATTER_CASES:
            pieces = scatter(data, _cut_points(k, chunk, fracs), errs)
            ours = p.segment_write_iov(pieces, N, chunk, 2, 5)
            ref = rp.segment_write_iov(pieces, N, chunk, 2, 5)
            assert np.array_equal(ours, ref), (fracs, errs)
        with pytest.raises(L.ErasureError, match="bytes in the scatter list"):
            p.segment_write_iov([data.reshape(-1)[:-8]], N, chunk)


def logical_stream_from_images(img, N, chunk, k, m, n_shift, first):
    """Undo the LUN placement: the [magic | chunk] stream in logical order that segjerase_write_func
    hands its LUN child (segment/jerasure.c:1826-1853), from device images (lun.c:1178-1223)."""
    n, lc = k + m, chunk + 4
    out = np.empty((N, n, lc), np.uint8)
    for d in range(n):
        rows = img[d].reshape(N, lc)
        for s in range(N):
            out[s, (d + (first + s) * n_shift) % n] = rows[s]
    return out.reshape(-1)


def gather_iovs(iovs):
    import ctypes as C
    return np.concatenate([np.frombuffer((C.c_uint8 * int(ln)).from_address(int(base)), np.uint8).copy()
                           for base, ln in iovs])


@pytest.mark.gpu
@pytest.mark.parametrize("method,k,m,chunk", [(L.REED_SOL_VAN, 6, 3, 65536), (L.CAUCHY_GOOD, 6, 3, 16384),
                                              (L.CAUCHY_GOOD, 10, 4, 65536)])
def test_segment_encode_iov_is_the_reference_hand_off(cuda, method, k, m, chunk):
    """lsec_segment_encode_iov: the iovec stream [magic | chunk] x (k+m) per stripe, in logical order,
    is byte-identical to what the restated segjerase_write_func over the real jerasure hands its LUN
    child; data iovecs point into the caller's pages (no data copy), parity and magics land in the
    caller's buffers; straddling stripes and error pages as the reference treats them."""
    N = 6
    data = np.stack([stripe(k, chunk, s + 21) for s in range(N)])
    with L.Plan.for_chunk(method, k, m, chunk) as p:
        rp = O.RefPlan(method, k, m, 8, p.packet_size)
        for fracs, errs in SCATTER_CASES:
            pieces = scatter(data, _cut_points(k, chunk, fracs), errs)
            iovs, par, mag, keep = p.segment_encode_iov(pieces, N, chunk)
            assert len(iovs) == 2 * (k + m) * N
            assert all(ln == (4 if i % 2 == 0 else chunk) for i, (_, ln) in enumerate(iovs))
            ref = logical_stream_from_images(rp.segment_write_iov(pieces, N, chunk, 1, 0), N, chunk, k, m, 1, 0)
            assert np.array_equal(gather_iovs(iovs), ref), (fracs, errs)
            # parity chunk r of stripe s is iovec 2((s(k+m) + k + r)) + 1, inside the caller's parity buffer
            assert iovs[2 * k + 1][0] == par.ctypes.data and iovs[0][0] == mag.ctypes.data
        # one piece: every data iovec points into the caller's array, in place
        flat = np.ascontiguousarray(data.reshape(-1))
        iovs, par, mag, keep = p.segment_encode_iov([flat], N, chunk)
        base = flat.ctypes.data
        for s in range(N):
            for j in range(k):
                assert iovs[2 * (s * (k + m) + j) + 1][0] == base + (s * k + j) * chunk
        with pytest.raises(L.ErasureError, match="bytes in the scatter list"):
            p.segment_encode_iov([flat[:-8]], N, chunk)


@pytest.mark.gpu
@pytest.mark.parametrize("method,k,m,C,w,packet", OTHER_CODES)
def test_other_codes_scatter_write_matches_reference(cuda, method, k, m, C, w, packet):
    """The scatter-list write for raid4, r6, Cauchy-orig and the bitmatrix codes: identical images."""
    N = 6
    data = np.stack([stripe(k, C, s + 19) for s in range(N)])
    with other_plan(method, k, m, C, w, packet) as p:
        rp = O.RefPlan(method, k, m, p.w, p.packet_size)
        for fracs, errs in SCATTER_CASES:
            pieces = scatter(data, _cut_points(k, C, fracs), errs)
            assert np.array_equal(p.segment_write_iov(pieces, N, C, 2, 5), rp.segment_write_iov(pieces, N, C, 2, 5)), \
                (fracs, errs)
