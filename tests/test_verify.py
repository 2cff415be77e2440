"""Verification / repair: segment read and full inspection.

The checker is the reference's own procedure -- jerase_control_check, jerase_brute_recovery,
and the per-stripe loops of segjerase_read_func / segjerase_inspect_full_func -- restated in
oracle/ref_harness.c over the real jerasure decode and zlib (segment/jerasure.c itself needs
APR and cannot be built here).  The GPU path must agree on every stripe status, every
reported bad-device map, every record the inspection writes back, and every byte of user
data, for cksum (adler32) and legacy magics, with and without repair.
"""
import numpy as np
import pytest

import lstore_amd as L
from lstore_amd import erasure as E
import oracle as O
from patterns import stripe

needs_ref = pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built")


def logical_records(img, nstr, chunk, n, n_shift=1, first=0):
    """device images [n, N*(C+4)] -> stripe-major logical records [N, n, C+4] (the LUN view)."""
    lc = chunk + 4
    buf = np.zeros((nstr, n, lc), np.uint8)
    for s in range(nstr):
        for j in range(n):
            d = (j - (first + s) * n_shift) % n
            buf[s, j] = img[d, s * lc:(s + 1) * lc]
    return buf


def damage(buf, k, m, rng, legacy=False):
    """Per stripe, one of the failure shapes the segment meets (seeded)."""
    nstr, n, lc = buf.shape
    kinds = []
    for s in range(nstr):
        kind = int(rng.integers(0, 12))
        kinds.append(kind)
        devs = rng.permutation(n)
        if legacy:  # old-school magics: one arbitrary value per stripe, not a checksum
            buf[s, :, :4] = rng.integers(1, 255, 4, dtype=np.uint8)
        if kind == 1:      # stale magic on one device
            buf[s, devs[0], 0] ^= 0x11
        elif kind == 2:    # stale magic on m devices
            for d in devs[:m]:
                buf[s, d, 1] ^= 0x22
        elif kind == 3:    # too few matching magics
            for i, d in enumerate(devs[:m + 1]):
                buf[s, d, 2] ^= i + 1
        elif kind == 4:    # silent corruption of one chunk
            buf[s, devs[0], 4 + int(rng.integers(0, lc - 4))] ^= 0x5A
        elif kind == 5:    # silent corruption of two chunks
            for d in devs[:2]:
                buf[s, d, 4 + int(rng.integers(0, lc - 4))] ^= 0xA5
        elif kind == 6:    # stale magic on one device, silent corruption on another
            buf[s, devs[0], 3] ^= 0x01
            buf[s, devs[1], 4 + 17] ^= 0xFF
        elif kind == 7:    # stale magic AND stale data on one device
            buf[s, devs[0], 0] ^= 0x40
            buf[s, devs[0], 4:4 + 64] ^= 0x33
        elif kind == 8:    # never written
            buf[s] = 0
        elif kind == 9:    # zero data, one device with a magic
            buf[s] = 0
            buf[s, devs[0], :4] = 7
        elif kind == 10:   # every chunk corrupted
            buf[s, :, 4 + 5] ^= 0x80
        # kind 0 / 11: clean
    return kinds


def make_buf(method, k, m, chunk, nstr, seed, legacy=False):
    data = np.stack([stripe(k, chunk, s + seed) for s in range(nstr)])
    with L.Plan.for_chunk(method, k, m, chunk) as p:
        img = p.segment_write(data, 1, 0)
    buf = logical_records(img, nstr, chunk, k + m)
    kinds = damage(buf, k, m, np.random.default_rng(seed), legacy)
    return data, buf, kinds


CASES = [(L.REED_SOL_VAN, 6, 3, 4096), (L.CAUCHY_GOOD, 6, 3, 8192), (L.REED_SOL_VAN, 4, 2, 2048),
         (L.CAUCHY_GOOD, 10, 4, 16384), (L.REED_SOL_VAN, 8, 3, 1024)]


@needs_ref
def test_reference_restatement_sanity(built):
    """The restated reference finds what it must: clean stripes pass, silent corruption of one
    chunk is located, too few matching magics are unrecoverable (CPU only)."""
    k, m, C = 6, 3, 1024
    rp = O.RefPlan(O.REED_SOL_VAN, k, m)
    data = np.stack([stripe(k, C, s) for s in range(4)])
    img = rp.segment_write(data, 4, C, 1, 0)
    buf = logical_records(img, 4, C, k + m)
    buf[1, 2, 4 + 9] ^= 1          # silent
    buf[2, 0, 0] ^= 1              # stale magic
    for d in range(4):
        buf[3, d, 1] ^= d + 1      # lost
    st, bm, rw, cnt, brute = rp.segment_inspect(buf.copy(), 4, C, 1, 0)
    assert st.tolist() == [0, 3, 2, 4]
    assert bm[1].tolist() == [0, 0, 1, 0, 0, 0, 0, 0, 0] and bm[2].tolist()[0] == 1
    assert cnt.tolist() == [3, 1, 1, 0] and brute[0] == 1
    out, rst, bad = rp.segment_read(img, 4, C, 1, 0, paranoid=1)
    assert bad == 0 and np.array_equal(out, data)


@pytest.mark.gpu
@needs_ref
@pytest.mark.parametrize("method,k,m,C", CASES)
@pytest.mark.parametrize("legacy", [False, True])
@pytest.mark.parametrize("fix", [False, True])
def test_inspect_matches_reference(cuda, method, k, m, C, legacy, fix):
    n, nstr = k + m, 48
    data, buf, kinds = make_buf(method, k, m, C, nstr, seed=k * 100 + C % 97 + 7 * legacy, legacy=legacy)
    with L.Plan.for_chunk(method, k, m, C) as p:
        ours = buf.copy()
        st, bm, rw, state = p.segment_inspect(ours, C, fix=fix, legacy_magic=legacy)
        rp = O.RefPlan(method, k, m, 8, p.packet_size)
        ref = buf.copy()
        rst, rbm, rrw, cnt, brute = rp.segment_inspect(ref, nstr, C, 0 if legacy else 1, int(fix))
    for s in range(nstr):
        assert st[s] == rst[s], (s, kinds[s], st[s], rst[s])
        assert np.array_equal(bm[s], rbm[s]), (s, kinds[s], bm[s], rbm[s])
    assert np.array_equal(rw, rrw)
    assert [state.bad_stripes, state.unrecoverable, state.silent_errors, state.empty_stripes] == cnt.tolist()
    assert state.brute_used == brute[0] and list(state.brute_badmap[:n]) == brute[1:].tolist()
    if fix:  # every record the inspection writes back is byte-identical
        sel = rw.astype(bool)
        assert np.array_equal(ours[sel], ref[sel])
    else:
        assert np.array_equal(ours, buf)  # without repair the buffer is left alone
    assert set(st.tolist()) >= {0, 1}


@pytest.mark.gpu
@needs_ref
def test_inspect_state_carries_between_calls(cuda):
    """Two calls over consecutive halves == one call (counters and the brute-force guess)."""
    method, k, m, C, nstr = L.REED_SOL_VAN, 6, 3, 4096, 40
    _, buf, _ = make_buf(method, k, m, C, nstr, seed=5)
    with L.Plan.for_chunk(method, k, m, C) as p:
        st_all, bm_all, _, s_all = p.segment_inspect(buf.copy(), C)
        state = E.InspectState()
        a = p.segment_inspect(np.ascontiguousarray(buf[:17]), C, state=state)
        b = p.segment_inspect(np.ascontiguousarray(buf[17:]), C, state=state)
    assert np.array_equal(np.concatenate([a[0], b[0]]), st_all)
    assert np.array_equal(np.concatenate([a[1], b[1]]), bm_all)
    assert (state.bad_stripes, state.silent_errors) == (s_all.bad_stripes, s_all.silent_errors)


@pytest.mark.gpu
@needs_ref
@pytest.mark.parametrize("method,k,m,C", CASES[:3])
@pytest.mark.parametrize("legacy", [False, True])
@pytest.mark.parametrize("paranoid", [False, True])
def test_read_matches_reference(cuda, method, k, m, C, legacy, paranoid):
    n, nstr, shift = k + m, 40, 1
    data, buf, kinds = make_buf(method, k, m, C, nstr, seed=3 * k + C % 89 + legacy, legacy=legacy)
    lc = C + 4
    img = np.zeros((n, nstr * lc), np.uint8)  # back to device images (LUN rotation)
    for s in range(nstr):
        for j in range(n):
            img[(j - s * shift) % n, s * lc:(s + 1) * lc] = buf[s, j]
    with L.Plan.for_chunk(method, k, m, C) as p:
        out, st, bad = p.segment_read(img, nstr, C, shift, 0, paranoid=paranoid, legacy_magic=legacy)
        rp = O.RefPlan(method, k, m, 8, p.packet_size)
        rout, rst, rbad = rp.segment_read(img, nstr, C, shift, 0, int(paranoid), 0 if legacy else 1)
    assert bad == rbad
    for s in range(nstr):
        assert st[s] == rst[s], (s, kinds[s], st[s], rst[s])
        if st[s] >= 0:
            assert np.array_equal(out[s], rout[s]), (s, kinds[s])


@pytest.mark.gpu
@needs_ref
@pytest.mark.parametrize("fix", [False, True])
def test_legacy_inspect_with_more_controls_than_one_compare_launch(cuda, fix):
    """Legacy magics with m = 18: up to m - |bad| = 17-18 control chunks per window, more than one
    chunk-compare launch holds (kMaxR = 16 pairs), so the comparison runs in several launches
    OR-ing into one flag per stripe.  Damage is limited to stale magics and single silent
    corruptions (the brute-force search over C(22, <= 17) sets would not finish for worse)."""
    method, k, m, C, nstr = L.REED_SOL_VAN, 4, 18, 1024, 12
    n = k + m
    data = np.stack([stripe(k, C, s + 77) for s in range(nstr)])
    with L.Plan.for_chunk(method, k, m, C) as p:
        img = p.segment_write(data, 1, 0)
    buf = logical_records(img, nstr, C, n)
    rng = np.random.default_rng(18)
    for s in range(nstr):
        buf[s, :, :4] = rng.integers(1, 255, 4, dtype=np.uint8)   # legacy: one arbitrary magic per stripe
        if s % 3 == 1:
            buf[s, int(rng.integers(0, n)), 0] ^= 0x11              # stale magic on one device
        elif s % 3 == 2:
            buf[s, int(rng.integers(0, n)), 4 + int(rng.integers(0, C))] ^= 0x5A  # silent corruption
    with L.Plan.for_chunk(method, k, m, C) as p:
        ours = buf.copy()
        st, bm, rw, state = p.segment_inspect(ours, C, fix=fix, legacy_magic=True)
        rp = O.RefPlan(method, k, m, 8, p.packet_size)
        ref = buf.copy()
        rst, rbm, rrw, cnt, brute = rp.segment_inspect(ref, nstr, C, 0, int(fix))
    assert st.tolist() == rst.tolist()
    assert np.array_equal(bm, rbm) and np.array_equal(rw, rrw)
    assert [state.bad_stripes, state.unrecoverable, state.silent_errors, state.empty_stripes] == cnt.tolist()
    assert 3 in st.tolist()   # the silent corruptions were found by the (short) brute-force search
    if fix:
        sel = rw.astype(bool)
        assert np.array_equal(ours[sel], ref[sel])


# The other codes of the plan API through the same read / inspect paths (raid4 has one parity
# chunk, r6 its own encode, the bitmatrix codes packets): (method, k, m, C, w, packet)
OTHER_CODES = [(L.RAID4, 6, 1, 4096, 8, 0), (L.REED_SOL_R6_OP, 6, 2, 4096, 8, 0), (L.CAUCHY_ORIG, 6, 3, 8192, 8, 0),
               (L.LIBERATION, 6, 2, 7 * 32 * 8, 7, 32), (L.BLAUM_ROTH, 6, 2, 6 * 24 * 8, 6, 24),
               (L.LIBER8TION, 6, 2, 8 * 32 * 8, 8, 32)]


def other_plan(method, k, m, C, w, packet):
    if packet:
        p = L.Plan.new(method, C, k, m, w, packet)
        p.form_encoding_matrix()
        p.form_decoding_matrix()
        return p
    return L.Plan.for_chunk(method, k, m, C)


@pytest.mark.gpu
@needs_ref
@pytest.mark.parametrize("method,k,m,C,w,packet", OTHER_CODES)
@pytest.mark.parametrize("legacy", [False, True])
def test_other_codes_read_and_inspect_match_reference(cuda, method, k, m, C, w, packet, legacy):
    n, nstr, shift = k + m, 36, 1
    data = np.stack([stripe(k, C, s + 31) for s in range(nstr)])
    with other_plan(method, k, m, C, w, packet) as p:
        rp = O.RefPlan(method, k, m, p.w, p.packet_size)
        img = p.segment_write(data, shift, 0)
        assert np.array_equal(img, rp.segment_write(data, nstr, C, shift, 0))
        buf = logical_records(img, nstr, C, n)
        kinds = damage(buf, k, m, np.random.default_rng(k + m + 5 * legacy), legacy)
        ours, ref = buf.copy(), buf.copy()
        st, bm, rw, state = p.segment_inspect(ours, C, fix=True, legacy_magic=legacy)
        rst, rbm, rrw, cnt, brute = rp.segment_inspect(ref, nstr, C, 0 if legacy else 1, 1)
        for s in range(nstr):
            assert st[s] == rst[s], (s, kinds[s], st[s], rst[s])
            assert np.array_equal(bm[s], rbm[s]), (s, kinds[s], bm[s], rbm[s])
        assert np.array_equal(rw, rrw)
        sel = rw.astype(bool)
        assert np.array_equal(ours[sel], ref[sel])
        dimg = np.zeros_like(img)
        lc = C + 4
        for s in range(nstr):
            for j in range(n):
                dimg[(j - s * shift) % n, s * lc:(s + 1) * lc] = buf[s, j]
        for paranoid in (False, True):
            out, rst_, bad = p.segment_read(dimg, nstr, C, shift, 0, paranoid=paranoid, legacy_magic=legacy)
            rout, rrst, rbad = rp.segment_read(dimg, nstr, C, shift, 0, int(paranoid), 0 if legacy else 1)
            assert bad == rbad and rst_.tolist() == rrst.tolist(), (paranoid, rst_.tolist(), rrst.tolist())
            for s in range(nstr):
                if rst_[s] >= 0:
                    assert np.array_equal(out[s], rout[s]), (s, kinds[s])


@pytest.mark.gpu
@pytest.mark.parametrize("method,k,m,C,w,packet", OTHER_CODES + [(L.REED_SOL_VAN, 6, 3, 4096, 8, 0)])
@pytest.mark.parametrize("missing", [0, 1])
def test_read_with_a_device_missing_rebuilds_every_stripe(cuda, method, k, m, C, w, packet, missing):
    """One device unreadable (NULL image); under the LUN rotation it holds a data chunk of some
    stripes and a parity chunk of others.  A stripe whose data devices all agree is returned as
    read (segment/jerasure.c:1416-1442); one missing a data device is rebuilt and verified.  In
    paranoid mode every stripe is verified, and raid4, whose decode leaves a lost parity alone
    (raid4.c:48), cannot verify a stripe without its parity: those stripes are unrecoverable, as
    in the reference, and their data is left out."""
    n, nstr = k + m, 2 * (k + m)
    data = np.stack([stripe(k, C, s + 5) for s in range(nstr)])
    held = [(missing + s) % n for s in range(nstr)]  # the logical chunk the missing device holds
    parity_lost = [s for s in range(nstr) if held[s] >= k]
    with other_plan(method, k, m, C, w, packet) as p:
        img = p.segment_write(data, 1, 0)
        for paranoid in (False, True):
            out, st, bad = p.segment_read(img, nstr, C, 1, 0, paranoid=paranoid, missing=(missing,))
            lost = parity_lost if paranoid and method == L.RAID4 else []
            assert bad == len(lost) and [s for s in range(nstr) if st[s] < 0] == lost, (paranoid, st.tolist())
            for s in range(nstr):
                assert st[s] == (-1 if s in lost else 1 if held[s] < k else 0), (s, st[s])
                if s not in lost:
                    assert np.array_equal(out[s], data[s]), s
