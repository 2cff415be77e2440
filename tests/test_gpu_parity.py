"""GPU parity: the HIP kernels behind the C ABI vs the reference's golden fixtures and the oracle.

Bar: bit-exact.  Every test goes through liblstore_ec.so -- the plan's fn-pointers
(encode_block / decode_block, as segment/jerasure.c:1847 / :245 call them), the batched
host calls, or the device-resident calls -- never through a Python or CPU fallback.
"""
import zlib

import numpy as np
import pytest

import lstore_amd as L
import oracle as O
from patterns import affine, stripe

pytestmark = pytest.mark.gpu


def assert_same(got, want):
    """bit-exact, or a message locating the differing bytes (stripe, shard, byte offsets)"""
    if np.array_equal(got, want):
        return
    d = np.argwhere(got != want)
    where = {}
    for idx in d:
        where.setdefault(tuple(int(x) for x in idx[:-1]), []).append(int(idx[-1]))
    msg = "; ".join(f"{k}: {len(v)} bytes in [{min(v)}, {max(v)}] got {got[k][min(v)]} want {want[k][min(v)]}"
                    for k, v in list(where.items())[:8])
    raise AssertionError(f"{len(d)} bytes differ: {msg}")

GPU_METHODS = (L.REED_SOL_VAN, L.REED_SOL_R6_OP, L.CAUCHY_ORIG, L.CAUCHY_GOOD, L.RAID4, L.LIBERATION, L.BLAUM_ROTH,
               L.LIBER8TION)


def case_input(v):
    return affine(v["k"], v["size"]) if v["pattern"] == "affine" else stripe(v["k"], v["size"], 0)


def make_plan(v):
    p = L.Plan.new(v["method"], v["size"], v["k"], v["m"], v["w"], v["packet"], 1 if v["method"] == L.RAID4 else 8)
    p.form_encoding_matrix()
    p.form_decoding_matrix()
    return p


def crcs(par):
    return ["%08x" % zlib.crc32(par[i].tobytes()) for i in range(par.shape[0])]


def gpu_cases(golden):
    return [v for v in golden["vectors"] if v["method"] in GPU_METHODS]


# ---------------------------------------------------------------- encode, host pointers via fn-pointer
def test_encode_block_matches_reference(cuda, golden):
    n = 0
    for v in gpu_cases(golden):
        data = case_input(v)
        par = np.full((v["m"], v["size"]), 0xA5, dtype=np.uint8)
        with make_plan(v) as p:
            p.encode_block([data[j] for j in range(v["k"])] + [par[i] for i in range(v["m"])])
        assert crcs(par) == v["parity_crc32"], (v["name"], v["k"], v["m"], v["size"])
        if v["full"]:
            assert np.array_equal(par, golden["small"][v["full"]])
        n += 1
    assert n >= 30


@pytest.mark.parametrize("method,k,w", [(L.LIBERATION, 7, 7), (L.LIBERATION, 11, 11), (L.BLAUM_ROTH, 10, 10),
                                        (L.BLAUM_ROTH, 4, 4), (L.LIBER8TION, 8, 8), (L.LIBER8TION, 3, 8),
                                        # w past the per-w kernels: the LDS-staged any-w kernel
                                        (L.LIBERATION, 37, 37), (L.LIBERATION, 32, 37), (L.BLAUM_ROTH, 36, 36),
                                        (L.BLAUM_ROTH, 40, 40),
                                        # k > 64: input groups + accumulate; w > 64: two output passes
                                        (L.LIBERATION, 67, 67), (L.LIBERATION, 71, 71)])
def test_liberation_family_vs_reference(cuda, method, k, w):
    """Generic GF(2) bitmatrix kernels vs the real reference (oracle/_ref) for every family member."""
    if not O.ref_available():
        pytest.skip("oracle/_ref not built")
    m, P = 2, 32
    size = w * P * 5
    data = stripe(k, size, w)
    rp = O.RefPlan(method, k, m, w, P)
    ref = rp.encode(data)
    par = np.zeros((m, size), np.uint8)
    with L.Plan.new(method, size, k, m, w, P, 8) as p:
        p.form_encoding_matrix()
        p.encode_block([data[j] for j in range(k)] + [par[i] for i in range(m)])
        assert np.array_equal(par, ref)
        full = np.vstack([data, par])
        for er in ([0], [k - 1], [k], [k + 1], [0, k - 1], [1, k], [k, k + 1]):
            sh = full.copy()
            sh[er] = 0
            assert p.decode_block([sh[i] for i in range(k + m)], er) == 0
            assert np.array_equal(sh, full), er


@pytest.mark.parametrize("method,k,w,P,nsuper", [
    (L.LIBERATION, 6, 7, 32, 40),     # 16 B lanes; 40 super-packets: a ragged last column tile
    (L.LIBERATION, 7, 7, 40, 33),     # P % 16 == 8: 8 B lanes
    (L.BLAUM_ROTH, 6, 6, 24, 50),     # (Jerasure packets are whole longs: P % 8 == 0)
    (L.LIBER8TION, 8, 8, 64, 24),
    (L.LIBER8TION, 3, 8, 16, 70),
    (L.BLAUM_ROTH, 16, 16, 32, 12),   # R*w = 32: 8 B lanes by the register cap
    # Cauchy at w = 8 / 16 / 32: the coefficient bitmatrices
    (L.CAUCHY_GOOD, 10, 8, 64, 30),   # w = 8, 8 B lanes
    (L.CAUCHY_ORIG, 8, 8, 32, 17),
    (L.CAUCHY_GOOD, 20, 8, 32, 9),    # 20 inputs, 6 outputs: 4 B lanes
    (L.CAUCHY_GOOD, 10, 16, 32, 20),  # 4 B lanes
    (L.CAUCHY_GOOD, 6, 32, 64, 9),
    (L.CAUCHY_ORIG, 5, 32, 16, 11),
])
def test_bitmatrix_network_vs_reference(cuda, method, k, w, P, nsuper):
    """Liberation-family codes on their compiled packet networks (ec_jit.cpp pktnet_source) once
    prepared: encode bit-exact vs the real reference (oracle/_ref), device-resident over three
    stripes and from host memory, and decodes of data, coding and mixed losses (double losses on
    a network) back to the encoded bytes (the MDS code's recovered bytes are unique)."""
    import torch

    if not O.ref_available():
        pytest.skip("oracle/_ref not built")
    m, n = (2 if method in (L.LIBERATION, L.BLAUM_ROTH, L.LIBER8TION) else 6 if k == 20 else 4), 3
    size = w * P * nsuper
    rng = np.random.default_rng(k * w + P)
    data = rng.integers(0, 256, (n, k, size), dtype=np.uint8)
    data[1] = 0xFF
    rp = O.RefPlan(method, k, m, w, P)
    want = np.stack([rp.encode(data[s]) for s in range(n)])
    losses = ([0], [k - 1], [k], [k + 1], [0, k - 1], [1, k], [k, k + 1]) + (([0, 2, k + 1, k + 3], [1, 3, 4]) if m >= 4 else ())
    # Cauchy at w = 8 with R <= 4 runs on the bit-sliced kernel by default (cauchy8_bitsliced_dw):
    # the hook puts every shape on its network, so the networks stay tested
    lib = L.lib()
    lib.lsec_test_set_cauchy8_policy(1)
    try:
        with L.Plan.new(method, size, k, m, w, P, 8) as p:
            assert p.form_encoding_matrix() == 0 and p.form_decoding_matrix() == 0
            p.prepare_encode()
            assert p.jit() == 1, "packet network not compiled"
            par = torch.full((n, m, size), 0x5A, dtype=torch.uint8, device="cuda")
            p.encode_dev(torch.from_numpy(data.copy()).cuda(), par)
            assert np.array_equal(par.cpu().numpy(), want)
            host = np.concatenate([data, np.zeros((n, m, size), np.uint8)], axis=1)
            p.encode_stripes(host)
            assert np.array_equal(host[:, k:], want)
            for er in losses:
                p.prepare_decode(er)
                if len(er) >= 2 and er[0] < k and method in (L.LIBERATION, L.BLAUM_ROTH, L.LIBER8TION):
                    assert p.jit(er) == 1, er  # two outputs on a network (single erasures: k_bitmatrix)
                sh = host.copy()
                sh[:, er] = 0x33
                p.decode_stripes(sh, er)
                assert_same(sh, host)
    finally:
        lib.lsec_test_set_cauchy8_policy(0)


@pytest.mark.parametrize("method,k,m,C,net", [
    (L.CAUCHY_GOOD, 10, 4, 4 << 20, False),   # c4: the bit-sliced kernel, 4 dwords per lane
    (L.CAUCHY_GOOD, 4, 2, 1 << 20, False),    # 1 dword per lane
    (L.CAUCHY_GOOD, 16, 4, 1 << 20, False),   # 4 dwords per lane from K = 16
    (L.CAUCHY_GOOD, 20, 6, 1 << 20, True),    # R = 6: the packet network
])
def test_cauchy8_kernel_by_shape(cuda, method, k, m, C, net):
    """Cauchy at w = 8 runs on the generic bit-sliced kernel for R <= 4 and on its compiled packet
    network beyond (cauchy8_bitsliced_dw, ec_plan.cpp; profiles/r06_v13_cauchy8_kernels_ab.txt):
    lsec_plan_jit says which, and the encode and a double-erasure decode are bit-exact against the
    reference either way, device-resident."""
    import torch

    if not O.ref_available():
        pytest.skip("oracle/_ref not built")
    n = 3
    with L.Plan.for_chunk(method, k, m, C) as p:
        p.prepare_encode()
        assert p.jit() == int(net), (k, m, C)
        rng = np.random.default_rng(k + C)
        data = rng.integers(0, 256, (n, k, C), dtype=np.uint8)
        rp = O.RefPlan(method, k, m, 8, p.packet_size)
        want = np.stack([rp.encode(data[s]) for s in range(n)])
        rp.close()
        d = torch.from_numpy(data).cuda()
        par = torch.full((n, m, C), 0x5A, dtype=torch.uint8, device="cuda")
        p.encode_dev(d, par)
        assert np.array_equal(par.cpu().numpy(), want)
        lost = [1, k]
        p.prepare_decode(lost)
        out = torch.zeros((n, 2, C), dtype=torch.uint8, device="cuda")
        p.decode_dev(d, par, lost, out=out)
        torch.cuda.synchronize()
        assert torch.equal(out[:, 0], d[:, 1]) and torch.equal(out[:, 1], par[:, 0])


@pytest.mark.parametrize("k", [128, 252])
def test_wide_liberation_decodes_round_trip(cuda, k):
    """Liberation with k = 128 (w = 131) and k = 252 (k + m = 254, w = nearest_prime(252) = 257
    from et_generate_plan, erasure_tools.c:756-757): encoded on the any-w bitmatrix kernel,
    bit-exact vs the real reference; then every kind of loss decodes back to the encoded bytes.
    The reference would decode lost data by inverting the whole (k*w)-square survivor bitmatrix
    (jerasure_invert_bitmatrix, jerasure.c:1049; 16 GB of ints at k = 252), which cannot finish
    here, so decode parity rests on the round trip (the MDS code's recovered bytes are unique)
    plus tests/test_bit_decode.py's rows-equal-the-dense-inversion check at small k."""
    if not O.ref_available():
        pytest.skip("oracle/_ref not built")
    m, P = 2, 8
    w = 131 if k == 128 else 257
    g = L.Plan.generate(k * w * 4096 * 2, L.LIBERATION, k, m)
    assert g.w == w
    g.close()
    size = w * P * 2
    data = stripe(k, size, w)
    ref = O.RefPlan(L.LIBERATION, k, m, w, P).encode(data)
    par = np.zeros((m, size), np.uint8)
    with L.Plan.new(L.LIBERATION, size, k, m, w, P, 8) as p:
        p.form_encoding_matrix()
        p.encode_block([data[j] for j in range(k)] + [par[i] for i in range(m)])
        assert np.array_equal(par, ref)
        full = np.vstack([data, par])
        for er in ([5], [k], [k, k + 1], [0, k - 1], [3, k + 1], [k - 1]):
            sh = full.copy()
            sh[er] = 0x5A
            assert p.decode_block([sh[i] for i in range(k + m)], er) == 0, (er, L.erasure.last_error())
            assert_same(sh, full)


# ---------------------------------------------------------------- wide fields (w = 16 / 32)
@pytest.mark.parametrize("method,k,m,w,size,P", [
    (L.REED_SOL_VAN, 6, 3, 16, 4104, 0),      # 4104 % 16 == 8: ragged last lane
    (L.REED_SOL_VAN, 10, 4, 32, 8200, 0),
    (L.REED_SOL_VAN, 20, 6, 16, 65536, 0),
    (L.REED_SOL_VAN, 12, 9, 32, 4096, 0),     # R = 9: launches of 4 + 4 + 1 rows at w = 32
    (L.REED_SOL_VAN, 4, 2, 16, 2 * 16384 + 8, 0),   # 3 transposed tiles, last one 8 bytes long
    (L.REED_SOL_VAN, 5, 3, 32, 3 * 32768 + 4104, 0),  # 4 tiles, last one ragged inside a lane
    (L.REED_SOL_R6_OP, 6, 2, 16, 2056, 0),
    (L.REED_SOL_R6_OP, 9, 2, 32, 4096, 0),
    (L.CAUCHY_GOOD, 6, 3, 16, 16 * 64 * 3, 64),
    (L.CAUCHY_ORIG, 5, 4, 16, 16 * 32 * 2, 32),
    (L.CAUCHY_GOOD, 10, 4, 32, 32 * 32 * 4, 32),
])
def test_wide_fields_vs_oracle(cuda, method, k, m, w, size, P):
    """RS / r6 over GF(2^16) / GF(2^32) (transposed bit-sliced kernel, little-endian words) and
    Cauchy at w = 16 / 32 (bit-sliced packet kernel): encode and every single + some double/triple
    erasure decodes, bit-exact vs the oracle restatement (pinned to the reference fixtures)."""
    import torch

    n = 3
    st = np.zeros((n, k + m, size), dtype=np.uint8)
    st[:, :k] = np.random.default_rng(k * w + m).integers(0, 256, (n, k, size), dtype=np.uint8)
    st[0, 0] = 0xFF
    with L.Plan.new(method, size, k, m, w, P, 8) as p:
        assert p.form_encoding_matrix() == 0 and p.form_decoding_matrix() == 0
        p.encode_stripes(st)
        for s in range(n):
            assert np.array_equal(st[s, k:], O.encode(method, st[s, :k], m, P, w)), s
        if O.ref_available():
            rp = O.RefPlan(method, k, m, w, P)
            assert np.array_equal(rp.encode(st[1, :k].copy()), st[1, k:])
            rp.close()
        full = st.copy()
        pats = [[e] for e in range(k + m)] + [[0, k], [k - 1, k + m - 1]]
        if m >= 3:
            pats.append([1, 2, k + 1])
        for pat in pats:
            st[:, pat] = 0x3C
            p.decode_stripes(st, pat)
            assert np.array_equal(st, full), pat
        d = torch.from_numpy(full[:, :k].copy()).to(cuda)
        par = torch.zeros((n, m, size), dtype=torch.uint8, device=cuda)
        p.encode_dev(d, par)
        out = torch.zeros((n, 2, size), dtype=torch.uint8, device=cuda)
        p.decode_dev(d, par, [0, k], out=out)
        torch.cuda.synchronize()
        assert np.array_equal(par.cpu().numpy(), full[:, k:])
        assert np.array_equal(out.cpu().numpy(), full[:, [0, k]])


# ---------------------------------------------------------------- encode, device-resident
def test_encode_dev_matches_reference(cuda, golden):
    import torch

    for v in gpu_cases(golden):
        data = torch.from_numpy(case_input(v)).to(cuda).unsqueeze(0).contiguous()
        par = torch.full((1, v["m"], v["size"]), 0x5A, dtype=torch.uint8, device=cuda)
        with make_plan(v) as p:
            p.encode_dev(data, par)
        torch.cuda.synchronize()
        assert crcs(par[0].cpu().numpy()) == v["parity_crc32"], (v["name"], v["k"], v["m"], v["size"])


# ---------------------------------------------------------------- decode (every erasure set of the fixtures)
def test_decode_block_matches_reference(cuda, golden):
    checked = 0
    for v in gpu_cases(golden):
        if not v["decode"]:
            continue
        data = case_input(v)
        with make_plan(v) as p:
            par = np.zeros((v["m"], v["size"]), dtype=np.uint8)
            p.encode_block([data[j] for j in range(v["k"])] + [par[i] for i in range(v["m"])])
            full = np.vstack([data, par])
            for d in v["decode"]:
                sh = full.copy()
                for e in d["erasures"]:
                    sh[e] = 0xEE
                rc = p.decode_block([sh[i] for i in range(sh.shape[0])], d["erasures"])
                assert rc == d["rc"], (v["name"], d["erasures"])
                if d["rc"] == 0 and d["recovered"] is not None:
                    assert np.array_equal(sh, full), (v["name"], v["k"], v["m"], d["erasures"])
                if d["recovered"] is None:  # raid4 lost parity: reference leaves it untouched
                    assert np.array_equal(sh[: v["k"]], full[: v["k"]])
                checked += 1
    assert checked > 100


def test_decode_dev_matches_reference_at_baseline_geometries(cuda, golden):
    """Device-resident decode at the BASELINE geometries the fixtures hold decodes for (c2/c3
    RS(6+3) 1 MiB, c4 Cauchy-good / RS(10+4) 4 MiB, ...): every erasure pattern the reference
    decoded, rebuilt shards compared with the CRC32 of what the reference rebuilt."""
    import torch

    checked = 0
    for v in gpu_cases(golden):
        if v["size"] < (1 << 20) or v["w"] != 8 or not v["decode"]:
            continue
        k, m, size = v["k"], v["m"], v["size"]
        data = torch.from_numpy(case_input(v)).to(cuda).unsqueeze(0).contiguous()
        par = torch.empty((1, m, size), dtype=torch.uint8, device=cuda)
        with make_plan(v) as p:
            p.encode_dev(data, par)
            for d in v["decode"]:
                if d["rc"] != 0 or not d["recovered"]:
                    continue
                er = sorted(set(d["erasures"]))
                out = torch.full((1, len(er), size), 0xEE, dtype=torch.uint8, device=cuda)
                p.decode_dev(data, par, er, out=out)
                torch.cuda.synchronize()
                assert crcs(out[0].cpu().numpy()) == d["rebuilt_crc32"], (v["name"], k, m, size, er)
                checked += 1
    assert checked >= 30


def test_decode_dev_roundtrip_all_single_and_double(cuda):
    import torch

    for method, k, m, size, P in [(L.REED_SOL_VAN, 6, 3, 65536, 0), (L.CAUCHY_GOOD, 10, 4, 65536, 1024),
                                  (L.CAUCHY_ORIG, 8, 3, 32768, 512), (L.REED_SOL_VAN, 20, 6, 16384, 0)]:
        n = 4
        g = torch.Generator(device="cpu").manual_seed(k * 100 + m)
        data = torch.randint(0, 256, (n, k, size), dtype=torch.uint8, generator=g).to(cuda)
        par = torch.empty((n, m, size), dtype=torch.uint8, device=cuda)
        with L.Plan.new(method, size, k, m, 8, P, 8) as p:
            p.form_encoding_matrix()
            p.encode_dev(data, par)
            pats = [[e] for e in range(k + m)] + [[0, k], [1, k - 1], [k - 1, k + m - 1]]
            if m >= 3:
                pats.append([0, 2, k + 1])
            for pat in pats:
                out = torch.full((n, len(pat), size), 0x11, dtype=torch.uint8, device=cuda)
                p.decode_dev(data, par, pat, out=out)
                torch.cuda.synchronize()
                full = torch.cat([data, par], dim=1)
                assert torch.equal(out, full[:, sorted(pat)]), (method, k, m, pat)


# ---------------------------------------------------------------- batched stripes vs oracle
def test_encode_stripes_host_batch_vs_oracle(cuda):
    for method, k, m, size, P in [(L.REED_SOL_VAN, 6, 3, 65536, 0), (L.CAUCHY_GOOD, 6, 3, 65536, 1024)]:
        n = 24
        st = np.zeros((n, k + m, size), dtype=np.uint8)
        for s in range(n):
            st[s, :k] = stripe(k, size, s)
        with L.Plan.new(method, size, k, m, 8, P, 8) as p:
            p.form_encoding_matrix()
            p.encode_stripes(st)
            for s in (0, 7, n - 1):
                assert np.array_equal(st[s, k:], O.encode(method, st[s, :k], m, P))
            lost = st[:, [0, k]].copy()
            st[:, [0, k]] = 0
            p.decode_stripes(st, [0, k])
            assert np.array_equal(st[:, [0, k]], lost)


def test_encode_dev_many_stripes_vs_oracle(cuda):
    import torch

    k, m, size, n = 6, 3, 1 << 20, 16
    data = torch.randint(0, 256, (n, k, size), dtype=torch.uint8, device=cuda)
    par = torch.empty((n, m, size), dtype=torch.uint8, device=cuda)
    with L.Plan.for_chunk(L.REED_SOL_VAN, k, m, size) as p:
        p.encode_dev(data, par)
        torch.cuda.synchronize()
        hd, hp = data.cpu().numpy(), par.cpu().numpy()
        for s in (0, 5, n - 1):
            assert np.array_equal(hp[s], O.encode(O.REED_SOL_VAN, hd[s], m))


# ---------------------------------------------------------------- edge cases the reference can hit
@pytest.mark.parametrize("size", [8, 16, 24, 1000, 4096 + 8, 8192 + 16, 65536 - 8])
def test_ragged_chunk_sizes_bytewise(cuda, size):
    size = size - size % 8
    k, m = 6, 3
    data = stripe(k, size, 3)
    par = np.zeros((m, size), dtype=np.uint8)
    with L.Plan.new(L.REED_SOL_VAN, size, k, m, 8, 8, 8) as p:
        p.form_encoding_matrix()
        p.encode_block([data[j] for j in range(k)] + [par[i] for i in range(m)])
        assert np.array_equal(par, O.encode(O.REED_SOL_VAN, data, m))
        full = np.vstack([data, par])
        sh = full.copy()
        sh[[1, 7]] = 0
        assert p.decode_block([sh[i] for i in range(k + m)], [1, 7]) == 0
        assert np.array_equal(sh, full)


@pytest.mark.parametrize("method,k,m,size", [
    (L.REED_SOL_VAN, 16, 4, 65536 + 4104),    # K >= 16: 16 B/lane shape + XOR-row path, ragged last tile
    (L.REED_SOL_VAN, 20, 6, 3 * 4096 + 8),
    (L.REED_SOL_VAN, 17, 5, 40960 + 16),      # generic-K kernel (KC = 0) with the XOR-row path
    (L.REED_SOL_VAN, 12, 10, 24576),          # R = 10 > 8: two launches (rows 0-7 with the XOR row, 8-9)
    (L.REED_SOL_R6_OP, 20, 2, 32768 + 24),    # r6: P row all ones
    (L.CAUCHY_ORIG, 10, 4, 8192),             # bitsliced (no all-ones row): unaffected control
])
def test_xor_row_and_wide_shapes_vs_oracle(cuda, method, k, m, size):
    """Kernel paths chosen by code width: wide codes (16 B/lane), the plain-XOR first row (all-ones
    coefficients) and launches split at 8 rows -- encode and decodes whose first decode row is
    all ones (P0 lost with data) or not, bit-exact vs the oracle."""
    import torch

    n = 3
    P = 128 if method == L.CAUCHY_ORIG else 0
    st = np.zeros((n, k + m, size), dtype=np.uint8)
    st[:, :k] = np.random.default_rng(k * 7 + m).integers(0, 256, (n, k, size), dtype=np.uint8)
    with L.Plan.new(method, size, k, m, 8, P or 8, 8) as p:
        assert p.form_encoding_matrix() == 0 and p.form_decoding_matrix() == 0
        d = torch.from_numpy(st[:, :k].copy()).to(cuda)
        par = torch.zeros((n, m, size), dtype=torch.uint8, device=cuda)
        p.encode_dev(d, par)
        torch.cuda.synchronize()
        hp = par.cpu().numpy()
        for s in range(n):
            assert np.array_equal(hp[s], O.encode(method, st[s, :k], m, P)), s
        full = np.concatenate([st[:, :k], hp], axis=1)
        for pat in ([k], [0, k], [1, k, k + m - 1], [0], list(range(min(m, 3)))):
            if len(pat) > m:
                continue
            sh = full.copy()
            sh[:, pat] = 0x77
            p.decode_stripes(sh, pat)
            assert np.array_equal(sh, full), pat


@pytest.mark.parametrize("method,k,m,size", [
    (L.REED_SOL_VAN, 40, 4, 8192),        # k beyond the compile-time K list: generic-K kernel
    (L.CAUCHY_GOOD, 40, 4, 8 * 64 * 4),
    (L.REED_SOL_VAN, 48, 16, 4096),       # R = 16: two 8-row launches
    (L.CAUCHY_ORIG, 30, 34, 8 * 32 * 2),  # more parity than data
    (L.REED_SOL_VAN, 70, 2, 4096),        # k > 64: two input groups, the second accumulating
    (L.REED_SOL_VAN, 100, 28, 4104),      # k + m = 128, ragged 8-byte tail
    (L.CAUCHY_GOOD, 100, 28, 8 * 64 * 2),
    (L.CAUCHY_ORIG, 120, 8, 8 * 32 * 2),
    (L.REED_SOL_VAN, 200, 56, 2048),      # k + m = 256: Jerasure's limit at w = 8 (reed_sol.c:247)
])
def test_wide_stripes_vs_oracle(cuda, method, k, m, size):
    """Stripes up to k + m = 256 (LSEC_MAX_DEVS): encode from host and device memory, stripe
    magic (in launches of 80 shards) and erasures spread over every input group, bit-exact vs
    the oracle and zlib."""
    import torch
    n = 2
    P = 64 if method == L.CAUCHY_GOOD else (32 if method == L.CAUCHY_ORIG else 0)
    st = np.zeros((n, k + m, size), dtype=np.uint8)
    st[:, :k] = np.random.default_rng(k + m).integers(0, 256, (n, k, size), dtype=np.uint8)
    with L.Plan.new(method, size, k, m, 8, P or 8, 8) as p:
        assert p.form_encoding_matrix() == 0 and p.form_decoding_matrix() == 0
        magic = p.encode_stripes_magic(st)
        for s in range(n):
            assert np.array_equal(st[s, k:], O.encode(method, st[s, :k], m, P)), s
            assert np.array_equal(magic[s], _je_magic(st[s])), s
        data = torch.from_numpy(st[:, :k].copy()).cuda()
        par = torch.zeros((n, m, size), dtype=torch.uint8, device="cuda")
        p.encode_dev(data, par)
        assert np.array_equal(par.cpu().numpy(), st[:, k:])
        full = st.copy()
        spread = list(range(0, k + m, max(1, (k + m) // m)))[:m]  # one erasure per stretch of devices
        for pat in ([0], [k + m - 1], list(range(min(m, 6))), [1, k, k + 1][: m], spread):
            st[:, pat] = 0x42
            p.decode_stripes(st, pat)
            assert np.array_equal(st, full), pat
        pat = spread
        dev = torch.from_numpy(full.copy()).cuda()
        dev[:, pat] = 0x42
        p.decode_dev(dev[:, :k], dev[:, k:], pat)
        assert np.array_equal(dev.cpu().numpy(), full)


@pytest.mark.parametrize("k,m,size", [
    (20, 6, 65536),          # RS(20+6): the c5 wide code, whole 16 B lanes
    (20, 6, 4096 * 3 + 24),  # ragged: the last lane's 16 B piece is 8 B
    (16, 6, 40968),          # R * K = 96: the smallest matrix served by a network
    (32, 8, 8192),           # the widest network (K = 32, R = 8)
    (12, 8, 16384 + 40),     # R = 8 over K = 12: 8 B lanes, ragged last lane
])
def test_xor_network_vs_oracle(cuda, k, m, size):
    """Wide RS codes run on their compiled XOR networks (ec_jit.cpp) once prepared: encode and
    an m-device decode (R = m rows over K = k survivors) bit-exact vs the oracle, device-resident
    and from host memory."""
    import torch
    n = 3
    rng = np.random.default_rng(k * 100 + m)
    st = np.zeros((n, k + m, size), dtype=np.uint8)
    st[:, :k] = rng.integers(0, 256, (n, k, size), dtype=np.uint8)
    st[1, :k] = 0xFF  # every bit set: every Horner step's doubling reduces
    lost = list(range(m))  # data shards 0..m-1: the decode matrix is dense
    with L.Plan.new(L.REED_SOL_VAN, size, k, m, 8, 8, 8) as p:
        assert p.form_encoding_matrix() == 0 and p.form_decoding_matrix() == 0
        p.prepare_encode()
        p.prepare_decode(lost)
        assert p.jit() == 1 and p.jit(lost) == 1, "network not compiled"
        want = np.stack([O.encode(L.REED_SOL_VAN, st[s, :k], m, 0) for s in range(n)])
        data = torch.from_numpy(st[:, :k].copy()).cuda()
        par = torch.full((n, m, size), 0x5A, dtype=torch.uint8, device="cuda")
        p.encode_dev(data, par)
        assert np.array_equal(par.cpu().numpy(), want)
        host = st.copy()
        p.encode_stripes(host)
        assert np.array_equal(host[:, k:], want)
        full = host.copy()
        host[:, lost] = 0x33
        p.decode_stripes(host, lost)
        assert_same(host, full)


@pytest.mark.parametrize("method,k,m,w,size,lost", [
    (L.REED_SOL_VAN, 6, 3, 16, 3 * 16384 + 40, [0, 1, 2]),   # ragged tail: the generic kernel finishes it
    (L.REED_SOL_VAN, 6, 3, 32, 2 * 32768, [1, 6 + 1]),
    (L.REED_SOL_VAN, 10, 4, 32, 2 * 32768 + 8, [0, 3, 5, 9]),
    (L.REED_SOL_VAN, 10, 4, 16, 16384 + 16, [2, 10 + 2]),
    (L.REED_SOL_VAN, 20, 6, 16, 16384 + 8, [0, 5, 7, 11, 13, 19]),
    (L.REED_SOL_R6_OP, 6, 2, 32, 32768 + 24, [0, 4]),
    (L.REED_SOL_VAN, 4, 2, 32, 8, [0, 1]),                  # smaller than one tile: generic kernel only
    (L.REED_SOL_VAN, 5, 3, 32, 5 * 16384 + 16, [0, 2, 4]),  # odd input count: a lone last input per tile
    (L.REED_SOL_VAN, 7, 4, 32, 3 * 16384, [1, 7, 8, 10]),   # decode mixing data and coding losses
    (L.REED_SOL_VAN, 10, 6, 32, 2 * 16384 + 8, [0, 2, 4, 6, 8, 13]),  # 6 rows: the split's widest
    (L.REED_SOL_VAN, 9, 5, 32, 16384, [1, 3, 5, 9, 12]),   # 5 rows, odd input count
    (L.REED_SOL_VAN, 19, 8, 16, 2 * 8192 + 16, [0, 2, 3, 7, 11, 18, 19, 26]),  # w = 16 split, 8 rows
])
def test_gfw_network_vs_oracle(cuda, method, k, m, w, size, lost):
    """RS / r6 at w = 16 / 32 run on their compiled bit-sliced XOR networks (ec_jit.cpp,
    gfw_source) once prepared: encode and a dense decode bit-exact vs the oracle restatement
    (pinned to the reference fixtures), device-resident and from host memory, with ragged tails
    and all-0xFF stripes (every reduction tap used)."""
    import torch

    n = 3
    rng = np.random.default_rng(k * w + m)
    st = np.zeros((n, k + m, size), dtype=np.uint8)
    st[:, :k] = rng.integers(0, 256, (n, k, size), dtype=np.uint8)
    st[1, :k] = 0xFF
    with L.Plan.new(method, size, k, m, w, 8, 8) as p:
        assert p.form_encoding_matrix() == 0 and p.form_decoding_matrix() == 0
        p.prepare_encode()
        p.prepare_decode(lost)
        assert p.jit() == 1 and p.jit(lost) == 1, "network not compiled"
        want = np.stack([O.encode(method, st[s, :k], m, 0, w) for s in range(n)])
        R = 2 if method == L.REED_SOL_R6_OP else m
        data = torch.from_numpy(st[:, :k].copy()).cuda()
        par = torch.full((n, m, size), 0x5A, dtype=torch.uint8, device="cuda")
        p.encode_dev(data, par)
        assert np.array_equal(par.cpu().numpy()[:, :R], want[:, :R])
        host = st.copy()
        p.encode_stripes(host)
        assert np.array_equal(host[:, k:k + R], want[:, :R])
        full = host.copy()
        host[:, lost] = 0x33
        p.decode_stripes(host, lost)
        assert_same(host, full)


@pytest.mark.parametrize("w,k,m", [(8, 200, 57), (16, 1000, 25), (32, 1020, 5)])
def test_stripe_width_limits_are_errors(cuda, w, k, m):
    """Stripes wider than the engine takes -- k + m > 256 at w = 8 (Jerasure's own limit there,
    reed_sol.c:247-248), > 1024 at w = 16 / 32 -- are refused with a message, never written
    past a table."""
    size = 64
    with L.Plan.new(L.REED_SOL_VAN, size, k, m, w, 8, 8) as p:
        st = np.zeros((1, k + m, size), np.uint8)
        with pytest.raises(L.ErasureError, match="k\\+m"):
            p.encode_stripes(st)


@pytest.mark.parametrize("method,k,m,w,size", [
    (L.REED_SOL_VAN, 300, 24, 16, 4104),     # 5 input groups, 3 row launches, ragged tail
    (L.REED_SOL_VAN, 280, 6, 32, 1024),      # k + m = 286: 5 input groups, 2 row launches
    (L.CAUCHY_GOOD, 260, 8, 16, 2 * 16 * 8),  # bit-sliced GF(2^16), packet 8
])
def test_wide_word_stripes_vs_oracle(cuda, method, k, m, w, size):
    """At w = 16 / 32 Jerasure takes k + m up to 2^w (reed_sol.c:247-248, cauchy.c:139); the engine
    takes up to 1024 there.  Encode from host and device memory, and decodes with erasures in
    every input group, bit-exact vs the oracle restatement."""
    import torch
    n = 2
    P = 8 if method == L.CAUCHY_GOOD else 0
    rng = np.random.default_rng(k * w + m)
    st = np.zeros((n, k + m, size), dtype=np.uint8)
    st[:, :k] = rng.integers(0, 256, (n, k, size), dtype=np.uint8)
    with L.Plan.new(method, size, k, m, w, P or 8, 8) as p:
        assert p.form_encoding_matrix() == 0 and p.form_decoding_matrix() == 0
        p.encode_stripes(st)
        for s in range(n):
            assert_same(st[s, k:], O.encode(method, st[s, :k], m, P, w))
        data = torch.from_numpy(st[:, :k].copy()).cuda()
        par = torch.zeros((n, m, size), dtype=torch.uint8, device="cuda")
        p.encode_dev(data, par)
        assert np.array_equal(par.cpu().numpy(), st[:, k:])
        full = st.copy()
        for pat in ([0], [k - 1, k + m - 1], list(range(0, k, k // min(m, 8)))[:m], [1, 65, 129, k])[: 4]:
            pat = sorted(set(pat))[:m]
            st[:, pat] = 0x42
            p.decode_stripes(st, pat)
            assert_same(st, full)


def test_randomized_plans_vs_oracle(cuda):
    """Seeded random plans across methods, word sizes, k, m, chunk and packet sizes, with
    random erasure sets: every parity and every rebuilt shard bit-exact vs the oracle."""
    import torch

    rng = np.random.default_rng(20261016)
    checked = 0
    for case in range(48):
        method = int(rng.choice([L.REED_SOL_VAN, L.REED_SOL_R6_OP, L.CAUCHY_ORIG, L.CAUCHY_GOOD, L.RAID4]))
        w = 8 if method == L.RAID4 or case % 4 else int(rng.choice([16, 32]))
        k = int(rng.integers(1, 25))
        m = 2 if method == L.REED_SOL_R6_OP else 1 if method == L.RAID4 else int(rng.integers(1, 9))
        if method in (L.CAUCHY_ORIG, L.CAUCHY_GOOD):
            P = 8 * int(rng.integers(1, 17))
            size = w * P * int(rng.integers(1, 5))
        else:
            P = 0
            size = 8 * int(rng.integers(1, 1025))
        n = int(rng.integers(1, 4))
        data = rng.integers(0, 256, (n, k, size), dtype=np.uint8)
        with L.Plan.new(method, size, k, m, w, P or 8, 1 if method == L.RAID4 else 8) as p:
            p.form_encoding_matrix()
            p.form_decoding_matrix()
            d = torch.from_numpy(data).to(cuda)
            par = torch.zeros((n, m, size), dtype=torch.uint8, device=cuda)
            p.encode_dev(d, par)
            torch.cuda.synchronize()
            hp = par.cpu().numpy()
            for s in range(n):
                assert np.array_equal(hp[s], O.encode(method, data[s], m, P, w)), (case, method, w, k, m, size, P)
            full = np.concatenate([data, hp], axis=1)
            e = int(rng.integers(1, m + 1))
            lost = sorted(rng.choice(k + m, size=e, replace=False).tolist())
            if method == L.RAID4 and lost[0] >= k:
                continue  # raid4.c:48 leaves a lost parity alone
            sh = full.copy()
            sh[:, lost] = 0x99
            p.decode_stripes(sh, lost)
            assert np.array_equal(sh, full), (case, method, w, k, m, size, P, lost)
            checked += 1
    assert checked >= 40


@pytest.mark.parametrize("P", [8, 16, 24, 40, 4096])
def test_bitsliced_packet_sizes(cuda, P):
    k, m = 6, 3
    size = 8 * P * 3
    data = stripe(k, size, 1)
    par = np.zeros((m, size), dtype=np.uint8)
    with L.Plan.new(L.CAUCHY_GOOD, size, k, m, 8, P, 8) as p:
        p.form_encoding_matrix()
        p.encode_block([data[j] for j in range(k)] + [par[i] for i in range(m)])
        assert np.array_equal(par, O.encode(O.CAUCHY_GOOD, data, m, P))


def test_error_paths(cuda):
    k, m = 6, 3
    with L.Plan.new(L.REED_SOL_VAN, 1024, k, m, 8, 8, 8) as p:
        p.form_encoding_matrix()
        sh = [np.zeros(1024, np.uint8) for _ in range(k + m)]
        assert p.decode_block(sh, []) == 0                       # nothing erased
        assert p.decode_block(sh, [0, 1, 2, 3]) == -1            # > m erasures
        assert p.decode_block(sh, [k + m]) == -1                 # out of range
        assert p.decode_block(sh, [2, 2]) == 0                   # duplicates collapse
        assert p.decode_block(sh, [0], block_size=1020) == -1    # not a multiple of 8
    with L.Plan.new(L.CAUCHY_GOOD, 4096, k, m, 8, 64, 8) as p:
        p.form_encoding_matrix()
        sh = [np.zeros(1024, np.uint8) for _ in range(k + m)]
        assert p.decode_block(sh, [0], block_size=1000) == -1    # not a multiple of w*packet
    with L.Plan.new(L.RAID4, 1024, k, 1, 8, 1, 1) as p:
        sh = [np.zeros(1024, np.uint8) for _ in range(k + 1)]
        assert p.decode_block(sh, [1, 1]) == -1                  # raid4.c:47 checks erasures[1]


def test_device_pointers_through_fn_pointer(cuda):
    """encode_block / decode_block with device pointers: used in place, no staging."""
    import torch

    k, m, size = 6, 3, 1 << 16
    data = torch.randint(0, 256, (k, size), dtype=torch.uint8, device=cuda)
    par = torch.zeros((m, size), dtype=torch.uint8, device=cuda)
    with L.Plan.for_chunk(L.REED_SOL_VAN, k, m, size) as p:
        p.encode_block([data[j].data_ptr() for j in range(k)] + [par[i].data_ptr() for i in range(m)], size)
        ref = O.encode(O.REED_SOL_VAN, data.cpu().numpy(), m)
        assert np.array_equal(par.cpu().numpy(), ref)
        keep = data[2].clone()
        data[2].zero_()
        rc = p.decode_block([data[j].data_ptr() for j in range(k)] + [par[i].data_ptr() for i in range(m)], [2], size)
        assert rc == 0
        assert torch.equal(data[2], keep)


def test_mixed_device_and_host_pointers_refused(cuda):
    """Stripes whose chunk pointers mix device and host memory are refused with a status, not
    launched: device-first batches have every chunk of their first and last stripe checked,
    multi-stripe host-first batches the last chunk of their first and last stripe."""
    import torch

    from lstore_amd import erasure as E

    k, m, size = 6, 3, 1 << 12
    dev = torch.zeros((2, k + m, size), dtype=torch.uint8, device=cuda)
    host = np.zeros((2, k + m, size), dtype=np.uint8)
    with L.Plan.for_chunk(L.REED_SOL_VAN, k, m, size) as p:
        dptr = [[dev[s, i].data_ptr() for i in range(k + m)] for s in range(2)]
        hptr = [[host[s, i].ctypes.data for i in range(k + m)] for s in range(2)]
        cases = [(dptr[0][:4] + hptr[0][4:], 1), (dptr[0][:-1] + hptr[0][-1:], 1),
                 (dptr[0] + dptr[1][:-1] + hptr[1][-1:], 2), (hptr[0] + hptr[1][:-1] + dptr[1][-1:], 2),
                 (hptr[0][:-1] + dptr[0][-1:] + hptr[1], 2)]
        for ptrs, n in cases:
            with pytest.raises(E.ErasureError, match="mix device and host"):
                p.encode_stripes_ptrs(L.Plan._ptr_array(ptrs), n, size)


# ---------------------------------------------------------------- full-size, size-independent properties
def test_full_size_roundtrip_and_linearity(cuda):
    import torch

    k, m, size, n = 6, 3, 1 << 20, 256   # 1.5 GiB of data
    g = torch.Generator(device=cuda).manual_seed(7)
    a = torch.randint(0, 256, (n, k, size), dtype=torch.uint8, device=cuda, generator=g)
    b = torch.randint(0, 256, (n, k, size), dtype=torch.uint8, device=cuda, generator=g)
    pa = torch.empty((n, m, size), dtype=torch.uint8, device=cuda)
    pb = torch.empty_like(pa)
    pab = torch.empty_like(pa)
    with L.Plan.for_chunk(L.REED_SOL_VAN, k, m, size) as p:
        p.encode_dev(a, pa)
        p.encode_dev(b, pb)
        p.encode_dev(a ^ b, pab)
        assert torch.equal(pab, pa ^ pb)  # GF(2^8)-linear
        for pat in ([0], [k - 1], [k], [k + 1], [0, 3, k + 2]):
            out = torch.empty((n, len(pat), size), dtype=torch.uint8, device=cuda)
            p.decode_dev(a, pa, pat, out=out)
            assert torch.equal(out, torch.cat([a, pa], 1)[:, pat])
    with L.Plan.for_chunk(L.CAUCHY_GOOD, k, m, size) as p:
        p.encode_dev(a, pa)
        p.encode_dev(b, pb)
        p.encode_dev(a ^ b, pab)
        assert torch.equal(pab, pa ^ pb)
        out = torch.empty((n, 1, size), dtype=torch.uint8, device=cuda)
        p.decode_dev(a, pa, [0], out=out)
        assert torch.equal(out[:, 0], a[:, 0])
    torch.cuda.synchronize()


def test_host_path_many_batches(cuda):
    """et_encode_stripes / et_decode_stripes across several staging batches (pipelined slots)."""
    k, m, size, n = 6, 3, 1 << 20, 40   # 64 MiB staging -> 7 stripes per batch -> 6 batches
    st = np.zeros((n, k + m, size), dtype=np.uint8)
    rng = np.random.default_rng(3)
    st[:, :k] = rng.integers(0, 256, (n, k, size), dtype=np.uint8)
    with L.Plan.for_chunk(L.REED_SOL_VAN, k, m, size) as p:
        p.encode_stripes(st)
        for s in range(n):
            assert np.array_equal(st[s, k:], O.encode(O.REED_SOL_VAN, st[s, :k], m)), s
        keep = st[:, [1, k + 2]].copy()
        st[:, [1, k + 2]] = 0
        p.decode_stripes(st, [1, k + 2])
        assert np.array_equal(st[:, [1, k + 2]], keep)


@pytest.mark.parametrize("method,k,m,size", [(L.REED_SOL_VAN, 20, 6, 4 << 20), (L.CAUCHY_GOOD, 10, 4, 8 << 20)])
def test_host_path_column_blocks(cuda, method, k, m, size):
    """Stripes larger than half the staging budget are processed as column blocks."""
    n = 2
    st = np.zeros((n, k + m, size), dtype=np.uint8)
    st[:, :k] = np.random.default_rng(k).integers(0, 256, (n, k, size), dtype=np.uint8)
    with L.Plan.for_chunk(method, k, m, size) as p:
        p.encode_stripes(st)
        for s in range(n):
            assert np.array_equal(st[s, k:], O.encode(method, st[s, :k], m, p.packet_size)), s
        keep = st[:, [0, k - 1, k]].copy()
        st[:, [0, k - 1, k]] = 7
        p.decode_stripes(st, [0, k - 1, k])
        assert np.array_equal(st[:, [0, k - 1, k]], keep)


def _pinned(shape):
    import torch

    return torch.empty(shape, dtype=torch.uint8, pin_memory=True).numpy()


@pytest.mark.parametrize("method,k,m,size,n", [(L.REED_SOL_VAN, 6, 3, 1 << 20, 40), (L.CAUCHY_GOOD, 10, 4, 8 << 20, 2)])
def test_host_path_pinned_buffers(cuda, method, k, m, size, n):
    """Page-locked caller buffers are DMA'd in place (no packing), across staging batches and
    column blocks; results identical to the oracle and to the pageable path."""
    st = _pinned((n, k + m, size))
    st[:] = 0
    st[:, :k] = np.random.default_rng(n).integers(0, 256, (n, k, size), dtype=np.uint8)
    ref = st.copy()
    with L.Plan.for_chunk(method, k, m, size) as p:
        p.encode_stripes(st)
        p.encode_stripes(ref)  # pageable copy through the packing path
        assert np.array_equal(st, ref)
        for s in (0, n // 2, n - 1):
            assert np.array_equal(st[s, k:], O.encode(method, st[s, :k], m, p.packet_size)), s
        keep = st[:, [1, k + 1]].copy()
        st[:, [1, k + 1]] = 0x5A
        p.decode_stripes(st, [1, k + 1])
        assert np.array_equal(st[:, [1, k + 1]], keep)


@pytest.mark.parametrize("method", [L.REED_SOL_VAN, L.CAUCHY_GOOD])
def test_strided_dma_lattices(cuda, method):
    """Pinned-DMA batches go as strided copies when their runs repeat at one stripe stride
    (issue_runs, ec_pinning.cpp): one lane (encode's data chunks), several lanes (erasures that
    split the survivors into runs of different lengths), and pointer arrays whose stripes do NOT
    sit at one stride (two allocations, stripes in shuffled order) -- every result equal to the
    oracle's."""
    k, m, size, n = 8, 4, 4 << 20, 6  # 4 MiB chunks: runs well above the in-place pinning thresholds
    rng = np.random.default_rng(11)
    st = np.zeros((n, k + m, size), np.uint8)
    st[:, :k] = rng.integers(0, 256, (n, k, size), dtype=np.uint8)
    with L.Plan.for_chunk(method, k, m, size) as p:
        p.encode_stripes(st)
        for s in (0, n - 1):
            assert np.array_equal(st[s, k:], O.encode(method, st[s, :k], m, p.packet_size)), s
        full = st.copy()
        for erased in ([2, 5, 9], [0, 3, 6, 11], [1, 8]):
            st[:, erased] = 0x3C
            p.decode_stripes(st, erased)
            assert np.array_equal(st, full), erased
        # stripes from two allocations, in shuffled order: no single stride
        a = full[: n // 2].copy()
        b = full[n // 2:].copy()
        order = [3, 0, 5, 1, 4, 2]
        rows = [(a if i < n // 2 else b)[i % (n // 2)] for i in order]
        for r in rows:
            r[k:] = 0
        addrs = [r[i].ctypes.data for r in rows for i in range(k + m)]
        p.encode_stripes_ptrs(p._ptr_array(addrs), n, size)
        for r, i in zip(rows, order):
            assert np.array_equal(r, full[i]), i
        for r in rows:
            r[[1, 2, k]] = 0
        p.decode_stripes_ptrs(p._ptr_array(addrs), n, size, [1, 2, k])
        for r, i in zip(rows, order):
            assert np.array_equal(r, full[i]), i


@pytest.mark.parametrize("method,k,m,size,n,w", [
    (L.REED_SOL_VAN, 8, 3, 512 << 10, 24, 8), (L.REED_SOL_VAN, 4, 2, 1 << 20, 16, 8),
    (L.REED_SOL_VAN, 16, 4, 256 << 10, 32, 8), (L.CAUCHY_GOOD, 6, 3, 1 << 20, 12, 8),
    (L.CAUCHY_GOOD, 10, 4, 2 << 20, 6, 8), (L.REED_SOL_VAN, 6, 3, 1 << 20, 12, 16),
    (L.CAUCHY_GOOD, 8, 4, 1 << 20, 8, 32)])
def test_host_batches_match_device_path(cuda, method, k, m, size, n, w):
    """Every stripe of a pageable host batch (pinned in place, strided copies; or packed) equals
    the device-resident path's result byte for byte, for encode and for decodes whose erasures
    split the survivors into one, two and three runs per stripe."""
    import torch

    rng = np.random.default_rng(k * 100 + m + w)
    st = np.zeros((n, k + m, size), np.uint8)
    st[:, :k] = rng.integers(0, 256, (n, k, size), dtype=np.uint8)
    with L.Plan.for_chunk(method, k, m, size, w=w) as p:
        d = torch.from_numpy(st[:, :k].copy()).cuda()
        par = torch.empty((n, m, size), dtype=torch.uint8, device="cuda")
        p.encode_dev(d, par)
        p.encode_stripes(st)
        torch.cuda.synchronize()
        assert np.array_equal(st[:, k:], par.cpu().numpy())
        full = st.copy()
        for erased in ([0], [1, k], [2, 5 % k, k + m - 1]):
            erased = sorted(set(erased))[:m]
            st[:, erased] = 0x96
            p.decode_stripes(st, erased)
            assert np.array_equal(st, full), erased


def test_pageable_batches_pinned_in_place_share_inputs(cuda):
    """Large pageable batches are pinned in place (hipHostRegister) for the call.  Threads that
    encode from the SAME data chunks at once (each into its own parity buffers) contend for
    the registration: the loser packs instead, nobody DMAs from pages another call is about
    to unregister, and every parity equals the oracle's."""
    import threading

    k, m, size, n = 6, 3, 1 << 20, 6  # 36 MiB of data: above the in-place threshold
    data = np.random.default_rng(7).integers(0, 256, (n, k, size), dtype=np.uint8)
    with L.Plan.for_chunk(L.REED_SOL_VAN, k, m, size) as p:
        want = [O.encode(O.REED_SOL_VAN, data[s], m) for s in range(n)]
        errors = []

        def worker(t):
            try:
                par = np.zeros((n, m, size), np.uint8)
                addrs = []
                for s in range(n):
                    addrs += [data[s, i].ctypes.data for i in range(k)]
                    addrs += [par[s, j].ctypes.data for j in range(m)]
                arr = p._ptr_array(addrs)
                for it in range(4):
                    par[:] = 0
                    p.encode_stripes_ptrs(arr, n, size)
                    for s in range(n):
                        if not np.array_equal(par[s], want[s]):
                            errors.append((t, it, s))
            except Exception as e:  # noqa: BLE001
                errors.append((t, repr(e)))

        th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errors, errors[:5]
        # and a pageable decode of a batch whose chunks are one dense region per stripe
        st = np.zeros((n, k + m, size), np.uint8)
        st[:, :k] = data
        p.encode_stripes(st)
        full = st.copy()
        st[:, [0, 4, k + 2]] = 0xA5
        p.decode_stripes(st, [0, 4, k + 2])
        assert np.array_equal(st, full)


@pytest.mark.parametrize("method", [L.REED_SOL_VAN, L.CAUCHY_GOOD])
def test_fn_pointer_pinned_and_pageable_callers_coalesced(cuda, method):
    """Concurrent single-stripe calls, half on page-locked and half on pageable buffers, go
    through the dispatcher together; each gets its own parity and rebuilds.  The page-locked
    ones (384 KiB runs) move by the copy-piece kernel, the pageable ones are packed."""
    import threading

    k, m, size = 6, 3, 65536
    with L.Plan.for_chunk(method, k, m, size) as p:
        errors = []

        def worker(t):
            try:
                rng = np.random.default_rng(100 + t)
                sh = _pinned((k + m, size)) if t % 2 else np.empty((k + m, size), np.uint8)
                for it in range(5):
                    sh[:k] = rng.integers(0, 256, (k, size), dtype=np.uint8)
                    sh[k:] = 0
                    p.encode_block([sh[i] for i in range(k + m)])
                    if not np.array_equal(sh[k:], O.encode(method, sh[:k], m, p.packet_size)):
                        errors.append((t, it, "encode"))
                    full = sh.copy()
                    lost = [(t + it) % (k + m)]
                    sh[lost] = 0
                    if p.decode_block([sh[i] for i in range(k + m)], lost) != 0 or not np.array_equal(sh, full):
                        errors.append((t, it, "decode"))
            except Exception as ex:  # noqa: BLE001
                errors.append((t, repr(ex)))

        threads = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
        for th in threads:
            th.start()
        for th in threads:
            th.join()
        assert not errors, errors


@pytest.mark.parametrize("devices", [(0, 0), (0, 0, 0)])
def test_host_batches_split_over_device_set(cuda, devices):
    """lsec_set_host_devices: a large host batch is cut into stripe ranges driven by one thread
    per listed device (here the one GPU listed several times), small calls round-robin; results
    identical to the oracle, including magics and decodes."""
    from lstore_amd import erasure as E

    k, m, size, n = 6, 3, 1 << 20, 23
    st = np.zeros((n, k + m, size), dtype=np.uint8)
    st[:, :k] = np.random.default_rng(len(devices)).integers(0, 256, (n, k, size), dtype=np.uint8)
    E.set_host_devices(devices)
    try:
        with L.Plan.for_chunk(L.CAUCHY_GOOD, k, m, size) as p:
            magic = p.encode_stripes_magic(st)
            for s in range(n):
                assert np.array_equal(st[s, k:], O.encode(O.CAUCHY_GOOD, st[s, :k], m, p.packet_size)), s
                assert np.array_equal(magic[s], _je_magic(st[s])), s
            assert np.array_equal(p.stripes_magic(st), magic)
            keep = st[:, [2, k]].copy()
            st[:, [2, k]] = 0
            p.decode_stripes(st, [2, k])
            assert np.array_equal(st[:, [2, k]], keep)
            one = st[5].copy()                       # a single small call (round-robin path)
            one[k:] = 0
            p.encode_block([one[i] for i in range(k + m)])
            assert np.array_equal(one, st[5])
    finally:
        E.set_host_devices(())
    with pytest.raises(L.ErasureError, match="outside"):
        E.set_host_devices((0, 99))


# ---------------------------------------------------------------- stripe magic (adler32, segment/jerasure.c:169-182)
def _je_magic(full):
    """je_cksum_calc: adler32 over the k+m chunks in order, 4 bytes little-endian (zlib)."""
    a = 1
    for row in full:
        a = zlib.adler32(row.tobytes(), a)
    return np.frombuffer(np.uint32(a).tobytes(), dtype=np.uint8)


@pytest.mark.parametrize("method,k,m,size", [(L.REED_SOL_VAN, 6, 3, 65536), (L.CAUCHY_GOOD, 10, 4, 1 << 20),
                                             (L.REED_SOL_VAN, 6, 3, 8200), (L.REED_SOL_VAN, 20, 6, 4 << 20)])
def test_stripe_magic_matches_zlib(cuda, method, k, m, size):
    import torch

    n = 5
    st = np.zeros((n, k + m, size), dtype=np.uint8)
    st[:, :k] = np.random.default_rng(size % 977).integers(0, 256, (n, k, size), dtype=np.uint8)
    st[1, :k] = 0xFF  # worst case for the modular sums
    with L.Plan.for_chunk(method, k, m, size) as p:
        magic = p.encode_stripes_magic(st)          # host path: GPU encode + GPU magic
        for s in range(n):
            assert np.array_equal(st[s, k:], O.encode(method, st[s, :k], m, p.packet_size))
            assert np.array_equal(magic[s], _je_magic(st[s])), s
        assert np.array_equal(p.stripes_magic(st), magic)
        d = torch.from_numpy(st[:, :k].copy()).to(cuda)
        par = torch.zeros((n, m, size), dtype=torch.uint8, device=cuda)
        mg = torch.zeros((n, 4), dtype=torch.uint8, device=cuda)
        p.encode_magic_dev(d, par, mg)
        torch.cuda.synchronize()
        assert np.array_equal(mg.cpu().numpy(), magic)


# ---------------------------------------------------------------- file tools et_encode / et_decode
@pytest.mark.parametrize("method,k,m", [(L.REED_SOL_VAN, 6, 3), (L.CAUCHY_GOOD, 4, 2)])
def test_file_tools_roundtrip(cuda, tmp_path, method, k, m):
    """et_encode / et_decode (erasure_tools.c:339-600): strip i of the data file at foffset + i*strip,
    parity strip i of the parity file at poffset + i*strip; missing data strips rebuilt in place."""
    import ctypes as C

    fsize = 3 * 1000 * 1000 + 17
    with L.Plan.generate(fsize, method, k, m) as p:
        strip = p.strip_size
        rng = np.random.default_rng(9)
        raw = rng.integers(0, 256, fsize, dtype=np.uint8)
        dfile, pfile = tmp_path / "data.bin", tmp_path / "parity.bin"
        foff, poff = 100, 7
        buf = np.full(foff + k * strip, ord("0"), np.uint8)   # bread pads with '0' past EOF
        buf[foff:foff + fsize] = raw
        dfile.write_bytes(buf[:foff + fsize].tobytes())
        lib = L.lib()
        assert lib.et_encode(p.ptr, str(dfile).encode(), foff, str(pfile).encode(), poff, 1 << 20) == 0
        strips = buf[foff:foff + k * strip].reshape(k, strip)
        par = O.encode(method, strips, m, p.packet_size)
        got = np.frombuffer(pfile.read_bytes(), np.uint8)
        for i in range(m):
            assert np.array_equal(got[poff + i * strip: poff + (i + 1) * strip], par[i]), i
        # lose data strip 1 and parity strip 0, rebuild
        damaged = bytearray(dfile.read_bytes())
        damaged[foff + strip: foff + 2 * strip] = b"\xee" * strip
        dfile.write_bytes(bytes(damaged))
        er = (C.c_int * 3)(1, k, -1)
        assert lib.et_decode(p.ptr, foff + fsize, str(dfile).encode(), foff, str(pfile).encode(), poff, 1 << 20, er) == 0
        fixed = np.frombuffer(dfile.read_bytes(), np.uint8)
        assert np.array_equal(fixed[foff:foff + fsize], raw)


# ---------------------------------------------------------------- gop-pool style concurrency
def test_concurrent_fn_pointer_calls(cuda):
    """encode_block / decode_block called from many threads on one shared plan (segment/jerasure.c:1937)."""
    import threading

    k, m, size = 6, 3, 65536
    with L.Plan.for_chunk(L.CAUCHY_GOOD, k, m, size) as p:
        errors = []

        def worker(t):
            try:
                rng = np.random.default_rng(t)
                for it in range(6):
                    data = rng.integers(0, 256, (k, size), dtype=np.uint8)
                    par = np.zeros((m, size), np.uint8)
                    p.encode_block([data[j] for j in range(k)] + [par[i] for i in range(m)])
                    if not np.array_equal(par, O.encode(O.CAUCHY_GOOD, data, m, p.packet_size)):
                        errors.append((t, it, "encode"))
                    full = np.vstack([data, par])
                    sh = full.copy()
                    lost = [(t + it) % (k + m), (t + it + 3) % (k + m)]
                    sh[lost] = 0
                    if p.decode_block([sh[i] for i in range(k + m)], lost) != 0 or not np.array_equal(sh, full):
                        errors.append((t, it, "decode"))
            except Exception as ex:  # noqa: BLE001
                errors.append((t, repr(ex)))

        threads = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
        for th in threads:
            th.start()
        for th in threads:
            th.join()
        assert not errors, errors


def test_hbm_copy_probe(cuda):
    """lsec_hbm_copy_dev (bench.py's HBM ceiling probe) copies exactly, ragged tails included,
    and refuses misaligned or non-16-multiple sizes."""
    import torch

    from lstore_amd import erasure as E

    lib = E.lib()
    st = torch.cuda.current_stream().cuda_stream
    for n in (0, 16, 8192, 8192 + 48, (3 << 20) + 16 * 7):
        src = torch.randint(0, 256, (n + 16,), dtype=torch.uint8, device=cuda)
        dst = torch.zeros(n + 16, dtype=torch.uint8, device=cuda)
        assert lib.lsec_hbm_copy_dev(dst.data_ptr(), src.data_ptr(), n, st) == 0
        torch.cuda.synchronize()
        assert torch.equal(dst[:n], src[:n])
        assert not dst[n:].any()
    buf = torch.zeros(64, dtype=torch.uint8, device=cuda)
    assert lib.lsec_hbm_copy_dev(buf.data_ptr(), buf.data_ptr() + 32, 24, st) == -1
    assert lib.lsec_hbm_copy_dev(buf.data_ptr() + 8, buf.data_ptr() + 32, 16, st) == -1


def test_hbm_mix_probe(cuda):
    """lsec_hbm_mix_dev (bench.py's encode-traffic probe) writes the XOR of the k inputs to each
    of the m outputs of every stripe, ragged tails included, and refuses bad arguments."""
    import torch

    from lstore_amd import erasure as E

    lib = E.lib()
    st = torch.cuda.current_stream().cuda_stream
    for k, m, C, N in ((6, 3, 8192 + 24, 5), (10, 4, 65536, 3), (1, 1, 8, 2)):
        d = torch.randint(0, 256, (N, k, C), dtype=torch.uint8, device=cuda)
        p = torch.zeros((N, m, C), dtype=torch.uint8, device=cuda)
        refs = [(d.data_ptr() + j * C, k * C) for j in range(k)] + [(p.data_ptr() + r * C, m * C) for r in range(m)]
        arr = L.Plan.shard_refs(refs)
        assert lib.lsec_hbm_mix_dev(arr, k, m, N, C, st) == 0
        torch.cuda.synchronize()
        x = np.bitwise_xor.reduce(d.cpu().numpy(), axis=1)
        for r in range(m):
            assert np.array_equal(p[:, r].cpu().numpy(), x)
    assert lib.lsec_hbm_mix_dev(arr, 0, 1, 1, 8, st) == -1
    assert lib.lsec_hbm_mix_dev(arr, 1, 1, 1, 12, st) == -1


# ---------------------------------------------------------------- SURVEY §8d c2 correctness patterns
def _special_stripes(k, size, P):
    """All-zero, all-0xFF and single-bit stripes: stripe 2 + j*8 + t has only bit t of one byte
    of data shard j set (the byte moves across packets and super-packet words with j and t),
    so every coefficient's action on every bit position is seen in isolation."""
    n = 2 + 8 * k
    st = np.zeros((n, k, size), dtype=np.uint8)
    st[1] = 0xFF
    for j in range(k):
        for t in range(8):
            off = ((j * 8 + t) * (P + 4) + 4 * t + j) % size
            st[2 + j * 8 + t, j, off] = 1 << t
    return st


@pytest.mark.parametrize("method,k,m,size", [(L.REED_SOL_VAN, 6, 3, 1 << 16), (L.CAUCHY_GOOD, 6, 3, 1 << 16),
                                             (L.CAUCHY_GOOD, 10, 4, 1 << 17), (L.REED_SOL_VAN, 10, 4, 1 << 16)])
def test_zero_ones_and_single_bit_patterns(cuda, method, k, m, size):
    """Device-resident encode (+ fused magic) and decodes on all-zero, all-0xFF and single-bit
    stripes: parity bit-exact vs the real reference when its build is present
    (else the restatement), magic vs zlib, every single and some double erasures rebuilt."""
    import torch

    with L.Plan.for_chunk(method, k, m, size) as p:
        P = p.packet_size
        hd = _special_stripes(k, size, max(P, 64))
        n = hd.shape[0]
        d = torch.from_numpy(hd).to(cuda)
        par = torch.full((n, m, size), 0x5A, dtype=torch.uint8, device=cuda)
        mg = torch.zeros((n, 4), dtype=torch.uint8, device=cuda)
        p.encode_magic_dev(d, par, mg)
        torch.cuda.synchronize()
        hp, hm = par.cpu().numpy(), mg.cpu().numpy()
        rp = O.RefPlan(method, k, m, 8, P) if O.ref_available() else None
        try:
            for s in range(n):
                want = rp.encode(hd[s].copy()) if rp else O.encode(method, hd[s], m, P)
                assert np.array_equal(hp[s], want), s
                assert np.array_equal(hm[s], _je_magic(np.vstack([hd[s], hp[s]]))), s
        finally:
            if rp:
                rp.close()
        assert not hp[0].any()                      # zero data -> zero parity
        full = np.concatenate([hd, hp], axis=1)
        pats = [[e] for e in range(k + m)] + [[0, 1], [k - 1, k], [0, k + m - 1]]
        for pat in pats:
            out = torch.zeros((n, len(pat), size), dtype=torch.uint8, device=cuda)
            p.decode_dev(d, par, pat, out=out)
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy(), full[:, pat]), pat


@pytest.mark.parametrize("method,k,m,size,n,shift,pinned", [(L.REED_SOL_VAN, 6, 3, 64 << 10, 200, 0, False),
                                                            (L.CAUCHY_GOOD, 10, 4, 256 << 10, 16, 0, False),
                                                            (L.REED_SOL_VAN, 20, 6, 32 << 10, 120, 0, False),
                                                            (L.REED_SOL_VAN, 6, 3, 64 << 10, 200, 8, False),
                                                            (L.REED_SOL_VAN, 6, 3, 64 << 10, 200, 0, True),
                                                            (L.CAUCHY_GOOD, 6, 3, 64 << 10, 64, 0, True),
                                                            (L.REED_SOL_VAN, 6, 3, 64 << 10, 40, 8, True)])
def test_small_run_batches(cuda, method, k, m, size, n, shift, pinned):
    """Large batches of small chunks (LStore's [stripe][k+m][C] pages, runs well under 4 MiB):
    pageable ones pack (no kernel ever touches per-call registrations of pageable pages, see
    InPlacePin); caller page-locked buffers (pinned=True) with small runs move by the copy-piece
    kernel after every chunk is checked, 8-byte-misaligned ones (shift=8) DMA.  Encode and a
    double-erasure decode are bit-exact either way."""
    _small_runs_case(method, k, m, size, n, shift, pinned)


def _small_runs_case(method, k, m, size, n, shift, pinned):
    if pinned:
        import torch
        raw = torch.zeros(n * (k + m) * size + 64, dtype=torch.uint8, pin_memory=True).numpy()
    else:
        raw = np.zeros(n * (k + m) * size + 64, dtype=np.uint8)
    off = (-raw.ctypes.data) % 16 + shift
    st = raw[off:off + n * (k + m) * size].reshape(n, k + m, size)
    st[:, :k] = np.random.default_rng(size + k).integers(0, 256, (n, k, size), dtype=np.uint8)
    with L.Plan.for_chunk(method, k, m, size) as p:
        p.encode_stripes(st)
        for s in (0, n // 3, n - 1):
            assert np.array_equal(st[s, k:], O.encode(method, st[s, :k], m, p.packet_size)), s
        full = st.copy()
        p.encode_stripes(st)                         # repeat: slots and piece lists reused
        assert np.array_equal(st, full)
        st[:, [1, k + m - 1]] = 0xA5
        p.decode_stripes(st, [1, k + m - 1])
        assert np.array_equal(st, full)


# ---------------------------------------------------------------- work-sharing tiles
# (launches of at least kTileQueueMinTiles = 16384 tiles take the queue)
@pytest.mark.parametrize("method,k,m,size,n", [
    (L.REED_SOL_VAN, 6, 3, 1 << 20, 160),     # the headline kernel (bytewise, 8 KiB tiles): 20480 tiles
    (L.REED_SOL_VAN, 20, 6, 256 << 10, 300),  # K >= 16 bytewise shape (4 KiB tiles), before any network binds
    (L.CAUCHY_GOOD, 6, 3, 1 << 20, 160),      # bit-sliced (1 KiB of packet columns per tile)
    (L.REED_SOL_VAN, 6, 3, 1000, 20001),      # ragged tiles, one per stripe; more than the persistent grid
])
def test_tile_sharing_is_bit_identical(cuda, method, k, m, size, n):
    """Work-sharing tiles (ec_kernels.h): workgroups that take tiles from an atomic counter per XCD
    eighth and then help the other eighths, for all tiles (shared) or after a static 7/8 of each
    eighth (tail).  Every tile must be coded exactly once: encode, decode and the fused stripe magic
    give the same bytes in every mode, launch after launch (the queue slots rotate and reset
    themselves), and match the oracle on sampled stripes."""
    import torch

    from lstore_amd import erasure as E

    g = torch.Generator(device=cuda).manual_seed(11)
    d = torch.randint(0, 256, (n, k, size), dtype=torch.uint8, device=cuda, generator=g)
    outs = {}
    try:
        with L.Plan.for_chunk(method, k, m, size) as p:
            for on in (E.TILES_STATIC, E.TILES_SHARED, E.TILES_TAIL, E.TILES_SHARED, E.TILES_STATIC, E.TILES_TAIL):
                E.set_tile_sharing(on)
                par = torch.zeros((n, m, size), dtype=torch.uint8, device=cuda)
                mg = torch.zeros((n, 4), dtype=torch.uint8, device=cuda)
                p.encode_magic_dev(d, par, mg)
                rb = torch.zeros((n, 2, size), dtype=torch.uint8, device=cuda)
                p.decode_dev(d, par, [0, k], out=rb)
                torch.cuda.synchronize()
                assert torch.equal(rb[:, 0], d[:, 0]) and torch.equal(rb[:, 1], par[:, 0]), on
                if on in outs:
                    assert torch.equal(par, outs[on][0]) and torch.equal(mg, outs[on][1]), on
                outs[on] = (par, mg)
            for mode in (E.TILES_SHARED, E.TILES_TAIL):
                assert torch.equal(outs[mode][0], outs[E.TILES_STATIC][0]), mode
                assert torch.equal(outs[mode][1], outs[E.TILES_STATIC][1]), mode
            hd, hp = d.cpu().numpy(), outs[E.TILES_TAIL][0].cpu().numpy()
            for s in (0, n // 2, n - 1):
                assert_same(hp[s], O.encode(method, hd[s], m, p.packet_size))
    finally:
        E.set_tile_sharing(E.TILES_TAIL)


def test_tile_sharing_concurrent_streams(cuda):
    """Launches from several threads on their own streams at once: each takes its own queue slot
    (one ring per device), so concurrent launches never share counters."""
    import threading

    import torch

    k, m, size, n = 6, 3, 256 << 10, 600  # 19200 tiles per launch: the queue path
    g = torch.Generator(device=cuda).manual_seed(5)
    d = torch.randint(0, 256, (n, k, size), dtype=torch.uint8, device=cuda, generator=g)
    with L.Plan.for_chunk(L.REED_SOL_VAN, k, m, size) as p:
        want = torch.empty((n, m, size), dtype=torch.uint8, device=cuda)
        p.encode_dev(d, want)
        torch.cuda.synchronize()
        errs = []

        def worker(i):
            try:
                s = torch.cuda.Stream()
                with torch.cuda.stream(s):
                    for _ in range(20):
                        par = torch.empty((n, m, size), dtype=torch.uint8, device=cuda)
                        p.encode_dev(d, par, stream=s)
                        s.synchronize()
                        if not torch.equal(par, want):
                            errs.append(i)
            except Exception as e:  # noqa: BLE001
                errs.append(repr(e))

        ts = [threading.Thread(target=worker, args=(i,)) for i in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert errs == []


POOL_SCRIPT = r"""
import ctypes, sys, threading
import numpy as np
sys.path.insert(0, sys.argv[1])
import lstore_amd as L
import oracle as O
lib = L.lib()
lib.lsec_test_staging_pool.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_longlong)]
k, m, C, n = 6, 3, 1 << 20, 32  # 288 MiB contiguous: pinned in place, slots of ~252 MiB of HBM
errors = []
plan = L.Plan.for_chunk(L.REED_SOL_VAN, k, m, C)
bar = threading.Barrier(8)


def worker(t):
    try:
        st = np.zeros((n, k + m, C), np.uint8)
        st[:, :k] = np.random.default_rng(t).integers(0, 256, (n, k, C), dtype=np.uint8)
        bar.wait()
        for _ in range(2):
            plan.encode_stripes(st)
        for s in (0, n - 1):
            if not np.array_equal(st[s, k:], O.encode(L.REED_SOL_VAN, st[s, :k], m, 0)):
                errors.append((t, s))
    except Exception as e:
        errors.append((t, repr(e)))


th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
for x in th:
    x.start()
for x in th:
    x.join()
out = (ctypes.c_longlong * 3)()
lib.lsec_test_staging_pool(0, out)
print(list(out), errors)
assert not errors, errors
assert out[0] >= 3 and out[1] <= 2, list(out)  # several pipelines ran; at most 2 keep the large halves
assert out[2] <= 2 * 3 * (300 << 20) + out[0] * 3 * (64 << 20), list(out)
print("ok")
"""


def test_staging_pool_keeps_at_most_two_large_device_halves(cuda):
    """Eight threads of large pageable batches (pinned in place, so their slots take the large
    device geometry, LSEC_DEV_STAGING_MB): afterwards at most two pooled pipelines keep their
    large device halves, so the HBM the pool holds does not grow with the peak thread count
    (ADVICE r05); every batch's parity bit-exact."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", POOL_SCRIPT, root], capture_output=True, text=True, timeout=110)
    assert out.returncode == 0 and out.stdout.strip().endswith("ok"), (out.stdout[-800:], out.stderr[-1500:])


@pytest.mark.parametrize("method,k,m,C,n,w", [
    (L.REED_SOL_VAN, 6, 3, 1 << 20, 64, 8),        # K1, tile queue (static 7/8 + shared tail)
    (L.REED_SOL_VAN, 6, 3, 65536 + 8, 9, 8),       # K1, static eighths, ragged last tile
    (L.CAUCHY_GOOD, 10, 4, 4 << 20, 12, 8),        # compiled packet network
    (L.REED_SOL_VAN, 20, 6, 256 << 10, 40, 8),     # compiled XOR network
    (L.REED_SOL_VAN, 10, 4, 1 << 20, 10, 16),      # compiled w = 16 network
])
def test_xcd_tile_phase_is_bit_identical(cuda, method, k, m, C, n, w):
    """The XCD tile phase (lsec_test_set_tile_phase; ApplyArgs::tile_phase, the networks' Args::phase)
    only changes which tile a workgroup takes: encode and single-erasure decode write the same bytes
    with it on and off, in the bytewise kernel's queue and static forms and in the compiled networks
    (mode 3 = both; the default, 1, has it on for the tile loops only)."""
    import torch

    lib = L.lib()
    with L.Plan.for_chunk(method, k, m, C, w) as p:
        p.prepare_encode()
        p.prepare_decode([1])
        g = torch.Generator(device=cuda).manual_seed(C + k)
        d = torch.randint(0, 256, (n, k, C), dtype=torch.uint8, device=cuda, generator=g)
        outs = []
        try:
            for phase in (0, 3, 1):
                lib.lsec_test_set_tile_phase(phase)
                par = torch.zeros((n, m, C), dtype=torch.uint8, device=cuda)
                p.encode_dev(d, par)
                rb = torch.zeros((n, 1, C), dtype=torch.uint8, device=cuda)
                p.decode_dev(d, par, [1], out=rb)
                torch.cuda.synchronize()
                outs.append((par, rb))
        finally:
            lib.lsec_test_set_tile_phase(1)  # the default
        for par, rb in outs[1:]:
            assert torch.equal(par, outs[0][0])
            assert torch.equal(rb[:, 0], d[:, 1])
        hp = outs[0][0][0].cpu().numpy()
        assert np.array_equal(hp, O.encode(method, d[0].cpu().numpy(), m, p.packet_size, w=w))
