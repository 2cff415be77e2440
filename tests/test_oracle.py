"""The oracle (CPU restatement, oracle/ec_oracle.c) pinned against the reference.

Pins, in order of strength:
  1. tests/golden/*  -- produced by the real reference (vendor/jerasure + raid4.c compiled from
     /root/reference by oracle/Makefile; generator tests/golden/make_golden.py)
  2. the known-answer anchors of SURVEY.md §8c (reference probe, input D_j[b] = (131j+7b+1) mod 256)
  3. oracle/_ref itself, when it is built (build container only)
"""
import hashlib
import zlib

import numpy as np
import pytest

import oracle as O
from patterns import affine, stripe


def case_input(v):
    return affine(v["k"], v["size"]) if v["pattern"] == "affine" else stripe(v["k"], v["size"], 0)


def test_oracle_encode_matches_golden(built, golden):
    n = 0
    for v in golden["vectors"]:
        if v["method"] in (O.BLAUM_ROTH, O.LIBERATION, O.LIBER8TION):
            continue  # the restatement has no liberation-family matrix builders (bitmatrix-only codes)
        data = case_input(v)
        par = O.encode(v["method"], data, v["m"], v["packet"], v["w"])
        assert ["%08x" % zlib.crc32(par[i].tobytes()) for i in range(v["m"])] == v["parity_crc32"], v
        assert [par[i][:16].tobytes().hex() for i in range(v["m"])] == v["parity_head"]
        if v["full"]:
            assert np.array_equal(par, golden["small"][v["full"]])
        n += 1
    assert n >= 60


def test_oracle_decode_matches_golden(built, golden):
    for v in golden["vectors"]:
        if v["method"] in (O.BLAUM_ROTH, O.LIBERATION, O.LIBER8TION) or not v["decode"] or v["size"] > 65536:
            continue
        data = case_input(v)
        par = O.encode(v["method"], data, v["m"], v["packet"], v["w"])
        full = np.vstack([data, par])
        for d in v["decode"]:
            sh = full.copy()
            for e in d["erasures"]:
                sh[e] = 0
            rc = O.decode(v["method"], sh, v["k"], d["erasures"], v["packet"], v["w"])
            if v["method"] == O.RAID4:
                # raid4_decode: >1 listed -> -1; lost parity -> untouched (raid4.c:47-52)
                if len(d["erasures"]) > 1:
                    assert d["rc"] == -1
                    continue
            assert rc == d["rc"], (v["name"], d)
            if rc == 0 and d["recovered"]:
                assert np.array_equal(sh, full)
            if rc == 0 and "rebuilt_crc32" in d and d["recovered"] is not None:
                got = ["%08x" % zlib.crc32(sh[e].tobytes()) for e in sorted(set(d["erasures"]))]
                assert got == d["rebuilt_crc32"], (v["name"], d["erasures"])


def test_golden_decode_covers_c4(golden):
    """The fixtures hold the reference's decodes at the c4 geometry (Cauchy-good 10+4 and RS 10+4,
    C = 4 MiB): every erasure pattern, with the CRC32 of the shards it rebuilt."""
    c4 = [v for v in golden["vectors"] if v["k"] == 10 and v["m"] == 4 and v["size"] == 4 << 20]
    assert {v["name"] for v in c4} == {"cauchy_good", "reed_sol_van"}
    for v in c4:
        ok = [d for d in v["decode"] if d["rc"] == 0]
        assert len(ok) >= 9 and all(d["recovered"] and d["rebuilt_crc32"] for d in ok)


# SURVEY.md §8c known-answer anchors (first 16 parity bytes / CRC32 per parity chunk)
ANCHORS = [
    (O.REED_SOL_VAN, 6, 3, 1024, 0, ["758aafc8", "423889eb", "dc91fbb9"],
     ["959f958bbd878dfbf58f959b8d879d8b", "34a12d25c638b2ae7e59a1751a25d3e3", "3d502e450bbdc37761a73a41275ad7a0"]),
    (O.CAUCHY_GOOD, 6, 3, 1024, 16, ["758aafc8", "fab531b6", "fc576e98"],
     [None, "da41082f16fd240b329980476e55bc63", "0cd02c2064a0c4c0bc105c2024c08440"]),
    (O.CAUCHY_GOOD, 10, 4, 4096, 64, ["68384314", "a4ea4f16", "5f2fa058", "54c29b92"],
     ["959b9d97ad8bf5fff58bad979d9b958f", "cdf0dbc6e9ec77726508331e01242fca",
      "d8e8e8f8e8d8a8b82858586878685828", "889bb6b984b7d23540d3eef1fccfea6d"]),
    (O.REED_SOL_VAN, 10, 4, 4096, 0, ["68384314", "6c0eb30a", "75b29d5f", "7d4e02ef"], None),
]


@pytest.mark.parametrize("meth,k,m,size,P,crc,head", ANCHORS)
def test_survey_anchors(built, meth, k, m, size, P, crc, head):
    par = O.encode(meth, affine(k, size), m, P)
    assert ["%08x" % zlib.crc32(par[i].tobytes()) for i in range(m)] == crc
    if head:
        for i, h in enumerate(head):
            if h:
                assert par[i][:16].tobytes().hex() == h


def test_survey_matrices(built):
    # SURVEY.md §8a a4/a5 (probe output of the reference)
    assert O.coding_matrix(O.REED_SOL_VAN, 6, 3).tolist() == [[1] * 6, [1, 225, 151, 172, 82, 200],
                                                               [1, 123, 245, 143, 244, 142]]
    assert O.coding_matrix(O.CAUCHY_GOOD, 6, 3).tolist() == [[1] * 6, [200, 151, 172, 1, 225, 166],
                                                              [202, 143, 114, 101, 200, 1]]
    assert O.coding_matrix(O.CAUCHY_GOOD, 10, 4)[3].tolist() == [1, 172, 123, 158, 195, 31, 143, 227, 82, 34]
    assert int(O.bitmatrix(O.coding_matrix(O.CAUCHY_GOOD, 10, 4)).sum()) == 888
    assert int(O.bitmatrix(O.coding_matrix(O.CAUCHY_GOOD, 20, 6)).sum()) == 3085


# et_generate_plan(k*C, cauchy_good, 6, 3, -1, -1, -1) packet sizes (reference probe)
@pytest.mark.parametrize("chunk,packet,strip", [(16384, 256, 16384), (65536, 1024, 65536), (262144, 4096, 262144),
                                                (1 << 20, 4096, 1 << 20), (196608, 3072, 196608),
                                                (100000, 784, 100352)])
def test_generate_plan_packets(built, chunk, packet, strip):
    g = O.generate_plan(6 * chunk, O.CAUCHY_GOOD, 6, 3)
    assert (g["packet_size"], g["strip_size"], g["w"]) == (packet, strip, 8)


def test_oracle_matrices_match_golden_plans(built, golden):
    for e in golden["plans"]:
        if e["matrix"] is None:
            continue
        mat = O.coding_matrix(e["method"], e["k"], e["m"], e["w"])
        assert mat is not None and mat.tolist() == e["matrix"], (e["name"], e["k"], e["m"], e["w"])
        if e["bitmatrix_ones"] is not None:
            assert int(O.bitmatrix(mat, e["w"]).sum()) == e["bitmatrix_ones"]


def test_adler32_matches_zlib(built):
    rng = np.random.default_rng(5)
    for n in (0, 1, 7, 5552, 5553, 100000):
        buf = rng.integers(0, 256, n, dtype=np.uint8)
        assert O.adler32(buf) == zlib.adler32(buf.tobytes())
    buf = np.full(1 << 20, 0xFF, np.uint8)  # worst case for the modulo reductions
    assert O.adler32(buf) == zlib.adler32(buf.tobytes())


def test_restatement_vs_real_reference(built):
    if not O.ref_available():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    rng = np.random.default_rng(11)
    for meth, k, m, w, size, P in [(O.REED_SOL_VAN, 12, 4, 8, 8192, 0), (O.CAUCHY_ORIG, 16, 4, 8, 8192, 32),
                                   (O.CAUCHY_GOOD, 5, 2, 8, 4096, 64), (O.REED_SOL_R6_OP, 9, 2, 8, 4096, 0),
                                   (O.REED_SOL_VAN, 7, 5, 16, 4096, 0), (O.REED_SOL_VAN, 7, 5, 32, 4096, 0),
                                   (O.CAUCHY_GOOD, 5, 2, 16, 4096, 32), (O.CAUCHY_GOOD, 9, 3, 32, 4096, 16),
                                   (O.REED_SOL_R6_OP, 9, 2, 32, 4096, 0)]:
        data = rng.integers(0, 256, (k, size), dtype=np.uint8)
        rp = O.RefPlan(meth, k, m, w, P)
        assert np.array_equal(rp.encode(data), O.encode(meth, data, m, P, w)), (meth, k, m, w)
        assert np.array_equal(rp.matrix(), O.coding_matrix(meth, k, m, w))
        rp.close()


def test_golden_schedules_are_self_consistent(golden):
    # a schedule fixture hashes to its recorded digest
    for e in golden["plans"]:
        if "schedule" in e:
            s = np.array(e["schedule"], dtype="<i4")
            assert hashlib.sha256(s.tobytes()).hexdigest() == e["schedule_sha256"]
            assert len(s) == e["schedule_ops"]
