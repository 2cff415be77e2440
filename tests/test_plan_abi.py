"""Host-side checks of liblstore_ec.so that need no GPU: exports, struct ABI, plan service.

The plan service (et_generate_plan / et_new_plan / form_* / nearest_prime / et_method_type)
is host logic; it must reproduce src/lio/erasure_tools.c + Jerasure's matrix builders
exactly, because the segment driver reads the plan struct's fields directly.
"""
import ctypes as C
import hashlib
import os
import re
import subprocess

import numpy as np
import pytest

import lstore_amd as L
import oracle as O
from lstore_amd import erasure as E

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "lstore_ec.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set(re.findall(r"^[A-Za-z_][\w \*]*?\b(\w+)\s*\(", text, flags=re.M))
    return {n for n in names if n not in ("if", "while", "for", "sizeof")}


def test_library_exports_every_header_symbol(built):
    lib = L.lib()
    declared = header_functions()
    assert declared == set(E.EXPORTS), declared ^ set(E.EXPORTS)
    for name in declared:
        assert hasattr(lib, name), name
    names = (C.c_char_p * 8).in_dll(lib, "JE_method")
    assert [names[i].decode() for i in range(8)] == list(L.JE_METHOD_NAMES)


def _offsets_program(include_dir, header):
    return f"""
#include <stddef.h>
#include <stdio.h>
#include "{header}"
int main(void) {{
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(struct lio_erasure_plan_t),
    offsetof(struct lio_erasure_plan_t, strip_size), offsetof(struct lio_erasure_plan_t, method),
    offsetof(struct lio_erasure_plan_t, data_strips), offsetof(struct lio_erasure_plan_t, parity_strips),
    offsetof(struct lio_erasure_plan_t, w), offsetof(struct lio_erasure_plan_t, packet_size),
    offsetof(struct lio_erasure_plan_t, base_unit), offsetof(struct lio_erasure_plan_t, encode_matrix),
    offsetof(struct lio_erasure_plan_t, encode_bitmatrix), offsetof(struct lio_erasure_plan_t, encode_schedule),
    offsetof(struct lio_erasure_plan_t, form_encoding_matrix), offsetof(struct lio_erasure_plan_t, form_decoding_matrix),
    offsetof(struct lio_erasure_plan_t, encode_block), offsetof(struct lio_erasure_plan_t, decode_block));
  return 0;
}}
"""


def _layout(tmp_path, incs, header, tag):
    src = tmp_path / f"off_{tag}.c"
    exe = tmp_path / f"off_{tag}"
    src.write_text(_offsets_program(incs[0], header))
    cmd = ["gcc", "-o", str(exe), str(src)] + [f"-I{i}" for i in incs]
    subprocess.run(cmd, check=True, capture_output=True)
    return subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()


def test_struct_layout_matches_ctypes_and_reference(tmp_path):
    ours = _layout(tmp_path, [os.path.join(ROOT, "include")], "lstore_ec.h", "ours")
    S = E.PlanStruct
    py = [C.sizeof(S)] + [getattr(S, f).offset for f, _ in S._fields_]
    assert [int(x) for x in ours] == py
    ref_dir = "/root/reference/src/lio"
    if os.path.isdir(ref_dir):  # build container only: compare with the reference header itself
        ref = _layout(tmp_path, [ref_dir, os.path.join(ref_dir, "lio")], "erasure_tools.h", "ref")
        assert ref == ours


def test_plans_match_reference_fixtures(built, golden):
    for e in golden["plans"]:
        with L.Plan.new(e["method"], 0, e["k"], e["m"], e["w"], 8, 8) as p:
            assert p.form_encoding_matrix() == 0, e["name"]
            assert p.form_decoding_matrix() == 0, e["name"]
            if e["matrix"] is not None:
                assert p.matrix().tolist() == e["matrix"], (e["name"], e["k"], e["m"])
            if e["bitmatrix_hex"] is not None:
                bm = p.bitmatrix()
                hexrows = ["%0*x" % (-(-bm.shape[1] // 4), int("".join(map(str, r)) + "0" * (-bm.shape[1] % 4), 2))
                           for r in bm]
                assert hexrows == e["bitmatrix_hex"], (e["name"], e["k"], e["m"])
            if e["schedule_sha256"] is not None:
                s = np.ascontiguousarray(p.schedule(), dtype="<i4")
                assert len(s) == e["schedule_ops"]
                assert hashlib.sha256(s.tobytes()).hexdigest() == e["schedule_sha256"], (e["name"], e["k"], e["m"])


def test_form_decoding_before_encoding_quirk(built):
    # cauchy_*_form_coding_matrix returns -1 when it forms the matrix while no schedule exists
    # (erasure_tools.c:142/:159), and 0 on every later call ("Already formed", :137/:152)
    for method in (L.CAUCHY_GOOD, L.CAUCHY_ORIG):
        with L.Plan.new(method, 0, 6, 3, 8, 8, 8) as p:
            assert p.form_decoding_matrix() == -1
            assert p.matrix() is not None and p.bitmatrix() is not None and p.schedule() is None
            assert p.form_decoding_matrix() == 0
            assert p.form_decoding_matrix() == 0
            assert p.form_encoding_matrix() == 0  # early return in the reference; we also fill the schedule
            assert p.form_decoding_matrix() == 0
    # liberation family: the same on the bitmatrix (:169-204)
    with L.Plan.new(L.LIBERATION, 0, 5, 2, 5, 8, 8) as p:
        assert p.form_decoding_matrix() == -1
        assert p.form_decoding_matrix() == 0
    with L.Plan.new(L.REED_SOL_VAN, 0, 6, 3, 8, 8, 8) as p:
        assert p.form_decoding_matrix() == 0
        assert p.form_decoding_matrix() == 0
        assert p.bitmatrix() is None and p.schedule() is None


def test_form_decoding_after_encoding(built):
    with L.Plan.new(L.CAUCHY_GOOD, 0, 6, 3, 8, 8, 8) as p:
        assert p.form_encoding_matrix() == 0 and p.schedule() is not None
        assert p.form_decoding_matrix() == 0


@pytest.mark.parametrize("method", [L.REED_SOL_VAN, L.CAUCHY_GOOD, L.CAUCHY_ORIG, L.REED_SOL_R6_OP, L.RAID4,
                                    L.LIBERATION, L.BLAUM_ROTH, L.LIBER8TION])
def test_generate_plan_matches_restatement(built, method):
    k, m = (6, 2) if method in (L.REED_SOL_R6_OP, L.LIBERATION, L.BLAUM_ROTH, L.LIBER8TION) else (6, 3)
    if method == L.RAID4:
        m = 1
    packet_code = method in (L.CAUCHY_GOOD, L.CAUCHY_ORIG, L.LIBERATION, L.BLAUM_ROTH, L.LIBER8TION)
    for fsize in [k * 16384, k * 65536, k * 262144, k * 1048576, k * 196608, k * 100000, 12345678, 1000, 6 * 4096]:
        ref = O.generate_plan(fsize, method, k, m)
        if packet_code and ref["strip_size"] * k != fsize and fsize % k == 0:
            # k chunks of C = fsize / k that no packet size divides: the reference builds this
            # plan and its schedule encode then overruns the chunks; the engine refuses it at
            # plan time (the segment maps NULL to -7).  Sizes that are not k equal chunks are
            # file-tool requests and keep the reference's padded plan.
            with pytest.raises(E.ErasureError, match="not a multiple of w\\*packet_size"):
                L.Plan.generate(fsize, method, k, m)
            continue
        with L.Plan.generate(fsize, method, k, m) as p:
            assert (p.w, p.packet_size, p.strip_size, p.base_unit) == (
                ref["w"], ref["packet_size"], ref["strip_size"], ref["base_unit"]), (method, fsize)


def test_generate_plan_increase_is_double_then_float(built):
    # `increase = (1.0*j) / file_size * 100` is computed in double and stored to a float
    # (erasure_tools.c:741, :893-894).  At this size the search stops at P = 4032 that way; the
    # same expression in float arithmetic gives 1.0 there and goes on to 4024.
    fsize = 18395501
    ref = O.generate_plan(fsize, L.REED_SOL_VAN, 6, 3)
    assert ref["packet_size"] == 4032
    with L.Plan.generate(fsize, L.REED_SOL_VAN, 6, 3) as p:
        assert (p.packet_size, p.strip_size) == (4032, ref["strip_size"])
    excess = ref["strip_size"] * 6 - fsize
    assert np.float32((1.0 * excess) / fsize * 100) < 1
    assert np.float32(excess) / np.float32(fsize) * np.float32(100) >= 1


def test_generate_plan_refuses_what_no_kernel_serves(built):
    with pytest.raises(E.ErasureError, match="not a multiple"):
        L.Plan.generate(6 * 100000, L.CAUCHY_GOOD, 6, 3)   # strip 100352, P = 784: C = 100000 cannot be encoded
    with L.Plan.generate(6 * 100000, L.REED_SOL_VAN, 6, 3) as p:  # matrix codes take any C % 8 == 0
        assert p.kernel == 1


def test_generate_plan_rejects_what_the_reference_rejects(built):
    with pytest.raises(E.ErasureError):
        L.Plan.generate(1 << 20, L.REED_SOL_R6_OP, 6, 3)          # r6 needs m == 2
    with pytest.raises(E.ErasureError):
        L.Plan.generate(1 << 20, L.RAID4, 6, 2)                   # raid4 needs m == 1
    with pytest.raises(E.ErasureError):
        L.Plan.generate(1 << 20, L.REED_SOL_VAN, 6, 3, w=7)       # w in {8,16,32}
    with pytest.raises(E.ErasureError):
        L.Plan.generate(1 << 20, L.CAUCHY_GOOD, 6, 3, -1, 2048, 1024)  # packet_low > packet_high
    with pytest.raises(E.ErasureError):
        L.Plan.generate(1 << 20, 9, 6, 3)                         # unknown method
    with pytest.raises(E.ErasureError):
        L.Plan.new(8, 0, 6, 3, 8, 8, 8)


def test_method_names_and_nearest_prime(built):
    for i, name in enumerate(L.JE_METHOD_NAMES):
        assert E.method_type(name) == i
        assert E.method_type(name.upper()) == i
    assert E.method_type("reed_sol") == -1
    primes = [2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53, 59, 61, 67, 71, 73, 79, 83, 89, 97, 101,
              103, 107, 109, 113, 127, 131, 137, 139, 149, 151, 157, 163, 167, 173, 179, 181, 191, 193, 197, 199,
              211, 223, 227, 229, 233, 239, 241, 251, 257]

    def ref_np(w, which):  # erasure_tools.c:50-77
        for i in range(1, 55):
            if w <= primes[i]:
                if which > 0:
                    return primes[i]
                if which < 0:
                    return primes[i - 1]
                return primes[i - 1] if w - primes[i - 1] < primes[i] - w else primes[i]
        return primes[54]

    for w in range(-2, 300):
        for which in (-1, 0, 1):
            assert E.nearest_prime(w, which) == ref_np(w, which), (w, which)


def test_no_gpu_means_loud_failure(built):
    """Without a GPU every compute entry point reports an error -- there is no CPU fallback."""
    if E.device_count() > 0:
        pytest.skip("a GPU is visible")
    with L.Plan.for_chunk(L.REED_SOL_VAN, 6, 3, 4096) as p:
        st = np.zeros((2, 9, 4096), np.uint8)
        with pytest.raises(E.ErasureError):
            p.encode_stripes(st)
        with pytest.raises(E.ErasureError):
            p.decode_stripes(st, [0])
        rc = p.decode_block([st[0, i] for i in range(9)], [0])
        assert rc == -1 and E.last_error()


def test_host_device_set_without_gpu(built):
    """lsec_set_host_devices: clearing the set always works; naming a device needs one."""
    E.set_host_devices(())
    if E.device_count() == 0:
        with pytest.raises(E.ErasureError):
            E.set_host_devices((0,))


def test_unsupported_method_is_an_error_not_a_fallback(built):
    with L.Plan.new(L.LIBERATION, 0, 6, 2, 263, 8, 8) as p:   # a prime w past the kernels' 257
        assert p.kernel == 0
        st = np.zeros((1, 8, 263 * 8 * 4), np.uint8)
        with pytest.raises(E.ErasureError, match="no GPU kernel"):
            p.encode_stripes(st)
    with L.Plan.new(L.LIBERATION, 0, 6, 2, 257, 8, 8) as p:   # w = 257: liberation k = 252..254
        assert p.kernel == 3
    for w in (37, 67):  # primes past the per-w kernels: the LDS-staged any-w bitmatrix kernel
        with L.Plan.new(L.LIBERATION, 0, 33, 2, w, 8, 8) as p:
            assert p.kernel == 3
    for w in (16, 32):
        with L.Plan.new(L.REED_SOL_VAN, 0, 6, 3, w, 8, 8) as p:
            assert p.kernel == 4   # wordwise GF(2^w)
        with L.Plan.new(L.CAUCHY_GOOD, 0, 6, 3, w, 8, 8) as p:
            assert p.kernel == 5   # bit-sliced GF(2^w)
    with L.Plan.generate(6 * 7 * 64 * 4, L.LIBERATION, 6, 2) as p:
        assert p.kernel == 3   # generic bitmatrix kernel


@pytest.mark.parametrize("w,k,m,ok", [(8, 250, 6, True), (8, 250, 7, False), (16, 1000, 24, True), (16, 1000, 25, False),
                                      (32, 1020, 4, True), (32, 1020, 5, False)])
def test_generate_plan_width_limits(built, w, k, m, ok):
    """k + m <= 256 at w = 8 (Jerasure's own limit there, reed_sol.c:247-248); <= 1024 for the
    GF(2^16) / GF(2^32) matrix codes (LSEC_MAX_DEVS_WIDE): wider plans are refused at plan time."""
    size = k * 4096
    if ok:
        with L.Plan.generate(size, L.REED_SOL_VAN, k, m, w) as p:
            assert (p.k, p.m, p.w) == (k, m, w)
    else:
        with pytest.raises(E.ErasureError, match="k\\+m outside"):
            L.Plan.generate(size, L.REED_SOL_VAN, k, m, w)
