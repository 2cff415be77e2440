"""bench.py's host-side pieces that need no GPU: the kernel label on the roofline line and the
synthetic input of SURVEY.md §8d (splitmix64, seed 0x4C53544F5245, stripe s at word s*k*C/8),
generated with torch's int64 arithmetic and checked against tests/patterns.py's numpy statement."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import bench  # noqa: E402
import patterns  # noqa: E402


def test_kernel_label_names_the_kernel_that_ran():
    # the generic kernel of each kind when no network serves the plan
    assert bench.kernel_label(1, False) == "k_gf8_bytewise (encode)"
    assert bench.kernel_label(2, False) == "k_gf8_bitsliced (encode)"
    # a Cauchy plan whose packet network is compiled (c4: jit_encode true) is not the bit-sliced kernel
    lab = bench.kernel_label(2, True)
    assert lab.startswith("lsec_xornet") and "k_gf8_bitsliced" in lab
    assert bench.kernel_label(4, True).startswith("lsec_xornet")
    # the in-run PMC pass's kernel name wins: it is the kernel rocprofv3 saw run
    name = "lsec_xornet"
    assert bench.kernel_label(2, False, name).startswith(name)
    assert bench.kernel_label(1, True, "void lsec::k_gf8_bytewise<3, 6, 2, true, 4, false, false>(lsec::ApplyArgs)") \
        .startswith("void lsec::k_gf8_bytewise<3, 6")


@pytest.mark.parametrize("k,C,N,first,pad", [(6, 4096, 5, 0, 0), (6, 4096, 4, 3, 64), (10, 8192, 3, 7, 1024),
                                             (4, 256, 9, 1, 8)])
def test_bench_stripes_are_the_survey_splitmix_stream(k, C, N, first, pad):
    torch = pytest.importorskip("torch")
    buf = torch.zeros(N * k * (C + pad), dtype=torch.uint8)
    # a small pass size so that several passes (and a pass boundary inside a row group) are covered
    bench.splitmix_rows(torch, buf.view(N * k, C + pad)[:, :C], first * k * C // 8, words_per_pass=3 * C // 8 + 5)
    got = buf.view(N, k, C + pad)[:, :, :C].numpy()
    for s in range(N):
        assert np.array_equal(got[s], patterns.stripe(k, C, first + s)), (s, first)
    if pad:
        assert not buf.view(N * k, C + pad)[:, C:].any()  # the pad bytes are not written


def test_splitmix_first_words_known_answer():
    # splitmix64 from seed 0 gives the published first outputs 0xE220A8397B1DCDAF, 0x6E789E6AA1B965F4
    torch = pytest.importorskip("torch")
    buf = torch.zeros((1, 16), dtype=torch.uint8)
    bench.splitmix_rows(torch, buf, 0, seed=0)
    words = buf.numpy().view(np.uint64)[0]
    assert int(words[0]) == 0xE220A8397B1DCDAF and int(words[1]) == 0x6E789E6AA1B965F4
