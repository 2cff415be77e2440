"""CPU test of how the pinned-DMA path groups its copies (issue_runs, ec_pinning.cpp): runs that
repeat at one stripe stride on both sides become strided copies (hipMemcpy2DAsync), one per run
position within the stripe; everything else goes run by run.  The hook plans the grouping without
the runtime (the registered-range check that may still split a lattice needs a GPU and is covered
by tests/test_gpu_parity.py::test_strided_dma_lattices).  Every plan must cover the runs exactly,
in order, with pitches no smaller than the rows."""
import ctypes

import numpy as np
import pytest

from lstore_amd import erasure as E

MiB = 1 << 20


def plan(runs):
    lib = E.lib()
    f = lib.lsec_test_lattices
    u64p = ctypes.POINTER(ctypes.c_uint64)
    f.argtypes = [u64p, u64p, u64p, ctypes.c_int, ctypes.POINTER(ctypes.c_int64), ctypes.c_int]
    f.restype = ctypes.c_int
    n = len(runs)
    d = (ctypes.c_uint64 * max(n, 1))(*[r[0] for r in runs])
    s = (ctypes.c_uint64 * max(n, 1))(*[r[1] for r in runs])
    b = (ctypes.c_uint64 * max(n, 1))(*[r[2] for r in runs])
    out = (ctypes.c_int64 * (5 * max(n, 1)))()
    g = f(d, s, b, n, out, max(n, 1))
    assert g >= 0
    return [tuple(out[5 * i:5 * i + 5]) for i in range(g)]


def check_cover(runs, groups):
    """the groups reproduce the runs exactly and in order"""
    i = 0
    for first, period, rows, sp, dp in groups:
        assert first == i
        if rows >= 2:
            for l in range(period):
                assert sp >= runs[first + l][2] and dp >= runs[first + l][2]
            for r in range(rows):
                for l in range(period):
                    d0, s0, b0 = runs[first + l]
                    assert runs[first + r * period + l] == (d0 + r * dp, s0 + r * sp, b0)
        else:
            assert period == 1 and rows == 1
        i += period * rows
    assert i == len(runs)


def stripes(n, k, m, C, ids, host=1 << 40, dev=1 << 44):
    """DMA runs an encode / decode issues for n stripes laid out [stripe][k+m][C] on the host,
    packed [stripe][ids][C] on the device, adjacent chunks merged as add_run does"""
    runs = []
    for s in range(n):
        for j, i in enumerate(ids):
            dst, src = dev + (s * len(ids) + j) * C, host + (s * (k + m) + i) * C
            if runs and runs[-1][0] + runs[-1][2] == dst and runs[-1][1] + runs[-1][2] == src:
                runs[-1] = (runs[-1][0], runs[-1][1], runs[-1][2] + C)
            else:
                runs.append((dst, src, C))
    return runs


def test_encode_inputs_are_one_lattice(built):
    runs = stripes(64, 8, 3, 512 << 10, range(8))
    g = plan(runs)
    check_cover(runs, g)
    assert g == [(0, 1, 64, 11 * (512 << 10), 8 * (512 << 10))]


@pytest.mark.parametrize("erased", [[2, 5], [0, 3, 6], [1], [0, 7]])
def test_decode_survivors_split_by_erasures(built, erased):
    k, m, C, n = 8, 4, MiB, 20
    ids = [i for i in range(k + m) if i not in erased][:k]
    runs = stripes(n, k, m, C, ids)
    g = plan(runs)
    check_cover(runs, g)
    lanes = len(runs) // n
    assert len(g) == 1 and g[0][1] == lanes and g[0][2] == n, g


def test_column_blocks_of_one_stripe(built):
    # one stripe, block [c0, c0+cb) of each of 6 survivors: rows at the chunk stride
    C, cb = MiB, 512 << 10
    runs = [((1 << 44) + j * cb, (1 << 40) + (1 + j) * C, cb) for j in range(6)]
    g = plan(runs)
    check_cover(runs, g)
    assert g == [(0, 1, 6, C, cb)]


def test_irregular_and_mixed_runs(built):
    rng = np.random.default_rng(5)
    # stripes from two allocations, shuffled: no common stride
    a, b = 1 << 40, 3 << 40
    order = [3, 0, 5, 1, 4, 2]
    runs = [((1 << 44) + i * 4 * MiB, (a if s < 3 else b) + (s % 3) * 6 * MiB, 4 * MiB) for i, s in enumerate(order)]
    check_cover(runs, plan(runs))
    # a regular stretch, then a new stride, then descending addresses
    runs = stripes(10, 4, 2, MiB, range(4))
    runs += [((1 << 45) + i * 8 * MiB, (2 << 40) + i * 9 * MiB, 4 * MiB) for i in range(5)]
    runs += [((1 << 46) + i * MiB, (5 << 40) - i * 2 * MiB, MiB) for i in range(4)]
    g = plan(runs)
    check_cover(runs, g)
    assert g[0][:3] == (0, 1, 10) and g[1][:3] == (10, 1, 5)
    assert all(x[2] == 1 for x in g[2:])  # descending: run by run
    # rows wider than the pitch (overlapping host rows): never a lattice
    runs = [((1 << 44) + i * 4 * MiB, (1 << 40) + i * MiB, 4 * MiB) for i in range(6)]
    g = plan(runs)
    check_cover(runs, g)
    assert all(x[2] == 1 for x in g)
    # random run lists always covered exactly
    for _ in range(200):
        n = int(rng.integers(0, 40))
        base = int(rng.integers(1, 1 << 20)) << 20
        stride = int(rng.integers(1, 8)) * MiB
        runs = []
        for i in range(n):
            if rng.random() < 0.7:
                runs.append(((1 << 44) + i * stride, base + i * (stride + MiB), int(rng.integers(1, 4)) * (256 << 10)))
            else:
                runs.append((int(rng.integers(1, 1 << 30)) << 12, int(rng.integers(1, 1 << 30)) << 12, 4096))
        check_cover(runs, plan(runs))


def test_empty(built):
    assert plan([]) == []


def test_wide_rows_go_one_by_one(built):
    # rows of 16 MiB and more: one copy each (kMaxLatticeRow)
    runs = stripes(8, 10, 4, 4 * MiB, range(10))  # 40 MiB rows
    g = plan(runs)
    check_cover(runs, g)
    assert all(x[2] == 1 for x in g)
    runs = stripes(8, 4, 2, 4 * MiB - 4096, range(4))  # just under 16 MiB
    g = plan(runs)
    check_cover(runs, g)
    assert g[0][:3] == (0, 1, 8)
