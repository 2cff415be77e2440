"""world_size-2 gloo rehearsal of the multi-GPU path (CPU only).

bench.py shards stripes statically over ranks with no data-path collective; these tests run
the same partition + timing reductions on two CPU processes and check that the union of the
per-rank work equals the single-process result (oracle encode of every stripe).
"""
import os
import socket
import zlib

import numpy as np
import pytest
import torch.multiprocessing as mp

from lstore_amd.partition import stripe_range


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, nstripes, out_q):
    import torch.distributed as dist

    import oracle as O
    from lstore_amd.partition import max_over_ranks, stripe_range, sum_over_ranks
    from patterns import stripe

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s0, s1 = stripe_range(nstripes, world, rank)
    crcs = {}
    for s in range(s0, s1):
        par = O.encode(O.REED_SOL_VAN, stripe(6, 4096, s), 3)
        crcs[s] = zlib.crc32(par.tobytes())
    dist.barrier()
    slowest = max_over_ranks(float(rank + 1))
    total = sum_over_ranks(s1 - s0)
    out_q.put((rank, crcs, slowest, total))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("nstripes", [7, 16])
def test_two_rank_partition_matches_single_process(built, nstripes):
    import oracle as O
    from patterns import stripe

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, nstripes, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    merged = {}
    for rank, crcs, slowest, total in res:
        assert slowest == 2.0 and total == nstripes
        assert not set(crcs) & set(merged)
        merged.update(crcs)
    assert sorted(merged) == list(range(nstripes))
    for s in range(nstripes):
        assert merged[s] == zlib.crc32(O.encode(O.REED_SOL_VAN, stripe(6, 4096, s), 3).tobytes())


def test_stripe_range_properties():
    for n in (0, 1, 7, 2048, 4097):
        for world in (1, 2, 4, 8):
            spans = [stripe_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        stripe_range(10, 2, 2)
    assert np.sum([b - a for a, b in (stripe_range(10, 3, r) for r in range(3))]) == 10
