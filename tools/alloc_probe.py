#!/usr/bin/env python3
"""Allocation vs layout probe (development tool).

Is the headline's padded / unpadded difference a property of the shard layout, or of the
physical HBM pages an allocation happens to get?  For each of several fresh allocations (the
caching allocator emptied in between, a spacer of varying size shifting where the next one
lands), time the RS(6+3) 1 MiB encode and single-erasure decode over the same stripes laid out
unpadded (shards C apart) and padded (C + 1024 apart) inside that one allocation.

python tools/alloc_probe.py [--trials 4] [--config rs63] [--json out.jsonl]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import ctypes  # noqa: E402

import torch  # noqa: E402

import lstore_amd as L  # noqa: E402


class RawDev:
    """A device buffer from hipMalloc / hipExtMallocWithFlags, seen by torch through
    __cuda_array_interface__ (no copy).  flags 4 = hipDeviceMallocContiguous."""
    hip = None

    def __init__(self, nbytes, flags=-1):
        if RawDev.hip is None:
            RawDev.hip = ctypes.CDLL("libamdhip64.so")
        p = ctypes.c_void_p()
        if flags < 0:
            rc = RawDev.hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes))
        else:
            rc = RawDev.hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(flags))
        if rc != 0:
            raise MemoryError(f"hip allocation of {nbytes} B with flags {flags}: error {rc}")
        self.ptr, self.n = p.value, nbytes
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (self.ptr, False),
                                         "version": 3, "strides": None}

    def tensor(self):
        return torch.as_tensor(self, device="cuda")

    def free(self):
        if self.ptr:
            torch.cuda.synchronize()
            RawDev.hip.hipFree(ctypes.c_void_p(self.ptr))
            self.ptr = 0

CONFIGS = {"rs63": (L.REED_SOL_VAN, 6, 3, 1 << 20), "cg63": (L.CAUCHY_GOOD, 6, 3, 1 << 20),
           "rs104_8m": (L.REED_SOL_VAN, 10, 4, 8 << 20)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="rs63")
    ap.add_argument("--trials", type=int, default=4)
    ap.add_argument("--pads", default="0,1024")
    ap.add_argument("--data-gib", type=float, default=24.0)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--json", default="")
    ap.add_argument("--alloc", default="torch",
                    help="torch | hipmalloc | contig (hipDeviceMallocContiguous); a comma list alternates per trial")
    a = ap.parse_args()
    meth, k, m, C = CONFIGS[a.config]
    pads = [int(x) for x in a.pads.split(",")]
    N = int(a.data_gib * 2**30 / (k * C))
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    plan = L.Plan.for_chunk(meth, k, m, C)
    plan.prepare_decode([0])
    out = []
    allocs = a.alloc.split(",")
    for trial in range(a.trials):
        alloc = allocs[trial % len(allocs)]
        torch.cuda.empty_cache()
        spacer = torch.empty(((trial * 37) % 11 + 1) << 28, dtype=torch.uint8, device=dev)  # 256 MiB .. 2.75 GiB
        P = max(pads)
        raws = []
        if alloc == "torch":
            dbuf = torch.randint(0, 256, (N * k * (C + P),), dtype=torch.uint8, device=dev)
            pbuf = torch.empty((N * m * (C + P),), dtype=torch.uint8, device=dev)
            rbuf = torch.empty((N * (C + P),), dtype=torch.uint8, device=dev)
        else:
            fl = 4 if alloc == "contig" else -1
            raws = [RawDev(N * n * (C + P), fl) for n in (k, m, 1)]
            dbuf, pbuf, rbuf = (r.tensor() for r in raws)
            g = torch.Generator(device=dev)
            g.manual_seed(trial)
            step = 1 << 30
            for o in range(0, dbuf.numel(), step):
                seg = dbuf[o:o + step]
                seg.copy_(torch.randint(0, 256, seg.shape, dtype=torch.uint8, device=dev, generator=g))
        del spacer
        views = {}
        for pad in pads:
            views[pad] = (dbuf[: N * k * (C + pad)].view(N, k, C + pad)[:, :, :C],
                          pbuf[: N * m * (C + pad)].view(N, m, C + pad)[:, :, :C],
                          rbuf[: N * (C + pad)].view(N, 1, C + pad)[:, :, :C])
        res = {p: ([], []) for p in pads}
        for _ in range(a.rounds):
            for pad in pads:
                d, p_, r = views[pad]
                plan.encode_dev(d, p_)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                ev[0].record(st)
                for _ in range(a.reps):
                    plan.encode_dev(d, p_)
                ev[1].record(st)
                for _ in range(a.reps):
                    plan.decode_dev(d, p_, [0], out=r)
                ev[2].record(st)
                torch.cuda.synchronize()
                res[pad][0].append(ev[0].elapsed_time(ev[1]) / a.reps)
                res[pad][1].append(ev[1].elapsed_time(ev[2]) / a.reps)
                assert torch.equal(r[:: max(1, N // 5), 0], d[:: max(1, N // 5), 0])
        for pad in pads:
            te, td = (sorted(x)[len(x) // 2] for x in res[pad])
            rec = {"config": a.config, "alloc": alloc, "trial": trial, "pad": pad, "data_va_mib": (dbuf.data_ptr() >> 20) & 0xFFFFF,
                   "encode_frac": round((k + m) * C * N / te / 8e9, 4), "decode_frac": round((k + 1) * C * N / td / 8e9, 4)}
            out.append(rec)
            print(json.dumps(rec), flush=True)
        del views, dbuf, pbuf, rbuf
        for r in raws:
            r.free()
    if a.json:
        with open(a.json, "w") as f:
            for r in out:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
