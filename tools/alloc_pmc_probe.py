#!/usr/bin/env python3
"""Allocation-placement probe with counters.

The headline RS(6+3) 1 MiB encode runs at 0.76 of 8 TB/s on some fresh allocations and at
0.80-0.83 on others (profiles/r03_v4_alloc_probe.jsonl).  This probe makes T fresh allocations of
the bench workload in ONE process (so one rocprofv3 --pmc pass sees both modes), and on each runs
exactly `reps` encodes then `reps` single-erasure decodes.  It prints one JSON line per trial with
the buffers' virtual addresses and the HIP-event launch times; tools/alloc_pmc_summary.py joins
the per-dispatch counters of each pass to the trials by dispatch order (the encode kernel is the
k_gf8_bytewise<3,...> instantiation, the decode k_gf8_bytewise<1,...>).

python tools/alloc_pmc_probe.py --trials 10 [--alloc torch|hipmalloc|vmm] [--json out.jsonl]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import lstore_amd as L  # noqa: E402
from alloc_probe import RawDev  # noqa: E402


class VmmDev:
    """A device buffer built with HIP's virtual memory API: physical chunks of `chunk` bytes
    (hipMemCreate), mapped back to back (or in a shuffled order) into one reserved VA range, so
    an allocation is made of many independently placed physical pieces instead of what one
    hipMalloc returns.  Seen by torch through __cuda_array_interface__ (no copy)."""
    hip = None

    class Prop(ctypes.Structure):
        _fields_ = [("type", ctypes.c_int), ("handle_type", ctypes.c_int), ("location", ctypes.c_int * 2),
                    ("win32", ctypes.c_void_p), ("compression", ctypes.c_ubyte), ("rdma", ctypes.c_ubyte),
                    ("usage", ctypes.c_ushort)]

    class Access(ctypes.Structure):
        _fields_ = [("location", ctypes.c_int * 2), ("flags", ctypes.c_int)]

    def __init__(self, nbytes, chunk, shuffle_seed=None):
        if VmmDev.hip is None:
            VmmDev.hip = ctypes.CDLL("libamdhip64.so")
        h = VmmDev.hip
        prop = VmmDev.Prop(1, 0, (ctypes.c_int * 2)(1, torch.cuda.current_device()), None, 0, 0, 0)
        gran = ctypes.c_size_t()
        assert h.hipMemGetAllocationGranularity(ctypes.byref(gran), ctypes.byref(prop), 1) == 0
        chunk = max(chunk, gran.value)
        n = -(-nbytes // chunk)
        self.size, self.chunk = n * chunk, chunk
        p = ctypes.c_void_p()
        assert h.hipMemAddressReserve(ctypes.byref(p), ctypes.c_size_t(self.size), ctypes.c_size_t(0), None,
                                      ctypes.c_ulonglong(0)) == 0
        self.ptr = p.value
        self.handles = []
        order = list(range(n))
        if shuffle_seed is not None:
            import random
            random.Random(shuffle_seed).shuffle(order)
        for i in range(n):
            hd = ctypes.c_ulonglong()
            rc = h.hipMemCreate(ctypes.byref(hd), ctypes.c_size_t(chunk), ctypes.byref(prop), ctypes.c_ulonglong(0))
            if rc != 0:
                raise MemoryError(f"hipMemCreate: error {rc}")
            self.handles.append(hd)
        for i, slot in enumerate(order):
            assert h.hipMemMap(ctypes.c_void_p(self.ptr + slot * chunk), ctypes.c_size_t(chunk), ctypes.c_size_t(0),
                               self.handles[i], ctypes.c_ulonglong(0)) == 0
        acc = VmmDev.Access((ctypes.c_int * 2)(1, torch.cuda.current_device()), 3)
        assert h.hipMemSetAccess(ctypes.c_void_p(self.ptr), ctypes.c_size_t(self.size), ctypes.byref(acc),
                                 ctypes.c_size_t(1)) == 0
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (self.ptr, False),
                                         "version": 3, "strides": None}

    def tensor(self):
        return torch.as_tensor(self, device="cuda")

    def free(self):
        if self.ptr:
            torch.cuda.synchronize()
            h = VmmDev.hip
            h.hipMemUnmap(ctypes.c_void_p(self.ptr), ctypes.c_size_t(self.size))
            for hd in self.handles:
                h.hipMemRelease(hd)
            h.hipMemAddressFree(ctypes.c_void_p(self.ptr), ctypes.c_size_t(self.size))
            self.ptr = 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=10)
    ap.add_argument("--stripes", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--alloc", default="torch",
                    help="torch | hipmalloc | contig | vmm:<chunk MiB>[:shuffle]; a comma list alternates per trial")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    k, m, C, N = 6, 3, 1 << 20, a.stripes
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    plan = L.Plan.for_chunk(L.REED_SOL_VAN, k, m, C)
    plan.prepare_decode([0])
    allocs = a.alloc.split(",")
    out = []
    for trial in range(a.trials):
        alloc = allocs[trial % len(allocs)]
        torch.cuda.empty_cache()
        spacer = torch.empty(((trial * 37) % 11 + 1) << 28, dtype=torch.uint8, device=dev)  # 256 MiB .. 2.75 GiB
        raws = []
        if alloc == "torch":
            dbuf = torch.randint(0, 256, (N * k * C,), dtype=torch.uint8, device=dev)
            pbuf = torch.empty((N * m * C,), dtype=torch.uint8, device=dev)
            rbuf = torch.empty((N * C,), dtype=torch.uint8, device=dev)
        elif alloc.startswith("vmm"):
            # vmm:<chunk MiB>[:shuffle]
            parts = alloc.split(":")
            chunk = int(parts[1]) << 20 if len(parts) > 1 else 2 << 20
            seed = trial if len(parts) > 2 and parts[2] == "shuffle" else None
            raws = [VmmDev(N * n * C, chunk, seed) for n in (k, m, 1)]
            dbuf, pbuf, rbuf = (r.tensor() for r in raws)
            g = torch.Generator(device=dev).manual_seed(trial)
            for o in range(0, dbuf.numel(), 1 << 30):
                seg = dbuf[o:o + (1 << 30)]
                seg.copy_(torch.randint(0, 256, seg.shape, dtype=torch.uint8, device=dev, generator=g))
        else:
            raws = [RawDev(N * n * C, 4 if alloc == "contig" else -1) for n in (k, m, 1)]
            dbuf, pbuf, rbuf = (r.tensor() for r in raws)
            g = torch.Generator(device=dev).manual_seed(trial)
            for o in range(0, dbuf.numel(), 1 << 30):
                seg = dbuf[o:o + (1 << 30)]
                seg.copy_(torch.randint(0, 256, seg.shape, dtype=torch.uint8, device=dev, generator=g))
        del spacer
        d = dbuf.view(N, k, C)
        p = pbuf.view(N, m, C)
        r = rbuf.view(N, 1, C)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.reps + 1)]
        ev[0].record(st)
        for i in range(a.reps):
            plan.encode_dev(d, p)
            ev[1 + i].record(st)
        for i in range(a.reps):
            plan.decode_dev(d, p, [0], out=r)
            ev[1 + a.reps + i].record(st)
        torch.cuda.synchronize()
        te = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(a.reps))
        td = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(a.reps, 2 * a.reps))
        ok = bool(torch.equal(r[:: max(1, N // 7), 0], d[:: max(1, N // 7), 0]))
        # the encode's first launch is cold (first touch of the parity pages): the median of the rest
        te_med, td_med = te[len(te) // 2], td[len(td) // 2]
        rec = {"trial": trial, "alloc": alloc,
               "va": {"data": hex(dbuf.data_ptr()), "parity": hex(pbuf.data_ptr()), "rebuilt": hex(rbuf.data_ptr())},
               "va_mod_2m": [x.data_ptr() % (2 << 20) for x in (dbuf, pbuf, rbuf)],
               "parity_minus_data_mib": (pbuf.data_ptr() - dbuf.data_ptr()) / 2**20,
               "encode_ms": round(te_med, 4), "decode_ms": round(td_med, 4),
               "encode_ms_all": [round(x, 4) for x in te], "decode_ms_all": [round(x, 4) for x in td],
               "encode_frac": round((k + m) * C * N / (te_med / 1e3) / 8e12, 4),
               "decode_frac": round((k + 1) * C * N / (td_med / 1e3) / 8e12, 4), "rebuild_ok": ok}
        out.append(rec)
        print(json.dumps(rec), flush=True)
        del d, p, r, dbuf, pbuf, rbuf
        for x in raws:
            x.free()
    if a.json:
        with open(a.json, "w") as f:
            for rec in out:
                f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
