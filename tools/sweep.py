#!/usr/bin/env python3
"""BASELINE config c5: mixed k+m sweep x chunk size x method, device-resident AND host-path.

For every (k, m) in {(4,2),(6,3),(8,3),(8,4),(10,4),(12,4),(16,4),(20,6)} x C in
{256 KiB .. 8 MiB} x {reed_sol_van, cauchy_good}: encode + single-erasure decode rates
  * device-resident (lsec_*_dev, HIP events), HBM GB/s and roofline fraction
  * host path (et_encode_stripes / et_decode_stripes from host memory: pack -> H2D -> kernel
    -> D2H -> unpack), i.e. with the PCIe copies included
and a bit-exact spot check against the CPU oracle.  One JSON line per case.
Under torchrun each rank sweeps its own GPU (static partition; no collectives but timing).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KM = [(4, 2), (6, 3), (8, 3), (8, 4), (10, 4), (12, 4), (16, 4), (20, 6)]
CHUNKS = [256 << 10, 512 << 10, 1 << 20, 2 << 20, 4 << 20, 8 << 20]


def link_rates(torch, dev, nbytes=1 << 30, reps=5):
    """This box's PCIe rate each way: one page-locked (hipHostMalloc) buffer <-> HBM, best of reps
    (the ceiling every host-path point is measured against)"""
    h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    best = {}
    for name, dst, src in (("h2d", d, h), ("d2h", h, d)):
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        t = []
        for _ in range(reps):
            t0 = time.perf_counter()
            dst.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
            t.append(time.perf_counter() - t0)
        best[name + "_GBps"] = round(nbytes / min(t) / 1e9, 2)
    # (both directions at once: tools/probes/duplex_probe.cpp -- torch copies on two streams
    # serialise and read as half the rate each, which the link does not)
    del h, d
    torch.cuda.empty_cache()
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--methods", default="reed_sol_van,cauchy_good")
    ap.add_argument("--km", default="")
    ap.add_argument("--chunks", default="")
    ap.add_argument("--dev-gib", type=float, default=8.0, help="user data per device-resident batch")
    ap.add_argument("--host-gib", type=float, default=1.0, help="user data per host-path batch")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default="")
    a = ap.parse_args()

    import torch

    import lstore_amd as L
    import oracle as O
    from lstore_amd import erasure as E

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local % torch.cuda.device_count())
    dev = torch.device("cuda", torch.cuda.current_device())
    km = [tuple(int(x) for x in p.split("+")) for p in a.km.split(",")] if a.km else KM
    chunks = [int(x) for x in a.chunks.split(",")] if a.chunks else CHUNKS
    out = open(a.out, "a") if a.out else None
    stream = torch.cuda.current_stream()
    link = link_rates(torch, dev)
    print(json.dumps({"config": "c5", "rank": rank, "link": link}), flush=True)
    if out:
        out.write(json.dumps({"config": "c5", "rank": rank, "link": link}) + "\n")
    for mname in a.methods.split(","):
        meth = E.JE_METHOD_NAMES.index(mname)
        for k, m in km:
            for C in chunks:
                plan = L.Plan.for_chunk(meth, k, m, C)
                plan.prepare_encode()
                plan.prepare_decode([0])
                N = max(2, int(a.dev_gib * 2**30 / (k * C)))
                data = torch.randint(0, 256, (N, k, C), dtype=torch.uint8, device=dev)
                par = torch.empty((N, m, C), dtype=torch.uint8, device=dev)
                rb = torch.empty((N, 1, C), dtype=torch.uint8, device=dev)
                plan.encode_dev(data, par)
                plan.decode_dev(data, par, [0], out=rb)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                ev[0].record(stream)
                for _ in range(a.reps):
                    plan.encode_dev(data, par)
                ev[1].record(stream)
                for _ in range(a.reps):
                    plan.decode_dev(data, par, [0], out=rb)
                ev[2].record(stream)
                torch.cuda.synchronize()
                te = ev[0].elapsed_time(ev[1]) / 1e3 / a.reps
                td = ev[1].elapsed_time(ev[2]) / 1e3 / a.reps
                # bit-exact spot check (last stripe) vs the oracle
                hd = data[N - 1].cpu().numpy()
                ok = bool(np.array_equal(O.encode(meth, hd, m, plan.packet_size), par[N - 1].cpu().numpy()))
                ok &= bool(torch.equal(rb[:, 0], data[:, 0]))
                del data, par, rb
                torch.cuda.empty_cache()
                # host path with copies included.  The device phase just handed ~12 GiB back to the
                # driver; for ~0.2 s after such a free, host<->device DMA runs at 60-70 % of its rate
                # (profiles/r05_v9_host_pattern.jsonl: a 2 s pause, or keeping the memory in torch's
                # cache, removes it), so pause, and warm the host batch with one untimed pair.
                torch.cuda.synchronize()
                time.sleep(1.0)
                Nh = max(2, int(a.host_gib * 2**30 / (k * C)))
                buf = np.empty((Nh, k + m, C), dtype=np.uint8)
                tile = np.random.default_rng(k * 31 + m).integers(0, 256, (1, k + m, C), dtype=np.uint8)
                buf[:] = tile
                plan.encode_stripes(buf)
                plan.decode_stripes(buf, [0])
                tes, tds = [], []
                for _ in range(a.reps):  # median of reps
                    t0 = time.perf_counter()
                    plan.encode_stripes(buf)
                    tes.append(time.perf_counter() - t0)
                    t0 = time.perf_counter()
                    plan.decode_stripes(buf, [0])
                    tds.append(time.perf_counter() - t0)
                the, thd = sorted(tes)[len(tes) // 2], sorted(tds)[len(tds) // 2]
                ok &= bool(np.array_equal(buf[0, k:], O.encode(meth, buf[0, :k], m, plan.packet_size)))
                gib_d, gib_h = k * C * N / 2**30, k * C * Nh / 2**30
                rec = {"config": "c5", "rank": rank, "method": mname, "k": k, "m": m, "chunk": C,
                       "packet": plan.packet_size, "kernel": "bytewise" if plan.kernel == 1 else "bitsliced",
                       "jit_encode": plan.jit(), "jit_decode": plan.jit([0]),
                       "dev_stripes": N, "enc_gibps": round(gib_d / te, 1), "dec_gibps": round(gib_d / td, 1),
                       "enc_hbm_frac": round((k + m) * C * N / te / 8e12, 4),
                       "dec_hbm_frac": round((k + 1) * C * N / td / 8e12, 4),
                       "host_stripes": Nh, "host_enc_gibps": round(gib_h / the, 2),
                       "host_dec_gibps": round(gib_h / thd, 2),
                       # the PCIe link's share each direction carries (encode: k*C in, m*C out per
                       # stripe; decode: k*C survivors in, C out), against this box's measured rates
                       "enc_h2d_link_frac": round(k * C * Nh / the / 1e9 / link["h2d_GBps"], 3),
                       "enc_d2h_link_frac": round(m * C * Nh / the / 1e9 / link["d2h_GBps"], 3),
                       "dec_h2d_link_frac": round(k * C * Nh / thd / 1e9 / link["h2d_GBps"], 3),
                       "dec_d2h_link_frac": round(C * Nh / thd / 1e9 / link["d2h_GBps"], 3),
                       "bit_exact": ok}
                line = json.dumps(rec)
                print(line, flush=True)
                if out:
                    out.write(line + "\n")
                    out.flush()
                plan.close()
                del buf


if __name__ == "__main__":
    main()
