#!/usr/bin/env python3
"""Headline benchmark: erasure encode+decode GiB/s (device-resident), RS(6+3), 1 MiB stripes.

BASELINE.json configs[1] (encode) + configs[2] (single-erasure decode), one MI355X per rank.
A step = encode N stripes (k data -> m parity) + decode the same N stripes with data shard 0
lost (k survivors -> 1 rebuilt shard), both through liblstore_ec.so's device-resident C ABI
(lsec_encode_dev / lsec_decode_dev) on the current torch stream.  Stripes are independent,
so ranks each own N stripes (static partition, weak scaling, no collective on the data
path; the only collectives are the timing barrier and the max-over-ranks reduction).

value = k*C*N*world / max_rank(step time) / 2^30  (data GiB/s, "N KiB stripes" = C per shard)

Device-resident layout: data [N][k][C], parity [N][m][C], every shard row followed by --pad
(default 1024) unused bytes, so the k+m streams of a stripe do not start on the same HBM
channel (shards exactly 1 MiB apart cost the encode ~8 %: profiles/r01_v15_pad_ab.txt).
layout.unpadded reports the same stripes with shards exactly C apart, launch-timed.

Also reported (same JSON line):
  roofline      encode kernel: algorithmic HBM bytes (k+m)*C*N per launch / avg launch time
                (HIP events on the launch stream) vs 8 TB/s
  cpu_baseline  the reference CPU path (oracle/_ref: vendor/jerasure via the plan dispatch)
                on a bounded sample of the same workload, on this box's host cores
  host_path     PCIe-inclusive rate of et_encode_stripes / et_decode_stripes from host memory
  hbm_copy_ref  this box's device-to-device copy rate (the practical HBM ceiling) and the
                encode / decode kernels' rates relative to it
Every run checks parity bit-exactly against the CPU oracle on sampled stripes.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK = 8.0e12  # B/s, MI355X HBM3E (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--stripes", type=int, default=4096, help="stripes per GPU (weak scaling)")
    ap.add_argument("--total-stripes", type=int, default=0,
                    help="if > 0: this many stripes split statically over the ranks (strong scaling)")
    ap.add_argument("--chunk", type=int, default=1 << 20, help="bytes per shard (C)")
    ap.add_argument("--k", type=int, default=6)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--method", default="reed_sol_van")
    ap.add_argument("--lost", type=int, default=0, help="shard lost in the decode half")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget for the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host-path", action="store_true")
    ap.add_argument("--variant", type=str, default="0,0", help="bytewise,bitsliced kernel variants")
    ap.add_argument("--pad", type=int, default=1024,
                    help="bytes left unused after every shard row in HBM (0 = shards exactly C apart)")
    ap.add_argument("--no-layout-ab", action="store_true", help="skip the unpadded-layout comparison")
    ap.add_argument("--no-copy-ref", action="store_true", help="skip the device-copy HBM reference")
    return ap.parse_args()


def cpu_baseline(method_id, k, m, C, P, lost, budget_s):
    """Reference CPU path (oracle/_ref) on a bounded sample: encode then decode, T threads."""
    import oracle as O

    if not O.ref_available():
        return None
    threads = max(1, min(16, os.cpu_count() or 1))
    # about budget_s of work at ~1 GiB/s/thread encode for RS; scale by threads, cap memory
    n = int(max(threads, min(512, budget_s * 0.5 * threads * (1 << 30) / (k * C) / 2)))
    tile = np.random.default_rng(1).integers(0, 256, size=(min(n, 8), k + m, C), dtype=np.uint8)
    buf = np.empty((n, k + m, C), dtype=np.uint8)
    for s0 in range(0, n, tile.shape[0]):
        buf[s0:s0 + tile.shape[0]] = tile[: n - s0]
    import ctypes as Ct

    base = buf.ctypes.data
    ptrs = (Ct.c_void_p * (n * (k + m)))(*[base + i * C for i in range(n * (k + m))])
    rp = O.RefPlan(method_id, k, m, 8, P)
    rp.encode_many(ptrs, min(n, threads), C, threads)  # warm tables / pages

    def passes(fn):
        # whole passes over the n-stripe buffer (far larger than the LLC) until half the budget
        t0, k_pass = time.perf_counter(), 0
        while True:
            rc = fn()
            k_pass += 1
            t = time.perf_counter() - t0
            if t >= budget_s / 2:
                return t / k_pass, k_pass, rc

    t_enc, p_enc, _ = passes(lambda: rp.encode_many(ptrs, n, C, threads))
    t_dec, p_dec, rc = passes(lambda: rp.decode_many(ptrs, n, C, threads, [lost]))
    rp.close()
    gib = k * C * n / 2**30
    return {"value": round(gib / (t_enc + t_dec), 3), "unit": "GiB/s", "cores": threads, "kind": "reference",
            "sample": f"{p_enc} encode passes then {p_dec} decode(lost {lost}) passes over {n} stripes x {k}+{m} x {C} B "
                      f"({round((t_enc * p_enc + t_dec * p_dec), 1)} s wall, {threads} pthreads), "
                      f"vendor/jerasure via oracle/_ref",
            "encode_gibps": round(gib / t_enc, 3), "decode_gibps": round(gib / t_dec, 3), "decode_rc": rc}


def pmc_traffic(k, m, C, N, kernel_kind):
    """HBM bytes per encode launch from the committed rocprofv3 PMC measurement
    (tools/pmc_traffic.py -> profiles/*_pmc_traffic.json), scaled to N stripes; None if no
    measurement exists for this geometry."""
    import glob

    prefix = "void lsec::k_gf8_bytewise<%d," % m if kernel_kind == 1 else "void lsec::k_gf8_bitsliced<%d," % m
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")), reverse=True):
        with open(f) as fh:
            d = json.load(fh)
        if (d.get("k"), d.get("m"), d.get("chunk")) != (k, m, C):
            continue
        for name, v in d["kernels"].items():
            if name.startswith(prefix):
                return int(v["traffic_per_stripe"] * N), os.path.relpath(f, ROOT)
    return None, None


def host_path_rate(L, plan, k, m, C, lost, nstripes, pinned=False, reps=3):
    """et_encode_stripes / et_decode_stripes from host memory (PCIe-inclusive), median of reps.

    pinned=False: pageable numpy buffers (LStore's cache pages) -> packed into the engine's
    pinned staging -> H2D -> kernel -> D2H -> unpacked.  pinned=True: page-locked buffers
    (torch pin_memory = hipHostMalloc), DMA'd in place with no host copies."""
    if pinned:
        import torch
        buf = torch.empty((nstripes, k + m, C), dtype=torch.uint8, pin_memory=True).numpy()
    else:
        buf = np.empty((nstripes, k + m, C), dtype=np.uint8)
    tile = np.random.default_rng(2).integers(0, 256, size=(min(nstripes, 8), k + m, C), dtype=np.uint8)
    for s0 in range(0, nstripes, tile.shape[0]):
        buf[s0:s0 + tile.shape[0]] = tile[: nstripes - s0]
    warm = min(nstripes, 16)  # a full staging batch: steady state, not first-call pinning
    plan.encode_stripes(buf[:warm])
    plan.decode_stripes(buf[:warm], [lost])
    te, td = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        plan.encode_stripes(buf)
        te.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        plan.decode_stripes(buf, [lost])
        td.append(time.perf_counter() - t0)
    te, td = sorted(te)[reps // 2], sorted(td)[reps // 2]
    gib = k * C * nstripes / 2**30
    return {"encode_gibps": round(gib / te, 2), "decode_gibps": round(gib / td, 2),
            "combined_gibps": round(gib / (te + td), 2), "stripes": nstripes,
            "note": ("page-locked host buffers -> DMA -> kernel -> DMA -> host" if pinned else
                     "pageable host buffers -> pinned staging -> H2D -> kernel -> D2H -> host")}


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    import lstore_amd as L
    from lstore_amd import erasure as E

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # one process per GPU; the only collectives are the timing barrier and the max-over-ranks
        # reduction (RCCL by default; LSEC_DIST_BACKEND=gloo lets ranks share one GPU for rehearsal)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local % torch.cuda.device_count())
        backend = os.environ.get("LSEC_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    bw_v, bs_v = (int(x) for x in a.variant.split(","))
    E.set_kernel_variant(bw_v, bs_v)

    method = E.JE_METHOD_NAMES.index(a.method)
    k, m, C, N = a.k, a.m, a.chunk, a.stripes
    if a.total_stripes > 0:
        from lstore_amd.partition import stripe_range
        s0, s1 = stripe_range(a.total_stripes, world, rank)
        N = max(1, s1 - s0)
    plan = L.Plan.for_chunk(method, k, m, C)
    P = plan.packet_size

    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    er = E._erasure_array([a.lost])
    plan.prepare_decode([a.lost])
    lib = E.lib()

    def workload(pad, seed):
        """Synthetic stripes resident in HBM: data [N][k][C], parity [N][m][C] and the rebuilt
        shard [N][1][C], every shard row followed by `pad` unused bytes (the device-resident
        layout).  Returns the tensors and the encode / decode launchers."""
        g = torch.Generator(device=dev).manual_seed(seed)
        data = torch.randint(0, 256, (N, k, C + pad), dtype=torch.uint8, device=dev, generator=g)[:, :, :C]
        par = torch.empty((N, m, C + pad), dtype=torch.uint8, device=dev)[:, :, :C]
        rebuilt = torch.empty((N, 1, C + pad), dtype=torch.uint8, device=dev)[:, :, :C]
        enc_refs, _, _ = plan.tensor_refs(data, par)
        enc_arr = plan.shard_refs(enc_refs)
        dec_refs = list(enc_refs)
        dec_refs[a.lost] = (rebuilt.data_ptr(), rebuilt.stride(0))
        dec_arr = plan.shard_refs(dec_refs)

        def encode():
            rc = lib.lsec_encode_dev(plan.ptr, enc_arr, N, C, sh)
            if rc:
                raise E.ErasureError(E.last_error())

        def decode():
            rc = lib.lsec_decode_dev(plan.ptr, dec_arr, N, C, er, sh)
            if rc:
                raise E.ErasureError(E.last_error())

        return data, par, rebuilt, encode, decode

    def launch_times(encode, decode, reps):
        """average encode / decode launch time (s), HIP events on the launch stream"""
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record(stream)
        for _ in range(reps):
            encode()
        ev[1].record(stream)
        for _ in range(reps):
            decode()
        ev[2].record(stream)
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / 1e3 / reps, ev[1].elapsed_time(ev[2]) / 1e3 / reps

    data, par, rebuilt, encode, decode = workload(a.pad, 1234 + rank)

    for _ in range(a.warmup):
        encode()
        decode()
    torch.cuda.synchronize()

    # ---- timed region: K steps, barrier + synchronize on both sides
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        encode()
        decode()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        from lstore_amd.partition import max_over_ranks
        elapsed = max_over_ranks(elapsed, dev if dist.get_backend() == "nccl" else None)

    # ---- per-kernel timing with HIP events on the launch stream (roofline)
    reps = max(3, min(10, a.steps))
    t_enc, t_dec = launch_times(encode, decode, reps)

    # ---- parity check (bit-exact vs the CPU oracle on sampled stripes)
    import oracle as O

    ok = True
    pick = sorted({0, N // 2, N - 1})
    hd = data[pick].cpu().numpy()
    hp = par[pick].cpu().numpy()
    hr = rebuilt[pick].cpu().numpy()
    for i in range(len(pick)):
        ref = O.encode(method, hd[i], m, P)
        ok &= bool(np.array_equal(ref, hp[i]))
        ok &= bool(np.array_equal(hr[i, 0], np.vstack([hd[i], hp[i]])[a.lost]))
    if not ok:
        print(json.dumps({"error": "parity mismatch vs oracle", "rank": rank}), flush=True)
        sys.exit(1)

    data_bytes = k * C * N
    enc_hbm = (k + m) * C * N
    dec_hbm = (k + 1) * C * N
    layout = {"shard_pad_bytes": a.pad}
    if a.pad and world == 1 and not a.no_layout_ab:
        # the same stripes in the unpadded layout (shards exactly C apart, as one cache page
        # holds them), launch-timed beside the padded one for the record
        del data, par, rebuilt
        torch.cuda.empty_cache()
        _, _, _, enc0, dec0 = workload(0, 1234 + rank)
        enc0()
        dec0()
        te0, td0 = launch_times(enc0, dec0, reps)
        layout["unpadded"] = {"encode_frac": round(enc_hbm / te0 / HBM_PEAK, 4),
                              "decode_frac": round(dec_hbm / td0 / HBM_PEAK, 4),
                              "value_from_launch_times": round(data_bytes / (te0 + td0) / 2**30, 2),
                              "padded_value_from_launch_times": round(data_bytes / (t_enc + t_dec) / 2**30, 2)}
        del enc0, dec0
        torch.cuda.empty_cache()
    copy_ref = None
    if world == 1 and not a.no_copy_ref:
        # the box's practical HBM ceiling beside the spec peak: streaming device copies of the
        # encode launch's byte count (half read, half written), HIP events on the launch stream --
        # the engine's probe kernel (lsec_hbm_copy_dev: the coding kernels' memory shape) and torch's copy_
        data = par = rebuilt = None
        torch.cuda.empty_cache()
        nb = enc_hbm // 2
        src = torch.empty(nb, dtype=torch.uint8, device=dev)
        dst = torch.empty_like(src)

        def probe():
            if lib.lsec_hbm_copy_dev(dst.data_ptr(), src.data_ptr(), nb, sh):
                raise E.ErasureError(E.last_error())

        def timed(fn):
            fn()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record(stream)
            for _ in range(reps):
                fn()
            ev[1].record(stream)
            torch.cuda.synchronize()
            return ev[0].elapsed_time(ev[1]) / 1e3 / reps

        t_probe, t_torch = timed(probe), timed(lambda: dst.copy_(src))
        copy_ref = {"what": "device->device copy of (k+m)*C*N/2 bytes, read+write counted",
                    "probe_GBps": round(2 * nb / t_probe / 1e9, 1), "probe_frac": round(2 * nb / t_probe / HBM_PEAK, 4),
                    "torch_copy_GBps": round(2 * nb / t_torch / 1e9, 1),
                    "encode_vs_probe": round((enc_hbm / t_enc) / (2 * nb / t_probe), 3),
                    "decode_vs_probe": round((dec_hbm / t_dec) / (2 * nb / t_probe), 3)}
        del src, dst
        torch.cuda.empty_cache()
    if a.total_stripes > 0:
        value = k * C * a.total_stripes * a.steps / elapsed / 2**30
    else:
        value = data_bytes * world * a.steps / elapsed / 2**30
    achieved = enc_hbm / t_enc
    traffic, traffic_src = pmc_traffic(k, m, C, N, plan.kernel)

    out = None
    if rank == 0:
        # the reference CPU path is timed at N=1 only (one process; at N>1 it would only delay the ranks' exit)
        cpu = None if (a.no_cpu or world > 1) else cpu_baseline(method, k, m, C, P, a.lost, a.cpu_seconds)
        host = None
        if not a.no_host_path and world == 1:
            ns = max(8, min(256, (4 << 30) // ((k + m) * C)))
            host = host_path_rate(L, plan, k, m, C, a.lost, ns)
            host["pinned"] = host_path_rate(L, plan, k, m, C, a.lost, ns, pinned=True)
        out = {
            "metric": "erasure encode+decode GiB/s (device-resident), RS(6+3) 1 MiB stripes"
            if (method, k, m, C) == (0, 6, 3, 1 << 20) else
            f"erasure encode+decode GiB/s (device-resident), {a.method}({k}+{m}) {C} B chunks",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong" if a.total_stripes > 0 else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (torch.randint bytes, resident in HBM)",
            "config": {"workload": f"{a.method}({k}+{m}) encode + decode(lost shard {a.lost}), C={C} B per shard, "
                                   f"{N} stripes/GPU, k*C={k * C} B user data per stripe",
                       "method": a.method, "k": k, "m": m, "chunk_bytes": C, "packet_size": P,
                       "stripes_per_gpu": N, "lost_shard": a.lost, "parallelism": f"static stripe partition x{world}"},
            "encode_gibps": round(data_bytes / t_enc / 2**30, 2),
            "decode_gibps": round(data_bytes / t_dec / 2**30, 2),
            "roofline": {"bound": "hbm", "achieved": round(achieved / 1e9, 1), "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": "gf8_bytewise (encode)" if plan.kernel == 1 else "gf8_bitsliced (encode)",
                         "algorithmic_bytes_per_launch": enc_hbm, "avg_launch_ms": round(t_enc * 1e3, 4),
                         "decode_achieved_GBps": round(dec_hbm / t_dec / 1e9, 1),
                         "decode_frac": round(dec_hbm / t_dec / HBM_PEAK, 4)},
            "layout": layout,
            "hbm_copy_ref": copy_ref,
            "cpu_baseline": cpu,
            "host_path": host,
            "parity_check": "bit-exact vs oracle on stripes %s" % pick,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    plan.close()


if __name__ == "__main__":
    main()
