#!/usr/bin/env python3
"""Kernel A/B bench (development tool): interleaved rounds of encode/decode per kernel variant.

python tools/kbench.py [--stripes N] [--rounds R] [--configs rs63,cg104,cg63,cg:K:M:C_KiB,...]
Prints HBM GB/s (algorithmic bytes / launch time, HIP events on the launch stream).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import lstore_amd as L  # noqa: E402
from lstore_amd import erasure as E  # noqa: E402

CONFIGS = {
    "rs63": (L.REED_SOL_VAN, 6, 3, 1 << 20),
    "rs104": (L.REED_SOL_VAN, 10, 4, 1 << 20),
    "cg63": (L.CAUCHY_GOOD, 6, 3, 1 << 20),
    "cg104": (L.CAUCHY_GOOD, 10, 4, 4 << 20),
    "rs206": (L.REED_SOL_VAN, 20, 6, 256 << 10),
    "rs128": (L.REED_SOL_VAN, 12, 8, 512 << 10),
    "rs166": (L.REED_SOL_VAN, 16, 6, 512 << 10),
    "rs248": (L.REED_SOL_VAN, 24, 8, 256 << 10),
    "rs104c4": (L.REED_SOL_VAN, 10, 4, 4 << 20),
    "rs104c8": (L.REED_SOL_VAN, 10, 4, 8 << 20),
    "cg104s": (L.CAUCHY_GOOD, 10, 4, 256 << 10),
    "cg104m": (L.CAUCHY_GOOD, 10, 4, 512 << 10),
    "cg104l": (L.CAUCHY_GOOD, 10, 4, 2 << 20),
    "cg164c8": (L.CAUCHY_GOOD, 16, 4, 8 << 20),
    "cg164c1": (L.CAUCHY_GOOD, 16, 4, 1 << 20),
    "rs84c4": (L.REED_SOL_VAN, 8, 4, 4 << 20),
    "cg206c4": (L.CAUCHY_GOOD, 20, 6, 4 << 20),
    "cg42c4": (L.CAUCHY_GOOD, 4, 2, 4 << 20),
    "rs83c8": (L.REED_SOL_VAN, 8, 3, 8 << 20),
    "rs164c8": (L.REED_SOL_VAN, 16, 4, 8 << 20),
    "rs63c8": (L.REED_SOL_VAN, 6, 3, 8 << 20),
    "cg206c1": (L.CAUCHY_GOOD, 20, 6, 1 << 20),
    "cg206c8": (L.CAUCHY_GOOD, 20, 6, 8 << 20),
    "cg124c4": (L.CAUCHY_GOOD, 12, 4, 4 << 20),
    "cg124c8": (L.CAUCHY_GOOD, 12, 4, 8 << 20),
    "rs164": (L.REED_SOL_VAN, 16, 4, 1 << 20),
    "rs124": (L.REED_SOL_VAN, 12, 4, 1 << 20),
    "rs84": (L.REED_SOL_VAN, 8, 4, 1 << 20),
    "cg206": (L.CAUCHY_GOOD, 20, 6, 256 << 10),
    # the c5 points under 0.70 in round 4 (r04_v15_sweep_c5.jsonl)
    "rs84c8": (L.REED_SOL_VAN, 8, 4, 8 << 20),
    "rs124c4": (L.REED_SOL_VAN, 12, 4, 4 << 20),
    "cg206c2": (L.CAUCHY_GOOD, 20, 6, 2 << 20),
    # wide fields (w = 16 / 32): transposed bit-sliced RS, bit-sliced Cauchy
    "rs63w16": (L.REED_SOL_VAN, 6, 3, 1 << 20, 16),
    "rs63w32": (L.REED_SOL_VAN, 6, 3, 1 << 20, 32),
    "rs104w16": (L.REED_SOL_VAN, 10, 4, 1 << 20, 16),
    "rs104w32": (L.REED_SOL_VAN, 10, 4, 1 << 20, 32),
    "rs106w32": (L.REED_SOL_VAN, 10, 6, 1 << 20, 32),
    "rs105w32": (L.REED_SOL_VAN, 10, 5, 1 << 20, 32),
    "rs206w16": (L.REED_SOL_VAN, 20, 6, 256 << 10, 16),
    "rs208w16": (L.REED_SOL_VAN, 20, 8, 256 << 10, 16),
    "rs165w16": (L.REED_SOL_VAN, 16, 5, 1 << 20, 16),
    "cg63w16": (L.CAUCHY_GOOD, 6, 3, 1 << 20, 16),
    "cg104w16": (L.CAUCHY_GOOD, 10, 4, 1 << 20, 16),
    "cg104w32": (L.CAUCHY_GOOD, 10, 4, 1 << 20, 32),
    # bitmatrix codes (K3): liberation w = 7, Blaum-Roth w = 6, liber8tion w = 8, raid4, r6
    "lib62": (L.LIBERATION, 6, 2, 7 << 17, 7),
    "br62": (L.BLAUM_ROTH, 6, 2, 6 << 17, 6),
    "l8t62": (L.LIBER8TION, 6, 2, 1 << 20, 8),
    "raid4_6": (L.RAID4, 6, 1, 1 << 20),
    "r6_62": (L.REED_SOL_R6_OP, 6, 2, 1 << 20),
    "cg63w32": (L.CAUCHY_GOOD, 6, 3, 1 << 20, 32),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--data-gib", type=float, default=24.0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--configs", default="rs63,cg104,cg63")
    ap.add_argument("--variants", default="0,0;1,0;0,2;0,4")
    ap.add_argument("--magic", action="store_true", help="also time fused encode+magic and standalone magic")
    ap.add_argument("--pad", type=int, default=0, help="bytes of padding after every shard (HBM channel spread)")
    ap.add_argument("--no-wait", action="store_true", help="do not wait for a network (A/B runs with it off)")
    ap.add_argument("--lost", default="0", help="erasures of the timed decode, e.g. 0,1,k+1 as ids (default: D0)")
    ap.add_argument("--mix", action="store_true",
                    help="also time lsec_hbm_mix_dev over the same shards: the encode's traffic, XOR only")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    variants = [tuple(int(x) for x in v.split(",")) for v in a.variants.split(";")]
    for name in a.configs.split(","):
        if name not in CONFIGS:  # "rs:K:M:C_KiB" / "cg:K:M:C_KiB"
            t, kk, mm, ck = name.split(":")
            CONFIGS[name] = ({"rs": L.REED_SOL_VAN, "cg": L.CAUCHY_GOOD}[t], int(kk), int(mm), int(ck) << 10)
        meth, k, m, C = CONFIGS[name][:4]
        w = CONFIGS[name][4] if len(CONFIGS[name]) > 4 else -1
        N = max(8, int(a.data_gib * 2**30 / (k * C)))
        plan = L.Plan.for_chunk(meth, k, m, C, w)
        data = torch.randint(0, 256, (N, k, C + a.pad), dtype=torch.uint8, device=dev)[:, :, :C]
        par = torch.empty((N, m, C + a.pad), dtype=torch.uint8, device=dev)[:, :, :C]
        lost = sorted({int(x) for x in a.lost.split(",")})
        out = torch.empty((N, len(lost), C), dtype=torch.uint8, device=dev)
        plan.prepare_encode()  # wide codes: wait for the compiled XOR network (variant 0,0 uses it)
        plan.prepare_decode(lost)
        import time
        # heavy networks can take longer than prepare's 30 s wait; only codes that get one
        # (ec_jit.cpp wants_xornet / wants_gfw_net / wants_pktnet)
        has_net = (w in (16, 32) and meth == L.REED_SOL_VAN) or (meth in (L.CAUCHY_GOOD, L.CAUCHY_ORIG) and k <= 32) or \
            (meth == L.REED_SOL_VAN and m * k >= 96) or meth in (L.LIBERATION, L.BLAUM_ROTH, L.LIBER8TION)
        t_end = time.time() + (90 if has_net and not a.no_wait else 0)
        while time.time() < t_end and not plan.jit():
            time.sleep(5)
            print(f"{name}: waiting for the encode network", flush=True)
        print(f"{name}: encode network {'ready' if plan.jit() else 'NOT ready'}", flush=True)
        plan.encode_dev(data, par)
        ref_par = par.clone()
        stream = torch.cuda.current_stream()
        res = {v: ([], []) for v in variants}
        tmix = []
        if a.mix:
            lib = E.lib()
            mrefs = L.Plan.shard_refs(plan.tensor_refs(data, par)[0])

            def mix():
                assert lib.lsec_hbm_mix_dev(mrefs, k, m, N, C, stream.cuda_stream) == 0
        for _ in range(a.rounds):
            if a.mix:
                mix()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.reps):
                    mix()
                e1.record(stream)
                torch.cuda.synchronize()
                tmix.append(e0.elapsed_time(e1) / a.reps)
                plan.encode_dev(data, par)  # restore the parity the variants are checked against
            for v in variants:
                E.set_kernel_variant(v[0], v[1])
                if len(v) > 2:  # a third field: the XCD tile phase (lsec_test_set_tile_phase)
                    E.lib().lsec_test_set_tile_phase(v[2])
                e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                plan.encode_dev(data, par)
                e0.record(stream)
                for _ in range(a.reps):
                    plan.encode_dev(data, par)
                e1.record(stream)
                for _ in range(a.reps):
                    plan.decode_dev(data, par, lost, out=out)
                e2.record(stream)
                torch.cuda.synchronize()
                res[v][0].append(e0.elapsed_time(e1) / a.reps)
                res[v][1].append(e1.elapsed_time(e2) / a.reps)
                assert torch.equal(par, ref_par), f"variant {v} changed parity"
                for i, e in enumerate(lost):
                    want = data[:, e] if e < k else ref_par[:, e - k]
                    assert torch.equal(out[:, i], want), f"variant {v} decode mismatch (shard {e})"
        E.set_kernel_variant(0, 0)
        net = int(plan.jit())
        for v in variants:
            te = sorted(res[v][0])[len(res[v][0]) // 2]
            td = sorted(res[v][1])[len(res[v][1]) // 2]
            eb = (k + m) * C * N
            db = (k + len(lost)) * C * N
            print(f"{name:6s} N={N:5d} variant={v} jit={net if v[:2] == (0, 0) else 0}  encode {te:8.3f} ms {eb / te / 1e6:7.1f} GB/s "
                  f"({eb / te / 8e9:5.1%})   decode {td:8.3f} ms {db / td / 1e6:7.1f} GB/s ({db / td / 8e9:5.1%})",
                  flush=True)
        if tmix:
            tm = sorted(tmix)[len(tmix) // 2]
            eb = (k + m) * C * N
            print(f"{name:6s} N={N:5d} mix probe (XOR of k to m, no GF)  {tm:8.3f} ms {eb / tm / 1e6:7.1f} GB/s ({eb / tm / 8e9:5.1%})",
                  flush=True)
        E.set_kernel_variant(0, 0)
        E.lib().lsec_test_set_tile_phase(1)  # the default
        if a.magic:
            mg = torch.zeros((N, 4), dtype=torch.uint8, device=dev)
            tm = []
            for fn in (lambda: plan.encode_magic_dev(data, par, mg), lambda: plan.stripe_magic_dev(data, par, mg)):
                fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.reps):
                    fn()
                e1.record(stream)
                torch.cuda.synchronize()
                tm.append(e0.elapsed_time(e1) / a.reps)
            eb = (k + m) * C * N
            print(f"{name:6s} encode+magic fused {tm[0]:8.3f} ms {eb / tm[0] / 1e6:7.1f} GB/s ({eb / tm[0] / 8e9:5.1%})   "
                  f"magic alone {tm[1]:8.3f} ms {eb / tm[1] / 1e6:7.1f} GB/s ({eb / tm[1] / 8e9:5.1%})", flush=True)
            del mg
        del data, par, out, ref_par
        plan.close()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
