#!/usr/bin/env python3
"""Headline benchmark: erasure encode+decode GiB/s (device-resident), RS(6+3), 1 MiB stripes.

BASELINE.json configs[1] (encode) + configs[2] (single-erasure decode), one MI355X per rank.
A step = encode N stripes (k data -> m parity) + decode the same N stripes with data shard 0
lost (k survivors -> 1 rebuilt shard), both through liblstore_ec.so's device-resident C ABI
(lsec_encode_dev / lsec_decode_dev) on the current torch stream.  Stripes are independent,
so ranks each own N stripes (static partition, weak scaling, no collective on the data
path; the only collectives are the timing barrier, the max-over-ranks reduction and the
gather of per-rank figures at the end).

value = k*C*N*world / max_rank(step time) / 2^30  (data GiB/s, "N KiB stripes" = C per shard)

Launching.  `bench.py --gpus N` with WORLD_SIZE unset starts N ranks itself (spawned before
anything touches the GPU); under torch.distributed.run (WORLD_SIZE set) it runs as one rank
and refuses a WORLD_SIZE that disagrees with --gpus.  The control plane (timing barrier, max,
gather) runs over gloo: the data path needs no collective, and gloo also lets ranks share one
GPU in a rehearsal.  LSEC_DIST_BACKEND=nccl puts it on RCCL instead.

Placement.  Every rank pins itself to the CPUs of its GPU's NUMA node (lsec_device_numa: PCI bus
id -> sysfs numa_node -> cpulist) before it allocates host buffers, so its host stripes, its
staging and the engine threads it starts are node-local.

Device-resident layout: data [N][k][C], parity [N][m][C] -- LStore's own layout (one cache
page holds a stripe's k chunks back to back, cache.c:3843; the parity buffer holds m,
segment/jerasure.c:1836).  --pad B leaves B unused bytes after every shard row instead;
layout.padded reports the same stripes with a 1 KiB pad, launch-timed, for the record.

Also reported (same JSON line):
  roofline      encode kernel: algorithmic HBM bytes (k+m)*C*N per launch / avg launch time
                (HIP events on the launch stream) vs 8 TB/s
  per_rank      every rank's own encode / decode launch rates and roofline fractions
  cpu_baseline  the reference CPU path (oracle/_ref: vendor/jerasure via the plan dispatch)
                on a bounded sample of the same workload, at 1 thread and at every usable
                host core of this box
  host_path     PCIe-inclusive rate of et_encode_stripes / et_decode_stripes from host memory;
                at N > 1 every rank runs it at the same time (barrier before every timed pass):
                per rank, and aggregated as sum of bytes / max time over ranks
  hbm_copy_ref  this box's device-to-device copy rate (the practical HBM ceiling) and the
                encode / decode kernels' rates relative to it
Every run checks parity bit-exactly against the reference (oracle/_ref) on sampled stripes.
"""
import argparse
import glob
import json
import os
import socket
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK = 8.0e12  # B/s, MI355X HBM3E (MI355X_MICROARCH.md)
HEADLINE = "erasure encode+decode GiB/s (device-resident), RS(6+3) 1 MiB stripes"


def parse(argv=None):
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
    ap.add_argument("--cpu-seconds", type=float, default=16.0, help="budget for the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host-path", action="store_true")
    ap.add_argument("--variant", type=str, default="0,0", help="bytewise,bitsliced kernel variants")
    ap.add_argument("--pad", type=int, default=0,
                    help="bytes left unused after every shard row in HBM (0 = LStore's layout, shards exactly C apart)")
    ap.add_argument("--no-layout-ab", action="store_true", help="skip the padded-layout comparison")
    ap.add_argument("--no-copy-ref", action="store_true", help="skip the device-copy HBM reference")
    ap.add_argument("--json-out", default="", help="also write rank 0's JSON line to this file")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the in-run rocprofv3 PMC traffic passes (roofline.traffic from a committed profile)")
    ap.add_argument("--share-gpus", action="store_true",
                    help="allow more ranks than visible GPUs (a rehearsal: ranks share devices, and the line says so)")
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------- CPU baseline
def usable_cpus():
    """(threads to use, CPUs visible): the affinity mask, capped by the cgroup CPU quota (the
    GPU box shows the whole machine's CPUs but grants a share of them)."""
    visible = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(-(-int(q) // int(p))))
    except (OSError, ValueError):
        pass
    return (min(visible, quota) if quota else visible), visible, quota


def cpu_baseline(method_id, k, m, C, P, lost, budget_s):
    """Reference CPU path (oracle/_ref: the real vendor/jerasure behind erasure_tools.c's
    dispatch) on a bounded sample of the workload, called per stripe as segment/jerasure.c:1847
    / :245 do: encode then decode(lost), at 1 thread and at every usable host core (each pthread
    takes a contiguous stripe range)."""
    import ctypes as Ct

    import oracle as O

    if not O.ref_available():
        return None
    threads, visible, quota = usable_cpus()
    rp = O.RefPlan(method_id, k, m, 8, P)

    def sample(nthreads, seconds, n):
        tile = np.random.default_rng(1).integers(0, 256, size=(min(n, 8), k + m, C), dtype=np.uint8)
        buf = np.empty((n, k + m, C), dtype=np.uint8)
        for s0 in range(0, n, tile.shape[0]):
            buf[s0:s0 + tile.shape[0]] = tile[: n - s0]
        base = buf.ctypes.data
        ptrs = (Ct.c_void_p * (n * (k + m)))(*[base + i * C for i in range(n * (k + m))])
        rp.encode_many(ptrs, min(n, nthreads), C, nthreads)  # warm tables / pages

        def passes(fn):
            # whole passes over the n-stripe buffer (far larger than the LLC) until the time is up
            t0, kp = time.perf_counter(), 0
            while True:
                rc = fn()
                kp += 1
                t = time.perf_counter() - t0
                if t >= seconds / 2:
                    return t / kp, kp, rc

        t_e, p_e, _ = passes(lambda: rp.encode_many(ptrs, n, C, nthreads))
        t_d, p_d, rc = passes(lambda: rp.decode_many(ptrs, n, C, nthreads, [lost]))
        gib = k * C * n / 2**30
        return {"value": round(gib / (t_e + t_d), 3), "encode_gibps": round(gib / t_e, 3),
                "decode_gibps": round(gib / t_d, 3), "threads": nthreads, "decode_rc": rc,
                "sample": f"{p_e} encode + {p_d} decode(lost {lost}) passes over {n} stripes "
                          f"({round(t_e * p_e + t_d * p_d, 1)} s)"}

    stripe_bytes = (k + m) * C
    # 1 thread: >= 512 MiB of stripes (beyond any one core's LLC slice), about 3/8 of the budget
    one = sample(1, budget_s * 0.375, max(2, min(512, (512 << 20) // stripe_bytes + 1)))
    allc = sample(threads, budget_s * 0.625, max(threads, min(512, (4608 << 20) // stripe_bytes + 1)))
    rp.close()
    return {"value": allc["value"], "unit": "GiB/s", "cores": threads, "kind": "reference",
            "sample": f"{allc['sample']} on {threads} pthreads; {one['sample']} on 1 thread; "
                      f"{k}+{m} x {C} B stripes, vendor/jerasure via oracle/_ref",
            "encode_gibps": allc["encode_gibps"], "decode_gibps": allc["decode_gibps"], "decode_rc": allc["decode_rc"],
            "threads_1": {k2: one[k2] for k2 in ("value", "encode_gibps", "decode_gibps")},
            "host_cpus_visible": visible, "cgroup_cpu_quota": quota}


def pmc_traffic(k, m, C, N, kernel_kind, pad):
    """HBM bytes per encode launch from the committed rocprofv3 PMC measurement of the same
    geometry and layout (tools/pmc_traffic.py -> profiles/*_pmc_traffic.json), scaled to N
    stripes; (None, None) when no measurement of this exact configuration exists."""
    import glob

    prefix = "void lsec::k_gf8_bytewise<%d," % m if kernel_kind == 1 else "void lsec::k_gf8_bitsliced<%d," % m
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")), reverse=True):
        with open(f) as fh:
            d = json.load(fh)
        if (d.get("k"), d.get("m"), d.get("chunk"), d.get("pad", 1024)) != (k, m, C, pad):
            continue
        for name, v in d["kernels"].items():
            if name.startswith(prefix):
                return int(v["traffic_per_stripe"] * N), os.path.relpath(f, ROOT)
    return None, None


def _run_killable(cmd, timeout, **kw):
    """subprocess.run in its own process group, the whole group killed on timeout (rocprofv3
    runs the profiled program as its own child)."""
    import signal
    import subprocess

    p = subprocess.Popen(cmd, start_new_session=True, **kw)
    try:
        return p.wait(timeout=timeout)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.wait()
        return None


# a launcher's rank variables: the PMC child is a single-rank run of rank 0's geometry
_DIST_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE",
             "GROUP_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def pmc_traffic_live(a, N):
    """roofline.traffic measured for this run's configuration: two rocprofv3 --pmc passes
    (FETCH_SIZE, then WRITE_SIZE: they do not fit one pass, MI355X_MICROARCH.md) over a 1-step
    child run of the same geometry, started before this process touches the GPU.  FETCH_SIZE and
    WRITE_SIZE are in KiB; gfx950 counts a coalesced streaming read at half its bytes, so FETCH is
    doubled (the guide's HBM section; checked against the algorithmic bytes in
    profiles/*_pmc_traffic.json).  The encode kernel is the engine kernel that writes the most.
    None when rocprofv3 is missing, this process already runs under a profiler, or a pass fails."""
    import csv
    import shutil
    import subprocess
    import tempfile

    if shutil.which("rocprofv3") is None or os.environ.get("LSEC_BENCH_PMC_CHILD"):
        return None
    if any(k.startswith("ROCPROF") for k in os.environ) or "rocprof" in os.environ.get("LD_PRELOAD", ""):
        return None
    args = ["--method", a.method, "--k", str(a.k), "--m", str(a.m), "--chunk", str(a.chunk), "--stripes", str(N),
            "--pad", str(a.pad), "--variant", a.variant, "--lost", str(a.lost), "--steps", "1", "--warmup", "0",
            "--no-cpu", "--no-host-path", "--no-layout-ab", "--no-copy-ref", "--no-pmc"]
    vals = {}
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            out = os.path.join(td, counter)
            cmd = ["rocprofv3", "--pmc", counter, "--kernel-trace", "--output-format", "csv", "-d", out, "-o", "pmc",
                   "--", sys.executable, os.path.abspath(__file__)] + args
            env = {key: v for key, v in os.environ.items() if key not in _DIST_ENV and not key.startswith("TORCHELASTIC")}
            rc = _run_killable(cmd, 240, cwd="/tmp", env=dict(env, TMPDIR="/tmp", LSEC_BENCH_PMC_CHILD="1"),
                               stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            if rc != 0:
                return None
            for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        name = row["Kernel_Name"]
                        if row.get("Counter_Name") == counter and "lsec" in name and "hbm_copy" not in name:
                            vals.setdefault((name, counter), []).append(float(row["Counter_Value"]) * 1024)
    med = {key: sorted(v)[len(v) // 2] for key, v in vals.items()}
    writes = {name: v for (name, c), v in med.items() if c == "WRITE_SIZE"}
    if not writes:
        return None
    name = max(writes, key=writes.get)
    fetch = med.get((name, "FETCH_SIZE"))
    if fetch is None:
        return None
    traffic = 2 * fetch + writes[name]
    return {"kernel": name, "fetch_raw": fetch, "write": writes[name], "traffic_per_stripe": traffic / N,
            "launches": len(vals.get((name, "FETCH_SIZE"), []))}


def host_path_aggregate(per_rank):
    """N > 1: whole-node PCIe-inclusive rate from every rank's concurrent passes: for pass i,
    sum of the ranks' user bytes / the slowest rank's time; median over passes."""
    out = {}
    for op in ("encode", "decode"):
        reps = min(len(r["times"][op + "_s"]) for r in per_rank)
        rates = sorted(sum(r["times"]["user_bytes"] for r in per_rank) /
                       max(r["times"][op + "_s"][i] for r in per_rank) / 2**30 for i in range(reps))
        out[op + "_gibps"] = round(rates[len(rates) // 2], 2)
    out["combined_gibps"] = round(1 / (1 / out["encode_gibps"] + 1 / out["decode_gibps"]), 2)
    return out


def host_path_rate(plan, k, m, C, lost, nstripes, pinned=False, reps=3, barrier=None):
    """et_encode_stripes / et_decode_stripes from host memory (PCIe-inclusive), median of reps.

    pinned=False: pageable numpy buffers (LStore's cache pages) -> pinned in place or packed
    into the engine's pinned staging -> H2D -> kernel -> D2H.  pinned=True: page-locked buffers
    (torch pin_memory = hipHostMalloc), DMA'd in place with no host copies.  barrier: called
    before every timed pass, so that ranks run their passes at the same time (N > 1); the raw
    pass times are returned in "times" for the aggregate."""
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
    te_all, td_all = [], []
    for _ in range(reps):
        if barrier:
            barrier()
        t0 = time.perf_counter()
        plan.encode_stripes(buf)
        te_all.append(time.perf_counter() - t0)
        if barrier:
            barrier()
        t0 = time.perf_counter()
        plan.decode_stripes(buf, [lost])
        td_all.append(time.perf_counter() - t0)
    te, td = sorted(te_all)[reps // 2], sorted(td_all)[reps // 2]
    gib = k * C * nstripes / 2**30
    return {"encode_gibps": round(gib / te, 2), "decode_gibps": round(gib / td, 2),
            "combined_gibps": round(gib / (te + td), 2), "stripes": nstripes,
            "times": {"encode_s": te_all, "decode_s": td_all, "user_bytes": k * C * nstripes},
            "note": ("page-locked host buffers -> DMA -> kernel -> DMA -> host" if pinned else
                     "pageable host buffers -> pinned staging -> H2D -> kernel -> D2H -> host")}


# the generic kernel of each lsec_plan_kernel kind (include/lstore_ec.h)
KERNEL_KINDS = {1: "k_gf8_bytewise", 2: "k_gf8_bitsliced", 3: "k_bitmatrix", 4: "k_gfw_transposed", 5: "k_gfw_bitsliced"}


def kernel_label(kind, jit, measured=None):
    """roofline.kernel: the encode kernel that actually ran.  `measured` is the kernel the in-run
    PMC pass saw write the most (the encode), named as rocprofv3 reports it; otherwise the plan
    says: its compiled network (lsec_xornet: XOR networks for wide RS codes and w = 16 / 32,
    packet networks for Cauchy and the liberation family, lsec_plan_jit) or the generic kernel of
    its kind."""
    if measured:
        return f"{measured} (encode; named by the in-run PMC pass)"
    generic = KERNEL_KINDS.get(kind, f"kind {kind}")
    if jit:
        return f"lsec_xornet (encode: compiled network in place of {generic})"
    return f"{generic} (encode)"


# SURVEY.md §8d's synthetic input: the splitmix64 stream from seed 0x4C53544F5245, stripe s's k
# data chunks at counter base s*k*C/8 (tests/patterns.py is the numpy statement of it)
SPLITMIX_SEED = 0x4C53544F5245


def _i64(x):
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >= 1 << 63 else x


def splitmix_rows(torch, rows, counter0, seed=SPLITMIX_SEED, words_per_pass=1 << 25):
    """rows (uint8 [R, C], C % 8 == 0, rows may be strided) <- the splitmix64 byte stream from
    word counter0 on, row after row: word i (1-based from counter0 + 1) is
    mix(seed + i * 0x9E3779B97F4A7C15).  int64 arithmetic wraps as uint64 does; the right shifts
    are masked to be logical."""
    R, C = rows.shape
    w = C // 8
    step = max(1, words_per_pass // w)
    for r0 in range(0, R, step):
        r1 = min(R, r0 + step)
        z = torch.arange(counter0 + r0 * w + 1, counter0 + r1 * w + 1, dtype=torch.int64, device=rows.device)
        z = z * _i64(0x9E3779B97F4A7C15) + _i64(seed)
        z = (z ^ ((z >> 30) & ((1 << 34) - 1))) * _i64(0xBF58476D1CE4E5B9)
        z = (z ^ ((z >> 27) & ((1 << 37) - 1))) * _i64(0x94D049BB133111EB)
        z = z ^ ((z >> 31) & ((1 << 33) - 1))
        rows[r0:r1].copy_(z.view(torch.uint8).view(r1 - r0, C))
        del z


# ----------------------------------------------------------------------------- the engine
class HipEngine:
    """The device-resident hot path: liblstore_ec.so's lsec_encode_dev / lsec_decode_dev on
    HBM-resident stripes, timed with HIP events on the launch stream."""

    def __init__(self, a, rank, world, local):
        import torch

        import lstore_amd as L
        from lstore_amd import erasure as E

        self.torch, self.L, self.E, self.a = torch, L, E, a
        ndev = torch.cuda.device_count()
        if local >= ndev and not a.share_gpus:
            raise SystemExit(f"rank {rank}: local rank {local} but {ndev} visible GPU(s); --share-gpus for a rehearsal")
        torch.cuda.set_device(local % ndev)
        self.dev = torch.device("cuda", torch.cuda.current_device())
        # control plane only (barrier, max, gather): gloo by default, RCCL opt-in
        self.backend = os.environ.get("LSEC_DIST_BACKEND", "gloo") if world > 1 else None
        # this rank's host threads and host buffers on its GPU's NUMA node (lsec_device_numa)
        self.numa = {"node": -1, "cpus": 0, "pinned": False}
        try:
            node, cpus = E.device_numa(self.dev.index)
            self.numa.update(node=node, cpus=len(cpus))
            if cpus and os.environ.get("LSEC_NUMA", "1") != "0":
                os.sched_setaffinity(0, cpus)
                self.numa["pinned"] = True
        except (E.ErasureError, OSError) as ex:
            self.numa["error"] = str(ex)
        bw_v, bs_v = (int(x) for x in a.variant.split(","))
        E.set_kernel_variant(bw_v, bs_v)
        self.method = E.JE_METHOD_NAMES.index(a.method)
        self.plan = L.Plan.for_chunk(self.method, a.k, a.m, a.chunk)
        self.P = self.plan.packet_size
        self.kernel = self.plan.kernel
        self.stream = torch.cuda.current_stream()
        self.sh = self.stream.cuda_stream
        self.er = E._erasure_array([a.lost])
        self.plan.prepare_encode()  # wide codes: wait for the plan's compiled XOR network
        self.plan.prepare_decode([a.lost])
        self.lib = E.lib()
        self.tensors = None
        self.flat = None
        # the layout A/B re-times the same stripes padded inside the SAME allocations: which
        # physical HBM pages an allocation gets moves these kernels by up to 8 % from one fresh
        # allocation to the next, the pad itself by about 1 % (profiles/r03_v4_alloc_probe.jsonl)
        self.room = 1024 if (world == 1 and not a.no_layout_ab) else 0

    @staticmethod
    def visible_devices():
        """GPUs this process can see (torch.cuda.device_count does not initialise HIP on this image,
        so the launcher may ask before it spawns the ranks)"""
        import torch
        return torch.cuda.device_count()

    def device_identity(self):
        """which physical GPU this rank runs on: index, PCI bus id and UUID"""
        props = self.torch.cuda.get_device_properties(self.dev)
        import ctypes
        buf = ctypes.create_string_buffer(64)
        hip = ctypes.CDLL("libamdhip64.so")
        bus = buf.value.decode() if hip.hipDeviceGetPCIBusId(buf, 64, self.dev.index) == 0 else None
        uuid = getattr(props, "uuid", None)
        return {"index": self.dev.index, "pci_bus_id": bus, "uuid": str(uuid) if uuid is not None else None,
                "name": props.name}

    def init_dist(self, dist):
        if self.backend == "nccl":
            dist.init_process_group("nccl", device_id=self.dev)
        else:
            dist.init_process_group(self.backend)

    def reduce_device(self, dist):
        return self.dev if dist.get_backend() == "nccl" else None

    def workload(self, N, pad, seed, first=0):
        """Synthetic stripes resident in HBM: data [N][k][C], parity [N][m][C] and the rebuilt
        shard [N][1][C], every shard row followed by `pad` unused bytes, in three flat
        allocations with room for the layout A/B's pad as well.  Returns the encode / decode
        launchers (the tensors stay referenced until drop())."""
        torch, a = self.torch, self.a
        k, m, C = a.k, a.m, a.chunk
        row = C + max(pad, self.room)
        self.flat = (torch.empty((N * k * row,), dtype=torch.uint8, device=self.dev),
                     torch.empty((N * m * row,), dtype=torch.uint8, device=self.dev),
                     torch.empty((N * row,), dtype=torch.uint8, device=self.dev))
        # the data chunks (global stripes first .. first+N-1) as the headline layout places them
        # (views(N, pad)), from SURVEY §8d's splitmix64 stream; the bytes between them stay as
        # allocated (only the layout A/B's timing passes read them)
        splitmix_rows(torch, self.flat[0][: N * k * (C + pad)].view(N * k, C + pad)[:, :C], first * k * C // 8)
        return self.views(N, pad)

    def views(self, N, pad):
        """encode / decode launchers over the flat allocations laid out with `pad` bytes after
        every shard row"""
        a, plan, lib, E = self.a, self.plan, self.lib, self.E
        k, m, C = a.k, a.m, a.chunk
        fd, fp, fr = self.flat
        data = fd[: N * k * (C + pad)].view(N, k, C + pad)[:, :, :C]
        par = fp[: N * m * (C + pad)].view(N, m, C + pad)[:, :, :C]
        rebuilt = fr[: N * (C + pad)].view(N, 1, C + pad)[:, :, :C]
        enc_refs, _, _ = plan.tensor_refs(data, par)
        enc_arr = plan.shard_refs(enc_refs)
        dec_refs = list(enc_refs)
        dec_refs[a.lost] = (rebuilt.data_ptr(), rebuilt.stride(0))
        dec_arr = plan.shard_refs(dec_refs)
        self.tensors = (data, par, rebuilt)

        def encode():
            if lib.lsec_encode_dev(plan.ptr, enc_arr, N, C, self.sh):
                raise E.ErasureError(E.last_error())

        def decode():
            if lib.lsec_decode_dev(plan.ptr, dec_arr, N, C, self.er, self.sh):
                raise E.ErasureError(E.last_error())

        return encode, decode

    def random_bytes(self, shape, seed=4321):
        """probe inputs: seeded random bytes like the coding kernels' stripes (HBM rates depend
        on the bytes moved, so a probe over zero pages would not be the same traffic)"""
        torch = self.torch
        g = torch.Generator(device=self.dev).manual_seed(seed)
        return torch.randint(0, 256, shape, dtype=torch.uint8, device=self.dev, generator=g)

    def drop(self):
        self.tensors = None
        self.flat = None
        self.torch.cuda.empty_cache()

    def sync(self):
        self.torch.cuda.synchronize()

    def launch_times(self, encode, decode, reps):
        """average encode / decode launch time (s), HIP events on the launch stream"""
        torch = self.torch
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record(self.stream)
        for _ in range(reps):
            encode()
        ev[1].record(self.stream)
        for _ in range(reps):
            decode()
        ev[2].record(self.stream)
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / 1e3 / reps, ev[1].elapsed_time(ev[2]) / 1e3 / reps

    def check(self, N):
        """Bit-exact parity of sampled stripes against the reference itself (oracle/_ref:
        vendor/jerasure), or the restatement when _ref is not built; the rebuilt shard must
        equal the lost one."""
        import oracle as O

        a = self.a
        data, par, rebuilt = self.tensors
        pick = sorted({0, N // 2, N - 1})
        hd, hp, hr = data[pick].cpu().numpy(), par[pick].cpu().numpy(), rebuilt[pick].cpu().numpy()
        ref = O.RefPlan(self.method, a.k, a.m, 8, self.P) if O.ref_available() else None
        ok = True
        for i in range(len(pick)):
            want = ref.encode(hd[i]) if ref else O.encode(self.method, hd[i], a.m, self.P)
            ok &= bool(np.array_equal(want, hp[i]))
            ok &= bool(np.array_equal(hr[i, 0], np.vstack([hd[i], hp[i]])[a.lost]))
        if ref:
            ref.close()
        return ok, ("bit-exact vs oracle/_ref (vendor/jerasure) on stripes %s" % pick if ref else
                    "bit-exact vs the oracle restatement on stripes %s (_ref not built)" % pick)

    def extras(self, N, t_enc, t_dec, rank, world, barrier=None):
        """N = 1 extras on rank 0: the padded layout A/B, the HBM copy probe and the CPU
        reference.  The PCIe-inclusive host path runs on every rank (concurrently at N > 1)."""
        a, torch, lib, E = self.a, self.torch, self.lib, self.E
        k, m, C = a.k, a.m, a.chunk
        out = {}
        enc_hbm, dec_hbm, data_bytes = (k + m) * C * N, (k + 1) * C * N, k * C * N
        reps = max(3, min(10, a.steps))
        layout = {"shard_pad_bytes": a.pad}
        if world == 1 and not a.no_layout_ab and self.flat is not None:
            # the same stripes with a 1 KiB pad after every shard row (or, when the headline is
            # padded, unpadded), in the headline's own allocations (so the same physical HBM
            # pages), launch-timed alternately with the headline layout for the record
            alt = 1024 if a.pad == 0 else 0
            enc0, dec0 = self.views(N, alt)
            enc1, dec1 = self.views(N, a.pad)
            enc0()
            dec0()
            t0s, t1s = [], []
            for _ in range(3):
                t0s.append(self.launch_times(enc0, dec0, reps))
                t1s.append(self.launch_times(enc1, dec1, reps))
            te0, td0 = (sorted(x)[1] for x in zip(*t0s))
            te1, td1 = (sorted(x)[1] for x in zip(*t1s))
            layout["same_allocation"] = True
            layout["headline_layout_retimed"] = {"encode_frac": round(enc_hbm / te1 / HBM_PEAK, 4),
                                                 "decode_frac": round(dec_hbm / td1 / HBM_PEAK, 4)}
            layout["padded" if alt else "unpadded"] = {
                "shard_pad_bytes": alt, "encode_frac": round(enc_hbm / te0 / HBM_PEAK, 4),
                "decode_frac": round(dec_hbm / td0 / HBM_PEAK, 4),
                "value_from_launch_times": round(data_bytes / (te0 + td0) / 2**30, 2),
                "headline_value_from_launch_times": round(data_bytes / (te1 + td1) / 2**30, 2)}
            del enc0, dec0, enc1, dec1
        out["layout"] = layout
        self.drop()
        if world == 1 and not a.no_copy_ref:
            # the box's practical HBM ceiling beside the spec peak: streaming device copies of the
            # encode launch's byte count (half read, half written), HIP events on the launch stream --
            # the engine's probe kernel (lsec_hbm_copy_dev: the coding kernels' memory shape) and torch's copy_
            nb = enc_hbm // 2
            src = self.random_bytes((nb,))
            dst = torch.empty_like(src)

            def probe():
                if lib.lsec_hbm_copy_dev(dst.data_ptr(), src.data_ptr(), nb, self.sh):
                    raise E.ErasureError(E.last_error())

            def timed(fn):
                fn()
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record(self.stream)
                for _ in range(reps):
                    fn()
                ev[1].record(self.stream)
                torch.cuda.synchronize()
                return ev[0].elapsed_time(ev[1]) / 1e3 / reps

            t_probe, t_torch = timed(probe), timed(lambda: dst.copy_(src))
            out["hbm_copy_ref"] = {
                "what": "device->device copy of (k+m)*C*N/2 bytes, read+write counted",
                "probe_GBps": round(2 * nb / t_probe / 1e9, 1), "probe_frac": round(2 * nb / t_probe / HBM_PEAK, 4),
                "torch_copy_GBps": round(2 * nb / t_torch / 1e9, 1),
                "encode_vs_probe": round((enc_hbm / t_enc) / (2 * nb / t_probe), 3),
                "decode_vs_probe": round((dec_hbm / t_dec) / (2 * nb / t_probe), 3)}
            del src, dst
            self.drop()
            # the encode's own traffic mix without its arithmetic: XOR of the k data shards written
            # to each of the m parity shards, in the encode kernel's tiles (lsec_hbm_mix_dev)
            md = self.random_bytes((N, k, C))
            mp = torch.empty((N, m, C), dtype=torch.uint8, device=self.dev)
            mrefs = self.plan.shard_refs([(md.data_ptr() + j * C, k * C) for j in range(k)] +
                                         [(mp.data_ptr() + r * C, m * C) for r in range(m)])

            def mix():
                if lib.lsec_hbm_mix_dev(mrefs, k, m, N, C, self.sh):
                    raise E.ErasureError(E.last_error())

            t_mix = timed(mix)
            out["hbm_copy_ref"]["encode_mix"] = {
                "what": "XOR of the k data shards to each of the m parity shards over N stripes: the encode's k:m bytes, no GF arithmetic",
                "frac": round(enc_hbm / t_mix / HBM_PEAK, 4),
                "encode_vs_mix": round(t_mix / t_enc, 3)}
            del md, mp
            self.drop()
            # the decode's own traffic mix without its arithmetic: a raid4 (k+1) decode of shard 0
            # is a plain XOR of the k survivors -- k reads : 1 write per column, as the decode
            xplan = self.L.Plan.for_chunk(E.JE_METHOD_NAMES.index("raid4"), k, 1, C)
            xd = self.random_bytes((N, k, C))
            xp = torch.empty((N, 1, C), dtype=torch.uint8, device=self.dev)
            refs, n, size = xplan.tensor_refs(xd, xp)
            t_xor = timed(lambda: xplan.decode_dev_refs(refs, n, size, [0], self.sh))
            out["hbm_copy_ref"]["xor_read_mix"] = {
                "what": "raid4(k+1) decode of shard 0 over N stripes: the decode's k:1 read:write bytes, XOR only",
                "frac": round(dec_hbm / t_xor / HBM_PEAK, 4),
                "decode_vs_xor": round(t_xor / t_dec, 3)}
            xplan.close()
            del xd, xp
            self.drop()
            out["hbm_copy_ref"]["decode_shape"] = self.decode_shape(N, timed)
            self.drop()
        if rank == 0 and world == 1:
            # the reference CPU path is timed at N=1 only (at N>1 it would only delay the ranks' exit)
            out["cpu_baseline"] = None if a.no_cpu else cpu_baseline(self.method, k, m, C, self.P, a.lost, a.cpu_seconds)
        if not a.no_host_path:
            # every rank: its own stripes from its own (node-local) host memory over its own link
            ns = max(8, min(256, (4 << 30) // ((k + m) * C)))
            host = host_path_rate(self.plan, k, m, C, a.lost, ns, barrier=barrier)
            host["pinned"] = host_path_rate(self.plan, k, m, C, a.lost, ns, pinned=True, barrier=barrier)
            out["host_path"] = host
        return out

    def decode_shape(self, N, timed):
        """The decode's own memory shape in a kernel that shares no code with it
        (lsec_hbm_decode_shape_dev: XOR of the decode's k survivors into one output, every IT / grab
        / XCD-order variant), timed on one fresh allocation together with the real decode over the
        same buffers, so both draw the same placement mode."""
        torch, a, lib, E = self.torch, self.a, self.lib, self.E
        k, m, C = a.k, a.m, a.chunk
        dec_hbm = (k + 1) * C * N
        dd = self.random_bytes((N, k, C))
        dq = torch.empty((N, m, C), dtype=torch.uint8, device=self.dev)
        dr = torch.empty((N, 1, C), dtype=torch.uint8, device=self.dev)
        refs = [(dd.data_ptr() + j * C, k * C) for j in range(k)] + [(dq.data_ptr() + r * C, m * C) for r in range(m)]
        enc_arr = self.plan.shard_refs(refs)
        dec_refs = list(refs)
        dec_refs[a.lost] = (dr.data_ptr(), C)
        dec_arr = self.plan.shard_refs(dec_refs)
        if lib.lsec_encode_dev(self.plan.ptr, enc_arr, N, C, self.sh):  # consistent parity
            raise E.ErasureError(E.last_error())
        survivors = [refs[j] for j in range(k + m) if j != a.lost][:k]
        probe_arr = self.plan.shard_refs(survivors + [(dr.data_ptr(), C)])

        def decode():
            if lib.lsec_decode_dev(self.plan.ptr, dec_arr, N, C, self.er, self.sh):
                raise E.ErasureError(E.last_error())

        variants = {}
        t_dec = timed(decode)
        for remap in (0, 1):
            for it in (1, 2, 4):
                if C % (4096 * it):
                    continue
                for g in (1, 2, 4):
                    v = it | g << 4 | remap << 8

                    def probe(v=v):
                        if lib.lsec_hbm_decode_shape_dev(probe_arr, k, N, C, v, self.sh):
                            raise E.ErasureError(E.last_error())

                    variants[f"it{it}_g{g}_{'xcd' if remap else 'rr'}"] = timed(probe)
        t_dec2 = timed(decode)  # the decode again after the sweep: the allocation's rate held
        del dd, dq, dr
        if not variants:
            return None
        best = min(variants, key=variants.get)
        td = min(t_dec, t_dec2)
        return {"what": "XOR of the decode's k survivors into one shard over N stripes in a kernel sharing no code with "
                        "the coding kernels (lsec_hbm_decode_shape_dev), every variant; the real decode timed before "
                        "and after on the same buffers",
                "best_variant": best, "best_frac": round(dec_hbm / variants[best] / HBM_PEAK, 4),
                "decode_frac_same_buffers": round(dec_hbm / td / HBM_PEAK, 4),
                "decode_frac_before_after": [round(dec_hbm / t_dec / HBM_PEAK, 4), round(dec_hbm / t_dec2 / HBM_PEAK, 4)],
                "decode_vs_shape": round(variants[best] / td, 3),
                "variants_frac": {key: round(dec_hbm / t / HBM_PEAK, 4) for key, t in variants.items()}}

    def kernel_name(self):
        return kernel_label(self.kernel, self.plan.jit(), (getattr(self.a, "traffic_live", None) or {}).get("kernel"))

    def traffic(self, N):
        live = getattr(self.a, "traffic_live", None)
        if live:
            return int(live["traffic_per_stripe"] * N), (
                "measured in this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over a 1-step child "
                f"run of this configuration, FETCH x2 (gfx950), kernel {live['kernel']}, median of {live['launches']} launches")
        return pmc_traffic(self.a.k, self.a.m, self.a.chunk, N, self.kernel, self.a.pad)

    def close(self):
        self.drop()
        self.plan.close()


# ----------------------------------------------------------------------------- one rank
def run_rank(a, rank, world, local, engine_cls=HipEngine):
    """One rank of the benchmark (also what tests/test_multirank.py runs over gloo with a CPU
    engine).  Returns rank 0's JSON dict (None on other ranks)."""
    import torch.distributed as dist

    from lstore_amd.partition import max_over_ranks, stripe_range

    eng = engine_cls(a, rank, world, local)
    if world > 1:
        # one process per GPU; the only collectives are the timing barrier, the max-over-ranks
        # reduction and the gather of per-rank figures (RCCL by default)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        eng.init_dist(dist)
    # which physical GPU every rank runs on, checked before any work: N ranks must be N devices
    # unless the run says it is a rehearsal (--share-gpus)
    ident = eng.device_identity() if hasattr(eng, "device_identity") else None
    idents = [ident]
    if world > 1:
        idents = [None] * world
        dist.all_gather_object(idents, ident)
    dup = duplicate_devices(idents)
    if dup and not a.share_gpus:
        if rank == 0:
            print(json.dumps({"error": f"ranks {dup} run on the same GPU; --share-gpus for a rehearsal",
                              "devices": idents}), flush=True)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        eng.close()
        raise SystemExit(1)
    k, m, C, N = a.k, a.m, a.chunk, a.stripes
    first = rank * N  # global index of this rank's first stripe
    if a.total_stripes > 0:
        first, s1 = stripe_range(a.total_stripes, world, rank)
        N = s1 - first
        if N <= 0:
            raise SystemExit(f"rank {rank}: --total-stripes {a.total_stripes} leaves no stripes for {world} ranks")
    encode, decode = eng.workload(N, a.pad, 1234 + rank, first)

    for _ in range(a.warmup):
        encode()
        decode()
    eng.sync()

    # ---- timed region: K steps, barrier + synchronize on both sides
    if world > 1:
        dist.barrier()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        encode()
        decode()
    eng.sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = max_over_ranks(elapsed, eng.reduce_device(dist))

    # ---- per-kernel timing on the launch stream (roofline), on every rank
    reps = max(3, min(10, a.steps))
    t_enc, t_dec = eng.launch_times(encode, decode, reps)

    # ---- parity check (bit-exact vs the reference on sampled stripes), on every rank
    ok, parity_note = eng.check(N)
    data_bytes = k * C * N
    enc_hbm = (k + m) * C * N
    dec_hbm = (k + 1) * C * N
    mine = {"rank": rank, "device": ident, "stripes": N, "parity_ok": ok,
            "encode_gibps": round(data_bytes / t_enc / 2**30, 2), "decode_gibps": round(data_bytes / t_dec / 2**30, 2),
            "encode_frac": round(enc_hbm / t_enc / HBM_PEAK, 4), "decode_frac": round(dec_hbm / t_dec / HBM_PEAK, 4),
            "avg_encode_launch_ms": round(t_enc * 1e3, 4), "avg_decode_launch_ms": round(t_dec * 1e3, 4)}
    if world > 1:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    else:
        per_rank = [mine]
    if not all(r["parity_ok"] for r in per_rank):
        if rank == 0:
            print(json.dumps({"error": "parity mismatch vs reference", "per_rank": per_rank}), flush=True)
        raise SystemExit(1)

    extras = eng.extras(N, t_enc, t_dec, rank, world, barrier=dist.barrier if world > 1 else None)
    host = extras.get("host_path")
    if host is not None:
        host["numa"] = getattr(eng, "numa", None)
        if world > 1:
            # every rank's concurrent host-path passes -> per-rank figures and the node aggregate
            ranks = [None] * world
            dist.all_gather_object(ranks, host)
            agg = {"what": "all ranks at once: sum of user bytes / slowest rank's pass time, median of passes",
                   "pageable": host_path_aggregate(ranks),
                   "pinned": host_path_aggregate([r["pinned"] for r in ranks]),
                   "per_rank": [{key: r.get(key) for key in ("encode_gibps", "decode_gibps", "numa")} |
                                {"pinned": {key: r["pinned"][key] for key in ("encode_gibps", "decode_gibps")}}
                                for r in ranks]}
            host = dict(host, aggregate=agg)
        host.pop("times", None)
        host["pinned"].pop("times", None)
    if a.total_stripes > 0:
        value = k * C * a.total_stripes * a.steps / elapsed / 2**30
    else:
        value = data_bytes * world * a.steps / elapsed / 2**30
    achieved = enc_hbm / t_enc
    traffic, traffic_src = eng.traffic(N)

    out = None
    if rank == 0:
        method = a.method
        out = {
            "metric": HEADLINE if (method, k, m, C) == ("reed_sol_van", 6, 3, 1 << 20) else
            f"erasure encode+decode GiB/s (device-resident), {method}({k}+{m}) {C} B chunks",
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
            "data": "synthetic: SURVEY §8d splitmix64 stream, seed 0x4C53544F5245, stripe s at word s*k*C/8, resident in HBM",
            "config": {"workload": f"{method}({k}+{m}) encode + decode(lost shard {a.lost}), C={C} B per shard, "
                                   f"{N} stripes/GPU, k*C={k * C} B user data per stripe",
                       "method": method, "k": k, "m": m, "chunk_bytes": C, "packet_size": eng.P,
                       "stripes_per_gpu": N, "lost_shard": a.lost, "shard_pad_bytes": a.pad,
                       "parallelism": f"static stripe partition x{world}" + (
                           f" (rehearsal: {world} ranks on {len({_dev_key(d) for d in idents})} GPU(s), --share-gpus)"
                           if dup else "")},
            "distinct_gpus": None if ident is None else len({_dev_key(d) for d in idents}),
            "encode_gibps": round(data_bytes / t_enc / 2**30, 2),
            "decode_gibps": round(data_bytes / t_dec / 2**30, 2),
            "roofline": {"bound": "hbm", "achieved": round(achieved / 1e9, 1), "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": eng.kernel_name(),
                         "algorithmic_bytes_per_launch": enc_hbm, "avg_launch_ms": round(t_enc * 1e3, 4),
                         "decode_achieved_GBps": round(dec_hbm / t_dec / 1e9, 1),
                         "decode_frac": round(dec_hbm / t_dec / HBM_PEAK, 4)},
            "per_rank": per_rank,
            "layout": extras.get("layout"),
            "hbm_copy_ref": extras.get("hbm_copy_ref"),
            "cpu_baseline": extras.get("cpu_baseline"),
            "host_path": host,
            "parity_check": parity_note,
        }
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    eng.close()
    return out


def _dev_key(d):
    return None if d is None else (d.get("uuid") or d.get("pci_bus_id") or d.get("index"))


def duplicate_devices(idents):
    """rank lists of ranks that share one physical GPU ([] when every rank has its own, or when
    the engine reports no identity)"""
    by = {}
    for r, d in enumerate(idents):
        key = _dev_key(d)
        if key is not None:
            by.setdefault(key, []).append(r)
    return [v for v in by.values() if len(v) > 1]


# ----------------------------------------------------------------------------- launching
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawned(rank, a, world, port, engine_cls):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    run_rank(a, rank, world, rank, engine_cls)


def preflight(a, engine_cls=HipEngine):
    """The launch's arguments against the launcher and the visible devices: 0, or 2 after printing
    the reason (before anything touches a GPU)."""
    env_world = os.environ.get("WORLD_SIZE")
    err = None
    if a.gpus < 1:
        err = f"--gpus {a.gpus} < 1"
    elif env_world is not None and int(env_world) != a.gpus:
        err = f"WORLD_SIZE={env_world} but --gpus {a.gpus}: launch one rank per GPU"
    else:
        visible = getattr(engine_cls, "visible_devices", None)
        ndev = visible() if visible else None
        if ndev is not None and a.gpus > ndev and not a.share_gpus:
            err = (f"--gpus {a.gpus} but {ndev} GPU(s) visible: one rank per GPU "
                   "(--share-gpus for a rehearsal that puts several ranks on one GPU)")
    if err:
        print(json.dumps({"error": err}), flush=True)
        return 2
    return 0


def launch(a, engine_cls=HipEngine):
    """Run the benchmark on a.gpus ranks; returns the process exit code."""
    env_world = os.environ.get("WORLD_SIZE")
    rc = preflight(a, engine_cls)
    if rc:
        return rc
    if env_world is not None:
        world = int(env_world)
        run_rank(a, int(os.environ.get("RANK", "0")), world, int(os.environ.get("LOCAL_RANK", "0")), engine_cls)
        return 0
    if a.gpus == 1:
        run_rank(a, 0, 1, 0, engine_cls)
        return 0
    # self-launch: N ranks, one process per GPU, spawned before this process touches the GPU
    import torch.multiprocessing as mp

    ctx = mp.start_processes(_spawned, args=(a, a.gpus, _free_port(), engine_cls), nprocs=a.gpus,
                             join=False, start_method="spawn")
    try:
        while not ctx.join():
            pass
    except mp.ProcessRaisedException as e:
        print(json.dumps({"error": "a rank failed", "detail": str(e)[-2000:]}), flush=True)
        return 1
    except mp.ProcessExitedException as e:
        print(json.dumps({"error": "a rank exited", "detail": str(e)[-2000:]}), flush=True)
        return 1
    return 0


def main():
    a = parse()
    rc = preflight(a)
    if rc:
        sys.exit(rc)
    if not a.no_pmc and os.environ.get("RANK", "0") == "0":
        # before this process touches the GPU (before it spawns ranks, or, under a launcher, on
        # rank 0 before it joins the others): the counter passes run rank 0's geometry as a
        # single-rank child under rocprofv3, on rank 0's GPU
        world = int(os.environ.get("WORLD_SIZE", a.gpus))
        n0 = a.stripes
        if a.total_stripes > 0:
            from lstore_amd.partition import stripe_range
            s0, s1 = stripe_range(a.total_stripes, world, 0)
            n0 = s1 - s0
        a.traffic_live = pmc_traffic_live(a, n0)
    sys.exit(launch(a))


if __name__ == "__main__":
    main()
