"""gloo rehearsal (2, 4 and 8 ranks) of bench.py's multi-GPU path (CPU only).

The ranks run bench.py's own code: ``bench.launch`` self-spawns them (WORLD_SIZE unset,
``--gpus 2``) and each runs ``bench.run_rank`` -- partition, warm-up, the barrier-bracketed
timed region, max-over-ranks, per-rank gather and rank 0's JSON line.  Only the engine is
swapped: ``OracleEngine`` below stands in for ``bench.HipEngine`` (no GPU here) and encodes /
decodes with the CPU restatement, recording a CRC per global stripe so the test can check that
the union of the ranks' work is exactly the single-process result.
"""
import json
import os
import shutil
import time
import zlib

import numpy as np
import pytest

import bench
from lstore_amd.partition import stripe_range


class _OracleHostPlan:
    """Plan.encode_stripes / decode_stripes over the CPU oracle (test infrastructure only)."""

    def __init__(self, O, method, k, m, P):
        self.O, self.method, self.k, self.m, self.P = O, method, k, m, P
        self.barriers = 0

    def encode_stripes(self, buf):
        for s in range(buf.shape[0]):
            buf[s, self.k:] = self.O.encode(self.method, buf[s, :self.k], self.m, self.P)

    def decode_stripes(self, buf, lost):
        for s in range(buf.shape[0]):
            assert self.O.decode(self.method, buf[s], self.k, list(lost), self.P) == 0


class OracleEngine:
    """bench.HipEngine's interface over the CPU oracle (test infrastructure only)."""

    def __init__(self, a, rank, world, local):
        import oracle as O

        self.O, self.a, self.rank, self.local = O, a, rank, local
        self.method = O.REED_SOL_VAN if a.method == "reed_sol_van" else O.CAUCHY_GOOD
        self.P = O.generate_plan(a.k * a.chunk, self.method, a.k, a.m)["packet_size"]
        self.kernel = 1
        self.stripes = None

    # a fake device set (the environment reaches spawned ranks): LSEC_TEST_FAKE_GPUS devices are
    # visible; LSEC_TEST_FAKE_SAME=1 makes every rank report the same physical device
    @staticmethod
    def visible_devices():
        return int(os.environ.get("LSEC_TEST_FAKE_GPUS", "64"))

    def device_identity(self):
        ndev = self.visible_devices()
        idx = 0 if os.environ.get("LSEC_TEST_FAKE_SAME") == "1" else self.local % ndev
        return {"index": idx, "pci_bus_id": "0000:%02x:00.0" % (0x10 + idx), "uuid": None, "name": "fake"}

    def init_dist(self, dist):
        dist.init_process_group("gloo")

    def reduce_device(self, dist):
        return None

    def workload(self, N, pad, seed, first=0):
        from patterns import stripe

        a, O = self.a, self.O
        self.first = first
        self.stripes = np.zeros((N, a.k + a.m, a.chunk), np.uint8)
        for s in range(N):
            self.stripes[s, :a.k] = stripe(a.k, a.chunk, first + s)
        self.rebuilt = np.zeros((N, a.chunk), np.uint8)

        def encode():
            for s in range(N):
                self.stripes[s, a.k:] = O.encode(self.method, self.stripes[s, :a.k], a.m, self.P)

        def decode():
            for s in range(N):
                sh = self.stripes[s].copy()
                sh[a.lost] = 0
                assert O.decode(self.method, sh, a.k, [a.lost], self.P) == 0
                self.rebuilt[s] = sh[a.lost]

        return encode, decode

    def sync(self):
        pass

    def launch_times(self, encode, decode, reps):
        t0 = time.perf_counter()
        encode()
        t1 = time.perf_counter()
        decode()
        return max(t1 - t0, 1e-9), max(time.perf_counter() - t1, 1e-9)

    def check(self, N):
        ok = all(np.array_equal(self.rebuilt[s], self.stripes[s, self.a.lost]) for s in range(N))
        dump = os.environ.get("LSEC_TEST_DUMP")
        if dump:
            crcs = {self.first + s: zlib.crc32(self.stripes[s, self.a.k:].tobytes()) for s in range(N)}
            with open(os.path.join(dump, f"rank{self.rank}.json"), "w") as f:
                json.dump(crcs, f)
        return ok, "rebuilt == lost shard (oracle engine)"

    def extras(self, N, t_enc, t_dec, rank, world, barrier=None):
        if self.a.no_host_path:
            return {}
        # bench.host_path_rate's concurrent passes over the oracle (both legs pageable here: no
        # page-locked memory without a GPU)
        plan = _OracleHostPlan(self.O, self.method, self.a.k, self.a.m, self.P)
        host = bench.host_path_rate(plan, self.a.k, self.a.m, self.a.chunk, self.a.lost, 4, barrier=barrier)
        host["pinned"] = bench.host_path_rate(plan, self.a.k, self.a.m, self.a.chunk, self.a.lost, 4, barrier=barrier)
        return {"host_path": host}

    def kernel_name(self):
        return "oracle (test engine)"

    def traffic(self, N):
        return None, None

    def close(self):
        self.stripes = None


def _args(*extra):
    return bench.parse(["--chunk", "4096", "--steps", "2", "--warmup", "1", "--no-cpu", "--no-host-path",
                        "--no-layout-ab", "--no-copy-ref", *extra])


@pytest.mark.parametrize("world,total", [(2, 7), (2, 16), (4, 16), (8, 16), (8, 9)])
def test_self_launched_ranks_match_single_process(built, tmp_path, monkeypatch, world, total):
    """bench.launch(--gpus N) with no external launcher: N gloo ranks, strong partition (the
    driver's 4- and 8-GPU runs rehearsed on the CPU)."""
    import oracle as O
    from patterns import stripe

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setenv("LSEC_TEST_DUMP", str(tmp_path))
    out = tmp_path / "line.json"
    rc = bench.launch(_args("--gpus", str(world), "--total-stripes", str(total), "--json-out", str(out)), OracleEngine)
    assert rc == 0
    line = json.loads(out.read_text())
    assert line["n_gpus"] == world and line["scaling"] == "strong"
    assert [r["rank"] for r in line["per_rank"]] == list(range(world))
    assert [r["stripes"] for r in line["per_rank"]] == [b - a for a, b in (stripe_range(total, world, r) for r in range(world))]
    assert all(r["parity_ok"] for r in line["per_rank"])
    assert line["value"] > 0 and line["ms_per_step"] > 0
    merged = {}
    for r in range(world):
        part = {int(s): c for s, c in json.loads((tmp_path / f"rank{r}.json").read_text()).items()}
        assert not set(part) & set(merged)
        merged.update(part)
    assert sorted(merged) == list(range(total))
    for s in range(total):
        assert merged[s] == zlib.crc32(O.encode(O.REED_SOL_VAN, stripe(6, 4096, s), 3).tobytes())


@pytest.mark.parametrize("world", [2, 8])
def test_self_launched_weak_scaling(built, tmp_path, monkeypatch, world):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setenv("LSEC_TEST_DUMP", str(tmp_path))
    out = tmp_path / "line.json"
    rc = bench.launch(_args("--gpus", str(world), "--stripes", "3", "--method", "cauchy_good", "--json-out", str(out)),
                      OracleEngine)
    assert rc == 0
    line = json.loads(out.read_text())
    assert line["n_gpus"] == world and line["scaling"] == "weak"
    assert [r["stripes"] for r in line["per_rank"]] == [3] * world
    seen = set()
    for r in range(world):
        seen |= {int(s) for s in json.loads((tmp_path / f"rank{r}.json").read_text())}
    assert seen == set(range(3 * world))  # rank r owns stripes [3r, 3r+3)


def test_host_path_on_every_rank_with_aggregate(built, tmp_path, monkeypatch):
    """N > 1: every rank times the host path (its passes barrier-aligned with the other ranks'),
    and rank 0 reports per-rank rates and the aggregate (sum of bytes / slowest rank's time)."""
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    out = tmp_path / "line.json"
    args = bench.parse(["--chunk", "4096", "--steps", "1", "--warmup", "0", "--no-cpu", "--no-layout-ab",
                        "--no-copy-ref", "--gpus", "2", "--stripes", "2", "--json-out", str(out)])
    assert bench.launch(args, OracleEngine) == 0
    line = json.loads(out.read_text())
    host = line["host_path"]
    agg = host["aggregate"]
    assert len(agg["per_rank"]) == 2
    for leg in ("pageable", "pinned"):
        assert agg[leg]["encode_gibps"] > 0 and agg[leg]["decode_gibps"] > 0
    # the aggregate is at most the sum of the ranks' own (median) rates, at least the slowest rank's
    assert agg["pageable"]["encode_gibps"] >= 0.5 * min(r["encode_gibps"] for r in agg["per_rank"])
    assert "times" not in host and "times" not in host["pinned"]


def test_host_path_aggregate_is_sum_over_max():
    ranks = [{"times": {"encode_s": [1.0, 2.0, 1.0], "decode_s": [1.0, 1.0, 1.0], "user_bytes": 2**30}},
             {"times": {"encode_s": [2.0, 1.0, 4.0], "decode_s": [0.5, 0.5, 0.5], "user_bytes": 2**30}}]
    agg = bench.host_path_aggregate(ranks)
    assert agg["encode_gibps"] == 1.0  # passes: 2/2, 2/2, 2/4 -> median 1
    assert agg["decode_gibps"] == 2.0
    assert agg["combined_gibps"] == round(1 / (1 / 1.0 + 1 / 2.0), 2)


def test_world_size_must_match_gpus(built, monkeypatch, capsys):
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.launch(_args("--gpus", "4"), OracleEngine) == 2
    assert "WORLD_SIZE=2" in capsys.readouterr().out


def test_more_ranks_than_gpus_is_refused_unless_shared(built, tmp_path, monkeypatch, capsys):
    """--gpus N beyond the visible devices is refused before any rank starts;
    --share-gpus runs it as a rehearsal and the line says so."""
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setenv("LSEC_TEST_FAKE_GPUS", "1")
    assert bench.launch(_args("--gpus", "2", "--stripes", "2"), OracleEngine) == 2
    assert "1 GPU(s) visible" in capsys.readouterr().out
    out = tmp_path / "line.json"
    assert bench.launch(_args("--gpus", "2", "--stripes", "2", "--share-gpus", "--json-out", str(out)), OracleEngine) == 0
    line = json.loads(out.read_text())
    assert line["distinct_gpus"] == 1 and "rehearsal" in line["config"]["parallelism"]
    assert [r["device"]["pci_bus_id"] for r in line["per_rank"]] == ["0000:10:00.0"] * 2


def test_ranks_on_one_device_are_refused(built, monkeypatch, capfd):
    """Two ranks that report the same physical GPU (bus id / UUID) stop before the timed region
    unless --share-gpus is given."""
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setenv("LSEC_TEST_FAKE_SAME", "1")
    assert bench.launch(_args("--gpus", "2", "--stripes", "2"), OracleEngine) == 1
    assert "run on the same GPU" in capfd.readouterr().out


def test_per_rank_devices_are_recorded(built, tmp_path, monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    out = tmp_path / "line.json"
    assert bench.launch(_args("--gpus", "2", "--stripes", "2", "--json-out", str(out)), OracleEngine) == 0
    line = json.loads(out.read_text())
    assert line["distinct_gpus"] == 2 and "rehearsal" not in line["config"]["parallelism"]
    assert [r["device"]["pci_bus_id"] for r in line["per_rank"]] == ["0000:10:00.0", "0000:11:00.0"]


def test_duplicate_devices():
    a, b = {"uuid": "u0", "pci_bus_id": "x"}, {"uuid": "u1", "pci_bus_id": "x"}
    assert bench.duplicate_devices([a, b]) == []  # the UUID decides when present
    assert bench.duplicate_devices([{"pci_bus_id": "x"}, {"pci_bus_id": "y"}, {"pci_bus_id": "x"}]) == [[0, 2]]
    assert bench.duplicate_devices([None, None]) == []


def test_pmc_child_runs_without_rank_variables(monkeypatch, tmp_path):
    """The in-run PMC pass at N > 1 runs rank 0's geometry as a single-rank child: the launcher's
    rank variables must not reach it (it would refuse WORLD_SIZE != --gpus)."""
    seen = {}

    def fake_run(cmd, timeout, **kw):
        seen["cmd"], seen["env"] = cmd, kw["env"]
        return 1  # as a failed pass: pmc_traffic_live gives up

    monkeypatch.setattr(bench, "_run_killable", fake_run)
    monkeypatch.setattr(shutil, "which", lambda x: "/bin/true")
    for key, v in (("RANK", "0"), ("WORLD_SIZE", "8"), ("LOCAL_RANK", "0"), ("MASTER_PORT", "1234")):
        monkeypatch.setenv(key, v)
    for key in [k for k in os.environ if k.startswith("ROCPROF")]:
        monkeypatch.delenv(key)
    assert bench.pmc_traffic_live(_args("--gpus", "8", "--total-stripes", "100"), 13) is None
    assert not {"RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"} & set(seen["env"])
    i = seen["cmd"].index("--stripes")
    assert seen["cmd"][i + 1] == "13" and "--total-stripes" not in seen["cmd"]


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


def test_usable_cpus_reports_quota_and_visible():
    threads, visible, quota = bench.usable_cpus()
    assert 1 <= threads <= visible
    if quota:
        assert threads <= quota
