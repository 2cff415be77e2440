"""bench.py's own multi-rank path on the GPU box: `bench.py --gpus 2` with no external launcher
(two ranks spawned by bench.py itself, sharing the one GPU over gloo), checked for the JSON
contract.  8-GPU runs belong to the driver; this is the N > 1 code path at small size."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_self_launches_two_ranks(cuda, tmp_path):
    out = tmp_path / "line.json"
    env = dict(os.environ, LSEC_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "-u", "bench.py", "--gpus", "2", "--stripes", "64", "--steps", "3", "--warmup", "1",
                        "--no-cpu", "--no-host-path", "--share-gpus", "--json-out", str(out)],
                       cwd=ROOT, env=env, timeout=240, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = json.loads(out.read_text())
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert [p["rank"] for p in line["per_rank"]] == [0, 1]
    assert all(p["parity_ok"] and p["stripes"] == 64 for p in line["per_rank"])
    assert line["parity_check"].startswith("bit-exact")
    assert line["value"] > 0 and line["roofline"]["frac"] > 0
    # the one-GPU box: both ranks on one device, and the line says it is a rehearsal
    assert line["distinct_gpus"] == 1 and "rehearsal" in line["config"]["parallelism"]
    assert line["per_rank"][0]["device"]["pci_bus_id"] == line["per_rank"][1]["device"]["pci_bus_id"]
    # the in-run PMC pass runs before the spawn at N > 1 too: traffic on the line
    assert line["roofline"]["traffic"] and "measured in this run" in line["roofline"]["traffic_source"]


@pytest.mark.gpu
def test_bench_refuses_more_ranks_than_gpus(cuda):
    """--gpus 2 on a one-GPU box without --share-gpus is refused before any rank starts"""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "-u", "bench.py", "--gpus", "2", "--stripes", "8", "--no-pmc"], cwd=ROOT, env=env,
                       timeout=120, capture_output=True, text=True)
    assert r.returncode == 2 and "GPU(s) visible" in r.stdout, r.stdout[-1000:] + r.stderr[-1000:]


def test_bench_refuses_mismatched_world_size(tmp_path):
    """(CPU) under an external launcher, WORLD_SIZE must equal --gpus"""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--stripes", "8"], cwd=ROOT, env=env, timeout=120,
                       capture_output=True, text=True)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stdout
