import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box via gpurun)")
    # an engine abort (ec_plan.cpp fatal) also appends its reason here: pytest's capture of fd 2
    # is lost with an aborting process
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    os.environ.setdefault("LSEC_FATAL_LOG", os.path.join(ROOT, "gpurun_out", "lsec_fatal.log"))


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np

    d = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(d, "plans.json")) as f:
        plans = json.load(f)["plans"]
    with open(os.path.join(d, "vectors.json")) as f:
        vectors = json.load(f)["vectors"]
    small = dict(np.load(os.path.join(d, "parity_small.npz"), allow_pickle=False))
    return dict(plans=plans, vectors=vectors, small=small)


@pytest.fixture(scope="session")
def built():
    """The engine library and the oracle restatement, built in-tree."""
    import oracle
    import lstore_amd

    lstore_amd.build_library()
    oracle.build()
    return True


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but torch.cuda is not available")
    import lstore_amd

    lstore_amd.build_library()
    return torch.device("cuda:0")
