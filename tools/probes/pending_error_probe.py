#!/usr/bin/env python3
"""Development probe: what sits in this thread's HIP last-error slot during a sweep-like run, and
what a pending error costs the host path (lsec::quiet runs its queries on a helper thread while the
caller's slot holds an error).  Prints one JSON line per step.

python tools/probes/pending_error_probe.py
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import lstore_amd as L  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")


def peek(step):
    print(json.dumps({"step": step, "pending": hip.hipPeekAtLastError()}), flush=True)


def timed(step, fn, reps=3):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    print(json.dumps({"step": step, "ms": [round(t * 1e3, 2) for t in ts], "pending_after": hip.hipPeekAtLastError()}),
          flush=True)


peek("start")
x = torch.randint(0, 256, (1 << 20,), dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
peek("after torch ops")
k, m, C = 8, 3, 512 << 10
n = (1 << 30) // (k * C)
buf = np.empty((n, k + m, C), dtype=np.uint8)
buf[:] = np.random.default_rng(1).integers(0, 256, (1, k + m, C), dtype=np.uint8)
p = L.Plan.for_chunk(L.REED_SOL_VAN, k, m, C)
p.prepare_decode([0])
peek("after plan")
p.encode_stripes(buf[:1])
peek("after 1-stripe encode")
timed("encode 1 GiB", lambda: p.encode_stripes(buf))
timed("decode 1 GiB", lambda: p.decode_stripes(buf, [0]))
d = torch.empty((4096, k, C), dtype=torch.uint8, device="cuda")
par = torch.empty((4096, m, C), dtype=torch.uint8, device="cuda")
p.encode_dev(d, par)
torch.cuda.synchronize()
peek("after device encode")
# a pending error of the caller's own, left unread
junk = np.zeros(1 << 16, np.uint8)
code = hip.hipHostUnregister(ctypes.c_void_p(junk.ctypes.data))
peek("caller error set (%d)" % code)
timed("encode 1 GiB, caller error pending", lambda: p.encode_stripes(buf))
timed("decode 1 GiB, caller error pending", lambda: p.decode_stripes(buf, [0]))
print(json.dumps({"step": "read", "got": hip.hipGetLastError(), "want": code}), flush=True)
timed("encode 1 GiB, slot clear", lambda: p.encode_stripes(buf))
