#!/usr/bin/env python3
"""LStore's free-after-op buffer lifetime (segment/jerasure.c:1689-1697, :1882, :1621) against the
engine's in-place registrations, as tests/test_small_calls.py::test_no_registration_outlives_its_call
runs it, with its counters printed (one JSON line per mode):
  default  LSEC_DEFER_UNPIN_MB=0: after every call, is its range still registered?  then munmap, a
           new mmap at the same addresses, and two copies of the new bytes by other HIP users
           (torch .cuda(), hipMemcpy), checked;
  optin    LSEC_DEFER_UNPIN_MB=256 (the opt-in background unpinner): counts only how many calls
           returned with their range still registered -- the window the opt-in leaves -- and does
           no copy from a recycled range under it.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from test_small_calls import FREE_AFTER_SCRIPT  # noqa: E402

for mode, mb in (("default", "0"), ("optin", "256")):
    out = subprocess.run([sys.executable, "-c", FREE_AFTER_SCRIPT, ROOT, mode], capture_output=True, text=True,
                         timeout=110, env=dict(os.environ, LSEC_DEFER_UNPIN_MB=mb))
    if out.returncode != 0:
        print(json.dumps({"mode": mode, "rc": out.returncode, "stderr": out.stderr[-1500:]}))
        sys.exit(1)
    st = json.loads(out.stdout.strip().splitlines()[-1])
    print(json.dumps({"mode": mode, "LSEC_DEFER_UNPIN_MB": mb, **st}), flush=True)
