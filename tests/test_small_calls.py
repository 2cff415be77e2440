"""The small-call path LStore uses: plan->encode_block / plan->decode_block once per stripe from
many pool threads (segment/jerasure.c:1847, :245, :1937).  Such calls are served zero-copy by
the stripe server (ec_server.hip): the calling thread posts column parts of its stripe to a
persistent kernel through page-locked slots, or names its own page-locked chunks.  Checked
bit-exactly against the oracle from many threads at once, across the server's idle retirement
and relaunch, with ragged chunk sizes, and across plans whose coefficient images reuse device
addresses while the server runs.
"""
import json
import os
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

import lstore_amd as L
import oracle as O

pytestmark = pytest.mark.gpu


def _pinned(shape):
    import torch

    return torch.empty(shape, dtype=torch.uint8, pin_memory=True).numpy()


GEOS = [(L.REED_SOL_VAN, 6, 3, 16384), (L.CAUCHY_GOOD, 6, 3, 16384), (L.REED_SOL_VAN, 10, 4, 8200),
        (L.CAUCHY_GOOD, 10, 4, 65536), (L.REED_SOL_VAN, 20, 6, 4096), (L.CAUCHY_ORIG, 4, 2, 2048),
        (L.REED_SOL_R6_OP, 6, 2, 24576), (L.RAID4, 6, 1, 16384)]


@pytest.mark.parametrize("method,k,m,C", GEOS)
def test_single_calls_match_oracle(cuda, method, k, m, C):
    with L.Plan.for_chunk(method, k, m, C) as p:
        rng = np.random.default_rng(C + k)
        R = 2 if method == L.REED_SOL_R6_OP else (1 if method == L.RAID4 else m)
        for pinned in (False, True):
            sh = _pinned((k + m, C)) if pinned else np.empty((k + m, C), np.uint8)
            for it in range(4):
                sh[:k] = rng.integers(0, 256, (k, C), dtype=np.uint8)
                sh[k:] = 0x77
                p.encode_block([sh[i] for i in range(k + m)])
                want = O.encode(method, np.ascontiguousarray(sh[:k]), m, p.packet_size)
                assert np.array_equal(sh[k:k + R], want[:R]), (pinned, it)
                full = sh.copy()
                lost = [it % k] if method == L.RAID4 else sorted({it % (k + m), (it * 5 + 1) % (k + m)})[:m]
                sh[lost] = 0xEE
                assert p.decode_block([sh[i] for i in range(k + m)], lost) == 0
                assert np.array_equal(sh, full), (pinned, it, lost)


def test_many_threads_mixed_plans_and_idle_gaps(cuda):
    """32 threads over four plans, pageable and page-locked buffers, with pauses longer than the
    server's 2 ms idle retirement so it is relaunched while others are mid-call."""
    plans = [L.Plan.for_chunk(mth, k, m, C) for mth, k, m, C in GEOS[:4]]
    errors = []

    def worker(t):
        try:
            rng = np.random.default_rng(1000 + t)
            p = plans[t % len(plans)]
            mth, k, m, C = GEOS[t % len(plans)]
            sh = _pinned((k + m, C)) if t % 3 == 0 else np.empty((k + m, C), np.uint8)
            for it in range(12):
                sh[:k] = rng.integers(0, 256, (k, C), dtype=np.uint8)
                p.encode_block([sh[i] for i in range(k + m)])
                if not np.array_equal(sh[k:], O.encode(mth, np.ascontiguousarray(sh[:k]), m, p.packet_size)):
                    errors.append((t, it, "encode"))
                full = sh.copy()
                lost = [(t + it) % (k + m)]
                sh[lost] = 0
                if p.decode_block([sh[i] for i in range(k + m)], lost) != 0 or not np.array_equal(sh, full):
                    errors.append((t, it, "decode"))
                if it % 4 == 3:
                    time.sleep(0.004 + 0.001 * (t % 3))
        except Exception as ex:  # noqa: BLE001
            errors.append((t, repr(ex)))

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(32)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    for p in plans:
        p.close()
    assert not errors, errors[:8]


def test_new_plans_while_the_server_runs(cuda):
    """Plans are destroyed and created while the server keeps running: a new plan's coefficient
    image may take a destroyed one's device address, and the server must read the new cells."""
    C = 16384
    rng = np.random.default_rng(5)
    for round_ in range(12):
        method, k, m = [(L.REED_SOL_VAN, 6, 3), (L.CAUCHY_GOOD, 6, 3), (L.REED_SOL_VAN, 4, 2)][round_ % 3]
        with L.Plan.for_chunk(method, k, m, C) as p:
            sh = np.empty((k + m, C), np.uint8)
            sh[:k] = rng.integers(0, 256, (k, C), dtype=np.uint8)
            p.encode_block([sh[i] for i in range(k + m)])
            assert np.array_equal(sh[k:], O.encode(method, np.ascontiguousarray(sh[:k]), m, p.packet_size)), round_


def test_server_timeout_leaves_no_late_writes(cuda):
    """A call whose parts the stripe server does not answer in time (the test hook holds every
    post) stops the server, cancels its parts and takes its own launch.  Nothing may serve those
    parts after the call has returned: the caller's page-locked chunks are served in place, so a
    late serve would write stale parity into buffers the caller has already reused."""
    import ctypes as C

    lib = L.lib()
    lib.lsec_test_server_hold.restype = C.c_longlong
    lib.lsec_test_server_hold.argtypes = [C.c_int, C.c_int]
    method, k, m, C_ = L.REED_SOL_VAN, 6, 3, 16384
    rng = np.random.default_rng(77)
    with L.Plan.for_chunk(method, k, m, C_) as p:
        t0 = lib.lsec_test_server_hold(1, 200)
        try:
            held = [_pinned((k + m, C_)), np.empty((k + m, C_), np.uint8)]
            for sh in held:
                sh[:k] = rng.integers(0, 256, (k, C_), dtype=np.uint8)
                sh[k:] = 0
                start = time.perf_counter()
                p.encode_block([sh[i] for i in range(k + m)])
                assert time.perf_counter() - start >= 0.15  # it waited for the held server
                assert np.array_equal(sh[k:], O.encode(method, np.ascontiguousarray(sh[:k]), m, p.packet_size))
                full = sh.copy()
                sh[1] = 0xEE
                assert p.decode_block([sh[i] for i in range(k + m)], [1]) == 0
                assert np.array_equal(sh, full)
            assert lib.lsec_test_server_hold(-1, 0) - t0 >= 4  # every call above timed out
        finally:
            lib.lsec_test_server_hold(0, 5000)
        # the caller reuses its buffers; the server now serves again (other calls relaunch it)
        for sh in held:
            sh[:] = 0xA5
        snap = [sh.copy() for sh in held]
        other = np.empty((k + m, C_), np.uint8)
        for it in range(20):
            other[:k] = rng.integers(0, 256, (k, C_), dtype=np.uint8)
            p.encode_block([other[i] for i in range(k + m)])
            assert np.array_equal(other[k:], O.encode(method, np.ascontiguousarray(other[:k]), m, p.packet_size))
            time.sleep(0.001 if it % 5 else 0.005)  # across idle retirements and relaunches
        time.sleep(0.05)
        for sh, want in zip(held, snap):
            assert np.array_equal(sh, want), "a cancelled part was served after its call returned"


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "build", "fnptr_bench")
REF = os.path.join(ROOT, "oracle", "_ref", "libjerasure_ref.so")


@pytest.mark.skipif(not (os.path.exists(BENCH) and os.path.exists(REF)), reason="build/fnptr_bench or oracle/_ref not built")
@pytest.mark.parametrize("chunk,threads,method,op,pinned,extra", [
    (16384, 128, "reed_sol_van", "encode", 0, {}), (16384, 128, "cauchy_good", "decode", 0, {}),
    (65536, 64, "cauchy_good", "encode", 1, {}), (1 << 20, 16, "reed_sol_van", "encode", 0, {}),
    (262144, 32, "reed_sol_van", "decode", 0, {"LSEC_ZC_SLOTS_MB": "4"}),
    # LStore's buffer lifetime: each call's parity / stripe buffer malloc'd for the call and freed
    # right after it (segment/jerasure.c:1689-1697, :1882, :1621); =2 makes every buffer a fresh
    # mmap and every free an munmap, so the next buffer reuses just-unmapped addresses
    (1 << 20, 2, "reed_sol_van", "encode", 0, {"FNPTR_FREE_AFTER": "2"}),
    (1 << 20, 4, "cauchy_good", "decode", 0, {"FNPTR_FREE_AFTER": "2"}),
    (1 << 20, 3, "cauchy_good", "decode", 0, {"FNPTR_FREE_AFTER": "1"}),
    (4 << 20, 2, "reed_sol_van", "encode", 0, {"FNPTR_FREE_AFTER": "1"})])
def test_fn_pointer_stress_bit_exact(cuda, chunk, threads, method, op, pinned, extra):
    """LStore's pattern in C (tools/fnptr_bench.c, FNPTR_VERIFY=1): every thread calls
    encode_block / decode_block on its own stripe for 1 s; before each call the chunks it must
    write are overwritten, after it they must equal the reference's (oracle/_ref) -- every
    call checked, at up to 128 threads (server slots, parking, one pointer query per call; the
    last case's zero-copy slots hit their page-locked budget and calls fall to the dispatcher)."""
    env = dict(os.environ, FNPTR_VERIFY="1", FNPTR_REF=REF, FNPTR_PINNED=str(pinned), **extra)
    out = subprocess.run([BENCH, str(chunk), str(threads), "1", method, op], env=env, capture_output=True,
                         text=True, timeout=100)
    assert out.returncode == 0, (out.returncode, out.stdout[-500:], out.stderr[-500:])
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    assert rec["verified"] > 0 and rec["mismatches"] == 0, rec


@pytest.mark.skipif(not (os.path.exists(BENCH) and os.path.exists(REF)), reason="build/fnptr_bench or oracle/_ref not built")
def test_inplace_stall_guard_under_mmap_churn(cuda):
    """Per-stripe 1 MiB decodes at two threads whose buffers are each a fresh mmap, munmapped right
    after the call (FNPTR_FREE_AFTER=2): DMA from pages pinned in place stalls ~25 ms a call there
    (profiles/r06_v2_free_after_churn.jsonl).  The stall guard (ec_engine.h) sees the stalls,
    suspends in-place pinning and the calls pack: every call bit-exact, and the median call back
    under a few milliseconds."""
    env = dict(os.environ, FNPTR_VERIFY="1", FNPTR_REF=REF, FNPTR_FREE_AFTER="2")
    out = subprocess.run([BENCH, str(1 << 20), "2", "3", "cauchy_good", "decode"], env=env, capture_output=True, text=True,
                         timeout=100)
    assert out.returncode == 0, (out.returncode, out.stdout[-500:], out.stderr[-500:])
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    assert rec["verified"] > 100 and rec["mismatches"] == 0, rec
    assert rec["per_call_us_p50"] < 3000, (rec, out.stderr[-500:])


STRESS = os.path.join(ROOT, "tools", "reg_stress.py")


@pytest.mark.parametrize("args", [
    ["--k", "6", "--m", "3", "--w", "16", "--chunk", "49192"],
    ["--method", "cauchy_good", "--k", "6", "--m", "3", "--chunk", "65536", "--stripes", "1"],
    ["--k", "6", "--m", "3", "--chunk", "1048576", "--stripes", "4"],
    ["--method", "cauchy_good", "--k", "6", "--m", "3", "--chunk", "65536", "--stripes", "2", "--pinned"],
    ["--method", "cauchy_good", "--k", "6", "--m", "3", "--chunk", "65536", "--stripes", "1", "--caller-registered"],
    ["--k", "6", "--m", "3", "--chunk", "65536", "--stripes", "8", "--caller-registered"],
])
def test_host_calls_under_memory_churn(cuda, args):
    """Host calls while the process frees and reallocates host memory between them (virtual
    ranges and physical pages recycled; tools/reg_stress.py --churn), with stripe-server calls in
    between: the zero-copy slots and server, the in-place-pinned DMA pipeline (36 MiB batches) and
    caller page-locked buffers reallocated every call, and caller-registered buffers (the caller
    hipHostRegister's each iteration's stripes and unregisters them after, as an allocator that pins
    its arenas).  Every call's bytes are checked against the oracle restatement.  (Kernels over per-call registrations of pageable pages failed exactly this,
    which is why no route uses them: DESIGN.md §1.)"""
    out = subprocess.run([sys.executable, STRESS, "--seconds", "5", "--churn", "--small-mix", *args],
                         capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, (out.stdout[-500:], out.stderr[-800:])
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    assert rec["iters"] > 10 and rec["bad_encode"] == 0 and rec["bad_decode"] == 0 and rec["bad_small"] == 0, rec


STALE_ERROR_SCRIPT = r"""
import ctypes, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import lstore_amd as L
import oracle as O
hip = ctypes.CDLL("libamdhip64.so")
junk = np.zeros(1 << 16, np.uint8)
rng = np.random.default_rng(3)


def pageable(n):
    return np.zeros(n, np.uint8), None


def registered(n):
    # the caller's own registration of its arena (DMA only inside the engine; telling it from
    # hipHostMalloc memory takes a query that fails for registered ranges)
    a = np.zeros(n + 4096, np.uint8)
    off = (-a.ctypes.data) % 4096
    a = a[off:off + n]
    assert hip.hipHostRegister(ctypes.c_void_p(a.ctypes.data), ctypes.c_size_t(n), 0) == 0
    return a, lambda: hip.hipHostUnregister(ctypes.c_void_p(a.ctypes.data))


def hostmalloc(n):
    p = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(n), 0) == 0
    a = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(p.value))
    return a, lambda: hip.hipHostFree(p)


for kind in (pageable, registered, hostmalloc):
    for C in (65536, 1 << 20):
        p = L.Plan.for_chunk(L.CAUCHY_GOOD, 6, 3, C)
        p.prepare_encode()
        p.prepare_decode([0])
        arena, free = kind(9 * C)
        d = arena.reshape(9, C)
        for _ in range(4):
            d[:6] = rng.integers(0, 256, (6, C), dtype=np.uint8)
            d[6:] = 0
            # an unregister of memory that was never registered fails and leaves its error in this
            # thread's HIP last-error slot, as the caller's own HIP calls can
            code = hip.hipHostUnregister(ctypes.c_void_p(junk.ctypes.data))
            assert code != 0
            p.encode_block([d[j] for j in range(9)])
            assert np.array_equal(d[6:], O.encode(L.CAUCHY_GOOD, d[:6], 3, p.packet_size)), (kind.__name__, C)
            # ... and exactly the caller's error is still there for the caller to read
            got = hip.hipGetLastError()
            assert got == code, (kind.__name__, C, "encode", got, code)
            want = d[0].copy()
            d[0] = 0
            code = hip.hipHostUnregister(ctypes.c_void_p(junk.ctypes.data))
            assert p.decode_block([d[j] for j in range(9)], [0]) == 0
            assert np.array_equal(d[0], want), (kind.__name__, C)
            got = hip.hipGetLastError()
            assert got == code, (kind.__name__, C, "decode", got, code)
        if free:
            # the caller's own release still works: the engine never re-registered (and so, at the
            # end of its call, unregistered) the caller's page-locked arena
            rc = free()
            assert rc == 0, (kind.__name__, C, "caller's release failed", rc)
        p.close()
print("ok")
"""


@pytest.mark.gpu
def test_stale_caller_hip_error_is_not_taken_for_a_launch_failure(cuda):
    """A HIP error the caller's own calls left pending (HIP keeps the last error per thread until
    it is read) must neither fail the engine's next launch nor be consumed by it: launches report
    hipLaunchKernel's own status (lsec::launch_kernel), and the engine never reads the last error
    to learn about them.  (Round 3 saw tools/reg_stress.py --caller-registered fail a 1 MiB call
    with the caller's hipHostUnregister error; its fix, clearing the error at every entry point,
    hid the caller's error from the caller: ADVICE r03.)  Served (64 KiB) and own-launch (1 MiB,
    9 MiB per call) stripes, bit-exact, with no retry, and the caller's error still pending."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", STALE_ERROR_SCRIPT, root], capture_output=True, text=True,
                         timeout=110)
    assert out.returncode == 0 and out.stdout.strip().endswith("ok"), (out.stdout[-500:], out.stderr[-800:])
    assert "retried with direct copies" not in out.stderr, out.stderr[-800:]


UNPIN_SCRIPT = r"""
import ctypes, sys, threading
import numpy as np
sys.path.insert(0, sys.argv[1])
import lstore_amd as L
from lstore_amd import erasure as E
import oracle as O
hip = ctypes.CDLL("libamdhip64.so")
k, m, C = 6, 3, 1 << 20
plan = L.Plan.for_chunk(L.CAUCHY_GOOD, k, m, C)
plan.prepare_encode()
plan.prepare_decode([0])
errors, arenas = [], []
lock = threading.Lock()


def worker(t):
    rng = np.random.default_rng(t)
    try:
        for it in range(30):
            # a fresh page-aligned pageable stripe per call, pinned in place by the call
            a = np.zeros(9 * C + 4096, np.uint8)
            off = (-a.ctypes.data) % 4096
            d = a[off:off + 9 * C].reshape(9, C)
            d[:k] = rng.integers(0, 256, (k, C), dtype=np.uint8)
            plan.encode_block([d[j] for j in range(9)])
            if not np.array_equal(d[k:], O.encode(L.CAUCHY_GOOD, d[:k], m, plan.packet_size)):
                errors.append((t, it, "encode"))
            want = d[0].copy()
            d[0] = 0
            plan.decode_block([d[j] for j in range(9)], [0])
            if not np.array_equal(d[0], want):
                errors.append((t, it, "decode"))
            with lock:
                arenas.append(d)
    except Exception as e:
        errors.append((t, repr(e)))


th = [threading.Thread(target=worker, args=(t,)) for t in range(3)]
for x in th:
    x.start()
for x in th:
    x.join()
assert not errors, errors[:5]
# every registration a call left to the background unpinner is gone after the drain: the caller
# can now register (and release) any of those ranges itself
E.host_unpin_drain()
for d in arenas[-24:]:
    p, n = ctypes.c_void_p(d.ctypes.data), ctypes.c_size_t(d.nbytes)
    assert hip.hipHostRegister(p, n, 0) == 0
    assert hip.hipHostUnregister(p) == 0
print("ok", len(arenas))
"""


def test_background_unpinner_and_drain(cuda):
    """The opt-in background unpinner (LSEC_DEFER_UNPIN_MB > 0; off by default).  Three threads of
    per-stripe 1 MiB calls on fresh pageable stripes (pinned in place; with other calls in flight,
    each call's registration is dropped by the background unpinner after it returns,
    ec_pinning.cpp): every result equals the oracle's, and after lsec_host_unpin_drain() the caller
    can register and release those ranges itself (INTEGRATION.md "Host buffers")."""
    out = subprocess.run([sys.executable, "-c", UNPIN_SCRIPT, ROOT], capture_output=True, text=True, timeout=110,
                         env=dict(os.environ, LSEC_DEFER_UNPIN_MB="256"))
    assert out.returncode == 0, (out.stdout[-500:], out.stderr[-1500:])
    assert out.stdout.strip().startswith("ok"), out.stdout[-300:]


FREE_AFTER_SCRIPT = r"""
import ctypes, json, sys, threading
import numpy as np
sys.path.insert(0, sys.argv[1])
mode = sys.argv[2]
import torch
import lstore_amd as L
import oracle as O
hip = ctypes.CDLL("libamdhip64.so")
libc = ctypes.CDLL(None, use_errno=True)
libc.mmap.restype = ctypes.c_void_p
libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
PROT_RW, MAP_PRIVATE_ANON, MAP_FIXED_NOREPLACE = 0x3, 0x22, 0x100000
MAP_FAILED = ctypes.c_void_p(-1).value


class Attr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


hip.hipPointerGetAttributes.argtypes = [ctypes.POINTER(Attr), ctypes.c_void_p]
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]


def registered(addr, n):
    # page-locked with HIP at either end of [addr, addr + n)?  (a failed query leaves an error in
    # this thread's last-error slot: read it, so torch's next launch check does not take it)
    for a in (addr, addr + n - 1):
        at = Attr()
        rc = hip.hipPointerGetAttributes(ctypes.byref(at), ctypes.c_void_p(a))
        if rc != 0:
            hip.hipGetLastError()
        elif at.type != 0:
            return True
    return False


def fresh(n, hint=None):
    p = libc.mmap(hint, n, PROT_RW, MAP_PRIVATE_ANON | (MAP_FIXED_NOREPLACE if hint else 0), -1, 0)
    return None if p in (None, MAP_FAILED) else p


def view(addr, n):
    return np.frombuffer((ctypes.c_uint8 * n).from_address(addr), dtype=np.uint8)


k, m, C = 6, 3, 1 << 20
S = (k + m) * C
plan = L.Plan.for_chunk(L.REED_SOL_VAN, k, m, C)
plan.prepare_encode()
plan.prepare_decode([0])
dev = torch.empty(S, dtype=torch.uint8, device="cuda")
stats = dict(calls=0, still_registered=0, reused_address=0, copies_checked=0, bad=[])
lock = threading.Lock()


def worker(t):
    rng = np.random.default_rng(100 + t)
    devt = torch.empty(S, dtype=torch.uint8, device="cuda")
    try:
        for it in range(24):
            a = fresh(S)
            d = view(a, S).reshape(k + m, C)
            d[:k] = rng.integers(0, 256, (k, C), dtype=np.uint8)
            want_p = O.encode(L.REED_SOL_VAN, np.ascontiguousarray(d[:k]), m, plan.packet_size)
            plan.encode_block([d[j] for j in range(k + m)])
            reg = registered(a, S)  # right after the call returned, other threads' calls in flight
            ok = np.array_equal(d[k:], want_p)
            want0 = d[0].copy()
            d[0] = 0
            plan.decode_block([d[j] for j in range(k + m)], [0])
            reg = registered(a, S) or reg
            ok = ok and np.array_equal(d[0], want0)
            with lock:
                stats["calls"] += 2
                stats["still_registered"] += int(reg)
                if not ok:
                    stats["bad"].append((t, it, "coding"))
            if mode == "optin":
                # count only: with the opt-in a registration may still be pending here, and a copy
                # from a recycled range under it is the hazard the default avoids
                libc.munmap(a, S)
                continue
            # LStore's pattern: free the buffer right after the op (segment/jerasure.c:1882), and
            # the next allocation lands at the same addresses
            libc.munmap(a, S)
            b = fresh(S, a) or fresh(S)
            with lock:
                stats["reused_address"] += int(b == a)
            y = view(b, S)
            y[:] = rng.integers(0, 256, S, dtype=np.uint8)
            # another HIP user of the process copies the new buffer: torch, and a plain hipMemcpy
            got = torch.from_numpy(y).cuda().cpu().numpy()
            good = np.array_equal(got, y)
            if hip.hipMemcpy(ctypes.c_void_p(devt.data_ptr()), ctypes.c_void_p(b), S, 1) != 0:
                good = False
            good = good and np.array_equal(devt.cpu().numpy(), y)
            with lock:
                stats["copies_checked"] += 2
                if not good:
                    stats["bad"].append((t, it, "copy of a recycled range", b == a))
            libc.munmap(b, S)
    except Exception as e:
        with lock:
            stats["bad"].append((t, repr(e)))


th = [threading.Thread(target=worker, args=(t,)) for t in range(3)]
for x in th:
    x.start()
for x in th:
    x.join()
print(json.dumps(stats))
"""


def _free_after(mode, extra_env=None):
    env = dict(os.environ, **(extra_env or {}))
    out = subprocess.run([sys.executable, "-c", FREE_AFTER_SCRIPT, ROOT, mode], capture_output=True, text=True,
                         timeout=110, env=env)
    assert out.returncode == 0, (out.stdout[-500:], out.stderr[-1500:])
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_no_registration_outlives_its_call(cuda):
    """LStore frees a call's buffers right after the op (the parity buffer, segment/jerasure.c:1689-1697
    and :1882; the read path's stripe buffer, :1621), and the allocator may hand the same addresses
    out again at once.  Three threads of 1 MiB per-stripe calls on freshly mmap'd stripes (pinned in
    place for the call), each munmap'd right after its call, with the next mmap asked for the same
    addresses; another HIP user of the process (torch's .cuda(), a plain hipMemcpy) then copies the
    new bytes.  With the default (LSEC_DEFER_UNPIN_MB=0) no range the engine registered is still
    registered when its call returns -- even while the other threads' calls are in flight -- so the
    copies see the new pages; every coding result is bit-exact."""
    st = _free_after("default", {"LSEC_DEFER_UNPIN_MB": "0"})
    assert st["calls"] == 144 and not st["bad"], st
    assert st["still_registered"] == 0, st
    assert st["copies_checked"] == 144 and st["reused_address"] > 0, st


def test_large_calls_progress_beside_back_to_back_small_calls(cuda):
    """An LStore process serving segments of different chunk sizes: two threads make back-to-back
    16 KiB decodes (the stripe server stays resident) while a third makes 1 MiB decodes, which pin
    their chunks in place and release them with hipHostUnregister -- a call that waits until the
    device is idle.  The releases stop the server and hold off its relaunch while they run
    (servers_yield_begin, ec_stripe_server.cpp); before that the 1 MiB calls made no progress at
    all until the small calls stopped (tools/probes/mixed_sizes_probe.c).  Every output checked."""
    k, m = 6, 3
    stop = threading.Event()
    errors, small_calls, large_lat = [], [0, 0], []

    def worker(C, idx):
        with L.Plan.for_chunk(L.CAUCHY_GOOD, k, m, C) as p:
            rng = np.random.default_rng(C + idx)
            sh = [rng.integers(0, 256, C, dtype=np.uint8) for _ in range(k)] + [np.zeros(C, np.uint8) for _ in range(m)]
            p.encode_block(sh)
            want = sh[0].copy()
            while not stop.is_set():
                sh[0][:] = 0xA5
                t0 = time.perf_counter()
                rc = p.decode_block(sh, [0])
                dt = time.perf_counter() - t0
                if rc != 0 or not np.array_equal(sh[0], want):
                    errors.append((C, rc))
                    return
                if C > 65536:
                    large_lat.append(dt)
                else:
                    small_calls[idx] += 1

    th = [threading.Thread(target=worker, args=(16384, i)) for i in range(2)]
    for t in th:
        t.start()
    time.sleep(0.3)  # the small calls run (and the server with them) before the large ones start
    big = threading.Thread(target=worker, args=(1 << 20, 0))
    big.start()
    time.sleep(2.5)
    stop.set()
    for t in th + [big]:
        t.join(timeout=60)
    assert not errors, errors
    assert sum(small_calls) > 1000, small_calls
    # a 1 MiB decode alone takes ~0.2 ms; starved, not one finished before the small calls stopped
    assert len(large_lat) >= 50, (len(large_lat), small_calls)
    assert max(large_lat) < 1.0, max(large_lat)
