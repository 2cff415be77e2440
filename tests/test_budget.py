"""CPU test of the zero-copy page-locked accounting (ec_engine.h PinnedBudget): each device's
stripe server region (~93 MiB) is accounted apart from the per-thread zero-copy slots, whose
budget (LSEC_ZC_SLOTS_MB) applies per device -- so with the in-process device set spread over
8 GPUs (lsec_set_host_devices), a device's threads get the same slot budget as with one GPU
(VERDICT r03 "multi-device accounting"; SURVEY §8e: per GPU its own pinned staging).  No GPU
is needed: the hook runs the accounting on a fresh instance."""
import ctypes

import pytest

from lstore_amd import erasure as E


def _lib():
    lib = E.lib()
    lib.lsec_test_pinned_budget.argtypes = [ctypes.c_int, ctypes.c_longlong, ctypes.c_longlong,
                                            ctypes.POINTER(ctypes.c_longlong)]
    lib.lsec_test_pinned_budget.restype = ctypes.c_longlong
    return lib


@pytest.mark.parametrize("budget_mb,slot_mb", [(1024, 9), (1024, 1), (4, 1)])
def test_slot_budget_is_per_device_and_servers_do_not_shrink_it(built, budget_mb, slot_mb):
    lib = _lib()
    got = {}
    for ndev in (1, 2, 8):
        srv = ctypes.c_longlong(0)
        got[ndev] = lib.lsec_test_pinned_budget(ndev, budget_mb, slot_mb, ctypes.byref(srv))
        assert got[ndev] >= 0, E.last_error()
        assert srv.value == ndev * 93, srv.value  # 992 slots x 96 KiB per device's server
    assert got[1] == got[2] == got[8] == budget_mb // slot_mb, got


def test_pinned_budget_hook_rejects_bad_arguments(built):
    assert _lib().lsec_test_pinned_budget(0, 1024, 1, None) == -1
    assert "bad arguments" in E.last_error()
