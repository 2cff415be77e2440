"""NUMA placement of a device's engine threads (per GPU its own host thread and
NUMA-local staging): PCI bus id -> <sysfs>/bus/pci/devices/<id>/numa_node -> the node's cpulist,
checked against a fake sysfs tree (no GPU needed)."""
import os

import pytest

from lstore_amd import erasure as E


def _tree(tmp_path, devices, nodes):
    for bus, node in devices.items():
        d = tmp_path / "bus" / "pci" / "devices" / bus
        d.mkdir(parents=True)
        (d / "numa_node").write_text(f"{node}\n")
    for node, cpulist in nodes.items():
        d = tmp_path / "devices" / "system" / "node" / f"node{node}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cpulist + "\n")
    return str(tmp_path)


def test_bus_to_node_to_cpus(tmp_path):
    root = _tree(tmp_path, {"0000:05:00.0": 0, "0000:c1:00.0": 1, "0000:75:00.0": -1},
                 {0: "0-3,8-9", 1: "4-7,10-11,64", 2: "12-15"})
    assert E.numa_for_bus(root, "0000:05:00.0") == (0, [0, 1, 2, 3, 8, 9])
    # hipDeviceGetPCIBusId may report upper-case hex digits; sysfs names are lower case
    assert E.numa_for_bus(root, "0000:C1:00.0") == (1, [4, 5, 6, 7, 10, 11, 64])
    # firmware without affinity (numa_node -1), an unknown function: no placement, no pinning
    assert E.numa_for_bus(root, "0000:75:00.0") == (-1, [])
    assert E.numa_for_bus(root, "0000:99:00.0") == (-1, [])


def test_cpulist_forms(tmp_path):
    root = _tree(tmp_path, {"0000:01:00.0": 3}, {3: " 0 , 2-4,7-7,, 9-8,x,11"})
    # malformed pieces (reversed range, garbage) are skipped, the rest parsed and deduplicated
    assert E.numa_for_bus(root, "0000:01:00.0") == (3, [0, 2, 3, 4, 7, 11])


def test_missing_cpulist_means_no_placement(tmp_path):
    root = _tree(tmp_path, {"0000:02:00.0": 5}, {})
    assert E.numa_for_bus(root, "0000:02:00.0") == (-1, [])


def test_this_host_devices_if_any():
    """On a GPU box every device's placement names CPUs this process may use (or none)."""
    n = E.lib().lsec_device_count()
    if n == 0:
        with pytest.raises(E.ErasureError):
            E.device_numa(0)
        return
    allowed = os.sched_getaffinity(0)
    for d in range(n):
        node, cpus = E.device_numa(d)
        assert set(cpus) <= allowed
        assert (node >= 0) or not cpus
