"""runtime/device.py + runtime/launch.py: the rank -> GPU -> NUMA -> CPU plan read from a fake sysfs tree, and the
affinity each launched rank actually runs with (CPU only)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_pytorch_hpc_amd.runtime import device  # noqa: E402


def fake_sysfs(tmp, layout, extra_cards=()):
    """layout: list of (numa_node, cpulist) per GPU in PCI order; also a non-AMD card and a render alias."""
    root = tmp / "sys"
    for i, (node, cpus) in enumerate(layout):
        bdf = f"0000:{0x05 + 0x10 * i:02x}:00.0"
        dev = root / "bus" / "pci" / "devices" / bdf
        dev.mkdir(parents=True)
        (dev / "vendor").write_text("0x1002\n")
        (dev / "class").write_text("0x120000\n")
        (dev / "numa_node").write_text(f"{node}\n")
        (dev / "local_cpulist").write_text(cpus + "\n")
        card = root / "class" / "drm" / f"card{len(layout) - 1 - i}"   # card numbering NOT in PCI order
        card.mkdir(parents=True)
        (card / "device").symlink_to(dev)
    for name, vendor in extra_cards:
        dev = root / "bus" / "pci" / "devices" / name
        dev.mkdir(parents=True)
        (dev / "vendor").write_text(vendor + "\n")
        (dev / "class").write_text("0x030000\n")
        (dev / "numa_node").write_text("0\n")
        card = root / "class" / "drm" / f"card{90 + len(list((root / 'class' / 'drm').iterdir()))}"
        card.mkdir(parents=True)
        (card / "device").symlink_to(dev)
    return str(root)


TWO_SOCKET = [(0, "0-3")] * 4 + [(1, "4-7")] * 4


def test_parse_cpulist():
    assert device.parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    assert device.parse_cpulist("") == []


def test_gpus_in_pci_order_and_filtered(tmp_path):
    root = fake_sysfs(tmp_path, TWO_SOCKET, extra_cards=[("0000:ff:00.0", "0x1a03")])   # an ASPEED BMC display
    g = device.gpus(root)
    assert [x.numa_node for x in g] == [0, 0, 0, 0, 1, 1, 1, 1]
    assert [x.bdf for x in g] == sorted(x.bdf for x in g)
    assert g[5].local_cpus == [4, 5, 6, 7]


def test_plan_splits_node_cores(tmp_path):
    root = fake_sysfs(tmp_path, TWO_SOCKET)
    b = device.plan(8, sysfs=root, env={}, allowed=list(range(8)))
    assert [x.cpus for x in b] == [[i] for i in range(8)]
    assert [x.numa_node for x in b] == [0] * 4 + [1] * 4
    assert all(x.omp_threads == 1 for x in b)
    # 4 ranks on a 16-core box: GPUs 0-3 are all on node 0 -> its cores split 4 ways
    root2 = fake_sysfs(tmp_path / "b", [(0, "0-7")] * 4 + [(1, "8-15")] * 4)
    b = device.plan(4, sysfs=root2, env={}, allowed=list(range(16)))
    assert [x.cpus for x in b] == [[0, 1], [2, 3], [4, 5], [6, 7]]
    # disjoint, and within the launcher's own affinity
    b = device.plan(2, sysfs=root2, env={}, allowed=[0, 1, 2, 8, 9])
    assert b[0].cpus == [0] and b[1].cpus == [1, 2]


def test_plan_honours_visible_devices(tmp_path):
    root = fake_sysfs(tmp_path, TWO_SOCKET)
    b = device.plan(2, sysfs=root, env={"HIP_VISIBLE_DEVICES": "6,1"}, allowed=list(range(8)))
    assert [x.gpu for x in b] == [6, 1] and [x.numa_node for x in b] == [1, 0]
    assert b[0].cpus == [4, 5, 6, 7] and b[1].cpus == [0, 1, 2, 3]


def test_plan_without_topology(tmp_path):
    b = device.plan(4, sysfs=str(tmp_path / "none"), env={}, allowed=list(range(8)))
    assert all(x.cpus == [] and x.omp_threads == 2 for x in b)


@pytest.mark.skipif(len(os.sched_getaffinity(0)) < 8, reason="needs 8 CPUs in the affinity mask")
def test_launcher_pins_each_rank(tmp_path):
    root = fake_sysfs(tmp_path, TWO_SOCKET)
    allowed = sorted(os.sched_getaffinity(0))[:8]
    # remap the fake tree onto the CPUs this container actually has
    for i, g in enumerate(device.gpus(root)):
        cpus = allowed[:4] if i < 4 else allowed[4:8]
        with open(os.path.join(root, "bus", "pci", "devices", g.bdf, "local_cpulist"), "w") as fh:
            fh.write(",".join(map(str, cpus)))
    script = tmp_path / "child.py"
    script.write_text("import os, json\n"
                      "print(json.dumps({'rank': int(os.environ['RANK']), 'aff': sorted(os.sched_getaffinity(0)),"
                      " 'omp': os.environ.get('OMP_NUM_THREADS'), 'numa': os.environ.get('DPH_NUMA_NODE')}))\n")
    env = {k: v for k, v in os.environ.items() if k not in ("OMP_NUM_THREADS", "HIP_VISIBLE_DEVICES",
                                                            "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")}
    env.update(DPH_SYSFS_ROOT=root, PYTHONPATH=ROOT)
    logs = tmp_path / "logs"
    p = subprocess.run([sys.executable, "-m", "distributed_pytorch_hpc_amd.runtime.launch", "--nproc", "8",
                        "--log-dir", str(logs), str(script)], env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert "rank 7 -> GPU 7 -> NUMA 1" in p.stderr
    for r in range(8):
        out = json.loads((logs / f"rank{r}.out").read_text().strip().splitlines()[-1])
        assert out["aff"] == [allowed[r]], out
        assert out["omp"] == "1" and out["numa"] == str(0 if r < 4 else 1)
    # --cpu-bind none leaves every rank with the launcher's affinity
    p = subprocess.run([sys.executable, "-m", "distributed_pytorch_hpc_amd.runtime.launch", "--nproc", "2",
                        "--cpu-bind", "none", "--log-dir", str(tmp_path / "l2"), str(script)], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    out = json.loads((tmp_path / "l2" / "rank1.out").read_text().strip().splitlines()[-1])
    assert out["aff"] == sorted(os.sched_getaffinity(0))


def test_plan_skips_cards_whose_render_node_is_not_exposed(tmp_path):
    """A container given GPUs 2 and 5 of 8 through device cgroups (no *_VISIBLE_DEVICES): sysfs lists all eight,
    /dev/dri holds only two render nodes, and HIP's ordinals 0 / 1 are those two cards."""
    root = fake_sysfs(tmp_path, TWO_SOCKET)
    drm = os.path.join(root, "class", "drm")
    cards = sorted(os.listdir(drm), key=lambda c: os.path.realpath(os.path.join(drm, c, "device")))
    dri = tmp_path / "dev" / "dri"
    dri.mkdir(parents=True)
    for i, c in enumerate(cards):   # PCI order i -> render node renderD(128 + i)
        (tmp_path / "sys" / "class" / "drm" / c / "device" / "drm" / f"renderD{128 + i}").mkdir(parents=True)
    for i in (2, 5):
        (dri / f"renderD{128 + i}").write_text("")
    g = device.gpus(root)
    assert [x.accessible for x in g] == [i in (2, 5) for i in range(8)]
    b = device.plan(2, sysfs=root, env={}, allowed=list(range(8)))
    assert [x.gpu for x in b] == [2, 5] and [x.numa_node for x in b] == [0, 1]
    # HIP_VISIBLE_DEVICES indexes the cards the process can open
    b = device.plan(1, sysfs=root, env={"HIP_VISIBLE_DEVICES": "1"}, allowed=list(range(8)))
    assert [x.gpu for x in b] == [5]
    # more ranks than exposed cards: nothing is bound
    b = device.plan(4, sysfs=root, env={}, allowed=list(range(8)))
    assert all(x.cpus == [] for x in b)
