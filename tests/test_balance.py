"""parallel/balance.py: LPT unit assignment, the store-backed unit queue, and GPU-local CPU pinning
read from a fake sysfs tree (KFD topology -> PCI address -> local_cpulist)."""
import os

import numpy as np

from fairify_amd.parallel import balance as BL


def _fake_sysfs(root, gpus):
    """gpus: list of (domain, bus, cpulist); a CPU node first, like the real KFD topology."""
    nodes = os.path.join(root, "class", "kfd", "kfd", "topology", "nodes")
    os.makedirs(os.path.join(nodes, "0"))
    with open(os.path.join(nodes, "0", "properties"), "w") as f:
        f.write("cpu_cores_count 64\nsimd_count 0\nlocation_id 0\ndomain 0\n")
    for k, (dom, bus, cl) in enumerate(gpus):
        d = os.path.join(nodes, str(k + 1))
        os.makedirs(d)
        with open(os.path.join(d, "properties"), "w") as f:
            f.write(f"cpu_cores_count 0\nsimd_count 1024\nlocation_id {bus << 8}\ndomain {dom}\n")
        pci = os.path.join(root, "bus", "pci", "devices", f"{dom:04x}:{bus:02x}:00.0")
        os.makedirs(pci)
        with open(os.path.join(pci, "local_cpulist"), "w") as f:
            f.write(cl + "\n")


def test_parse_cpulist():
    assert BL.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert BL.parse_cpulist("") == []


def test_numa_local_slices(tmp_path, monkeypatch):
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    # 8 GPUs: 0-3 on socket 0 (CPUs 0-15), 4-7 on socket 1 (CPUs 16-31)
    gpus = [(0, 0x10 + k, "0-15" if k < 4 else "16-31") for k in range(8)]
    _fake_sysfs(str(tmp_path), gpus)
    assert BL.gpu_pci_addresses(str(tmp_path))[5] == "0000:15:00.0"
    cpus = list(range(32))
    sets = [BL.rank_cpuset(r, 8, cpus, sysfs=str(tmp_path)) for r in range(8)]
    assert sets[0] == [0, 1, 2, 3] and sets[3] == [12, 13, 14, 15]
    assert sets[4] == [16, 17, 18, 19] and sets[7] == [28, 29, 30, 31]
    assert sorted(c for s in sets for c in s) == cpus            # disjoint cover
    # two ranks on GPUs of different sockets: each gets its whole socket
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "1,6")
    assert BL.rank_cpuset(0, 2, cpus, sysfs=str(tmp_path)) == list(range(16))
    assert BL.rank_cpuset(1, 2, cpus, sysfs=str(tmp_path)) == list(range(16, 32))
    # allowed CPUs restrict the local sets
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES")
    assert BL.rank_cpuset(4, 8, list(range(8)) + list(range(16, 24)), sysfs=str(tmp_path)) == [16, 17]


def test_numa_one_visible_gpu_per_rank(tmp_path, monkeypatch):
    """Each rank sees only its own GPU (HIP_VISIBLE_DEVICES=<one id>): local rank r is physical GPU r,
    so the 4 ranks of a socket split its CPUs 4 ways (not 8 ways as if every rank were a peer)."""
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    gpus = [(0, 0x10 + k, "0-15" if k < 4 else "16-31") for k in range(8)]
    _fake_sysfs(str(tmp_path), gpus)
    cpus = list(range(32))
    sets = []
    for r in range(8):
        monkeypatch.setenv("HIP_VISIBLE_DEVICES", str(r))
        sets.append(BL.rank_cpuset(r, 8, cpus, sysfs=str(tmp_path)))
    assert sets[0] == [0, 1, 2, 3] and sets[5] == [20, 21, 22, 23]
    assert sorted(c for s in sets for c in s) == cpus
    # more local ranks than GPUs in the node: peers unknown -> contiguous slices
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
    assert BL.rank_cpuset(9, 16, cpus, sysfs=str(tmp_path)) == [18, 19]


def test_fallback_contiguous(tmp_path):
    # no KFD topology: the contiguous slices of the allowed CPUs
    cpus = list(range(16))
    assert BL.rank_cpuset(1, 4, cpus, sysfs=str(tmp_path)) == [4, 5, 6, 7]
    assert BL.rank_cpuset(3, 4, cpus, sysfs=str(tmp_path), numa=False) == [12, 13, 14, 15]
    assert BL.rank_cpuset(5, 8, [0, 1, 2], sysfs=str(tmp_path)) == [2]


def test_lpt_bound():
    rng = np.random.default_rng(0)
    c = rng.pareto(1.5, 200) + 0.1
    for w in (2, 4, 8):
        a = BL.lpt_assign(c, w)
        loads = BL.rank_loads(a, c)
        assert sorted(u for r in a for u in r) == list(range(200))
        assert loads.max() <= loads.mean() + c.max() + 1e-9
