"""Host placement of the ranks of an 8-GPU node (placement.py; SURVEY.md §8e's scaling
risks: decode cores, PCIe root complexes, NUMA placement of the pinned batches), on fake
sysfs trees -- no HIP runtime, no GPU."""
import json
import os
import subprocess
import sys

import pytest

from low_level_feature_extraction_amd import placement as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def fake_sysfs(tmp, gpu_nodes, node_cpus, smt=None, quota=None, cpu_kfd_nodes=2):
    """gpu_nodes: NUMA node of GPU 0..n-1; node_cpus: {node: "cpulist"}; smt: cpu -> its
    sibling (SMT pairs)."""
    topo = tmp / "class" / "kfd" / "kfd" / "topology" / "nodes"
    for i in range(cpu_kfd_nodes):
        (topo / str(i)).mkdir(parents=True)
        (topo / str(i) / "properties").write_text("cpu_cores_count 64\nsimd_count 0\n")
    for g, node in enumerate(gpu_nodes):
        k = cpu_kfd_nodes + g
        bus = 0x05 + 0x20 * g
        (topo / str(k)).mkdir(parents=True)
        (topo / str(k) / "properties").write_text(
            f"cpu_cores_count 0\nsimd_count 1024\nlocation_id {bus << 8}\ndomain 0\n")
        dev = tmp / "bus" / "pci" / "devices" / ("0000:%02x:00.0" % bus)
        dev.mkdir(parents=True)
        (dev / "numa_node").write_text(f"{node}\n")
    for node, cl in node_cpus.items():
        d = tmp / "devices" / "system" / "node" / f"node{node}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cl + "\n")
    for c, s in (smt or {}).items():
        d = tmp / "devices" / "system" / "cpu" / f"cpu{c}" / "topology"
        d.mkdir(parents=True)
        (d / "thread_siblings_list").write_text(P.format_cpulist([c, s]) + "\n")
    if quota:
        (tmp / "fs" / "cgroup").mkdir(parents=True)
        (tmp / "fs" / "cgroup" / "cpu.max").write_text(f"{quota * 100000} 100000\n")
    return str(tmp)


def two_socket(tmp, quota=None):
    # 2 sockets x 32 cores x 2 threads: node 0 = cores 0-31 (+ siblings 64-95), node 1 =
    # cores 32-63 (+ 96-127); GPUs 0-3 on node 0, 4-7 on node 1
    smt = {c: c + 64 for c in range(64)}
    smt.update({c + 64: c for c in range(64)})
    return fake_sysfs(tmp, [0, 0, 0, 0, 1, 1, 1, 1], {0: "0-31,64-95", 1: "32-63,96-127"}, smt, quota)


def test_cpulist_roundtrip():
    assert P.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert P.format_cpulist([11, 0, 1, 2, 3, 8, 10]) == "0-3,8,10-11"
    assert P.parse_cpulist("") == []


def test_gpus_from_kfd_topology(tmp_path):
    sys_root = two_socket(tmp_path)
    g = P.gpus(sys_root, env={})
    assert [x["numa_node"] for x in g] == [0, 0, 0, 0, 1, 1, 1, 1]
    assert g[0]["bdf"] == "0000:05:00.0" and g[7]["bdf"] == "0000:e5:00.0"
    # HIP_VISIBLE_DEVICES renumbers: device 0 of this process is the node's GPU 5
    assert [x["numa_node"] for x in P.gpus(sys_root, env={"HIP_VISIBLE_DEVICES": "5,2"})] == [1, 0]
    assert P.gpus(str(tmp_path / "none"), env={}) == []


def test_eight_ranks_on_two_nodes_get_disjoint_core_slices_of_their_gpus_node(tmp_path):
    sys_root = two_socket(tmp_path)
    allowed = range(128)
    plans = [P.plan(r, 8, sysfs=sys_root, env={}, allowed=allowed, quota=None) for r in range(8)]
    for r, p in enumerate(plans):
        k = r % 4
        base = 32 * (r // 4) + 8 * k  # eight whole cores of the GPU's node, with their siblings
        assert p["_cpu_set"] == list(range(base, base + 8)) + list(range(base + 64, base + 72)), r
        assert p["numa_node"] == r // 4 and p["source"] == "numa" and p["threads"] == 16
        assert p["gpu_bdf"] == "0000:%02x:00.0" % (0x05 + 0x20 * r)
    sets = [set(p["_cpu_set"]) for p in plans]
    assert all(not (sets[a] & sets[b]) for a in range(8) for b in range(a + 1, 8))
    assert set().union(*sets) == set(range(128))
    assert plans[5]["cpus"] == "40-47,104-111"


def test_quota_caps_the_thread_budget_and_affinity_limits_the_set(tmp_path):
    sys_root = two_socket(tmp_path, quota=64)  # a 64-CPU cgroup quota over 8 ranks: 8 threads each
    p = P.plan(2, 8, sysfs=sys_root, env={}, allowed=range(128))
    assert p["n_cpus"] == 16 and p["threads"] == 8
    # the process may only run on node 0's first 16 cores: its four ranks share them
    q = [P.plan(r, 8, sysfs=sys_root, env={}, allowed=list(range(16)) + list(range(64, 80)), quota=None)
         for r in range(4)]
    assert [x["_cpu_set"] for x in q] == [[0, 1, 2, 3, 64, 65, 66, 67], [4, 5, 6, 7, 68, 69, 70, 71],
                                          [8, 9, 10, 11, 72, 73, 74, 75], [12, 13, 14, 15, 76, 77, 78, 79]]


def test_ranks_sharing_one_gpu_split_its_node(tmp_path):
    sys_root = two_socket(tmp_path)
    a, b = (P.plan(r, 2, gpu_of_rank=[0, 0], sysfs=sys_root, env={}, allowed=range(128), quota=None)
            for r in range(2))
    assert a["_cpu_set"] == list(range(0, 16)) + list(range(64, 80))
    assert b["_cpu_set"] == list(range(16, 32)) + list(range(80, 96))
    assert a["numa_node"] == b["numa_node"] == 0


def test_without_numa_information_the_usable_cpus_split_evenly(tmp_path):
    sys_root = fake_sysfs(tmp_path, [-1, -1], {}, cpu_kfd_nodes=1)
    p = [P.plan(r, 2, sysfs=sys_root, env={}, allowed=range(10), quota=None) for r in range(2)]
    assert [x["_cpu_set"] for x in p] == [[0, 1, 2, 3, 4], [5, 6, 7, 8, 9]]
    assert all(x["source"] == "even split" and x["numa_node"] is None for x in p)


def test_bind_pins_the_process_and_sets_the_pool_budget(tmp_path):
    """In a child process (the binding is process-wide): the CPUs this test may use as two
    fake nodes; rank 1 of 2 gets the second node's CPUs, libllfe / decode.py pool sizes follow."""
    cpus = sorted(os.sched_getaffinity(0))
    if len(cpus) < 2:
        pytest.skip("needs two CPUs")
    half = len(cpus) // 2
    sys_root = fake_sysfs(tmp_path, [0, 1], {0: P.format_cpulist(cpus[:half]), 1: P.format_cpulist(cpus[half:])})
    code = ("import json, os, sys; sys.path.insert(0, %r)\n"
            "from low_level_feature_extraction_amd import placement, decode\n"
            "p = placement.bind(1, 2, sysfs=%r, env={}, quota=None)\n"
            "print(json.dumps({'plan': p, 'aff': sorted(os.sched_getaffinity(0)), "
            "'env': os.environ.get('LLFE_RANK_CPUS'), 'decode': decode.default_decode_threads()}))"
            % (ROOT, sys_root))
    env = dict(os.environ)
    env.pop("LLFE_DECODE_THREADS", None)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 0, out.stderr
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["aff"] == cpus[half:]
    assert d["plan"]["source"] == "numa" and d["plan"]["numa_node"] == 1
    assert int(d["env"]) == d["decode"] == len(cpus) - half
    env["LLFE_NUMA_BIND"] = "0"
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["plan"] is None and d["aff"] == cpus
