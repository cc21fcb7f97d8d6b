"""Host placement of one GPU rank on a multi-GPU node.

The path shards images over GPUs with no data-path collective, so what limits an 8-rank
node is host-side: decode cores, PCIe root complexes and the NUMA placement of the pinned
host batches.  The reference runs one worker process per core share
(``gunicorn -w 4``, /root/reference/Dockerfile:26); here one process runs per GPU, and this
module gives each rank the CPUs of its GPU's NUMA node:

* GPU -> PCI device -> NUMA node, read from sysfs without starting a HIP runtime: HIP
  numbers the GPUs in kfd topology order (``/sys/class/kfd/kfd/topology/nodes/*``, the
  nodes with SIMDs), each node's ``domain`` / ``location_id`` give its PCI address, and
  ``/sys/bus/pci/devices/<bdf>/numa_node`` its node (``*_VISIBLE_DEVICES`` filters apply);
* the node's CPUs (``/sys/devices/system/node/node<N>/cpulist``, within this process's
  affinity mask) are split evenly, whole cores (SMT siblings together) at a time, among
  the ranks whose GPUs sit on that node -- per node, not usable / LOCAL_WORLD_SIZE;
* ``bind()`` pins the calling thread to that set before any pool starts, so the contour
  pool (libllfe), the decode pool (decode.py) and every pinned host buffer the rank
  allocates afterwards (first touch: the local node) live on the GPU's node, and exports
  ``LLFE_RANK_CPUS`` (the rank's thread budget: the set's size, capped by its share of a
  cgroup cpu.max quota), which libllfe's and decode.py's pool sizes then use as is.

Without NUMA information (no sysfs node, numa_node -1) the usable CPUs are split evenly in
rank order instead (``source: "even split"``).  ``LLFE_NUMA_BIND=0`` disables binding.
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, List, Optional, Sequence


def parse_cpulist(text: str) -> List[int]:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]"""
    out: List[int] = []
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def format_cpulist(cpus: Iterable[int]) -> str:
    s = sorted(set(cpus))
    parts, i = [], 0
    while i < len(s):
        j = i
        while j + 1 < len(s) and s[j + 1] == s[j] + 1:
            j += 1
        parts.append(str(s[i]) if i == j else f"{s[i]}-{s[j]}")
        i = j + 1
    return ",".join(parts)


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def _visible_filter(n: int, env) -> List[int]:
    """Indices (into the kfd GPU list) this process sees: ROCR_VISIBLE_DEVICES, then
    HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES over what remains (integer lists; other
    forms -- UUIDs -- are not filtered here)."""
    idx = list(range(n))
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is None:
            continue
        try:
            sel = [int(x) for x in v.split(",") if x.strip() != ""]
        except ValueError:
            continue
        idx = [idx[i] for i in sel if 0 <= i < len(idx)]
        if var != "ROCR_VISIBLE_DEVICES":
            break  # HIP_VISIBLE_DEVICES takes precedence over CUDA_VISIBLE_DEVICES
    return idx


def gpus(sysfs: str = "/sys", env=None) -> List[Dict]:
    """The GPUs HIP will number 0, 1, ...: [{"kfd_node", "bdf", "numa_node"}]."""
    env = os.environ if env is None else env
    root = os.path.join(sysfs, "class", "kfd", "kfd", "topology", "nodes")
    try:
        nodes = sorted(int(d) for d in os.listdir(root) if d.isdigit())
    except OSError:
        return []
    found = []
    for n in nodes:
        txt = _read(os.path.join(root, str(n), "properties"))
        if txt is None:
            continue
        props = {}
        for line in txt.splitlines():
            kv = line.split()
            if len(kv) == 2:
                props[kv[0]] = kv[1]
        if int(props.get("simd_count", "0")) <= 0:
            continue  # a CPU node
        loc, dom = int(props.get("location_id", "0")), int(props.get("domain", "0"))
        bdf = "%04x:%02x:%02x.%x" % (dom, loc >> 8, (loc >> 3) & 0x1F, loc & 7)
        numa = _read(os.path.join(sysfs, "bus", "pci", "devices", bdf, "numa_node"))
        found.append({"kfd_node": n, "bdf": bdf, "numa_node": int(numa) if numa and numa.strip() else -1})
    return [found[i] for i in _visible_filter(len(found), env)]


def node_cpus(node: int, sysfs: str = "/sys") -> List[int]:
    txt = _read(os.path.join(sysfs, "devices", "system", "node", f"node{node}", "cpulist"))
    return parse_cpulist(txt) if txt else []


def _cores(cpus: Sequence[int], sysfs: str) -> List[List[int]]:
    """cpus grouped by physical core (SMT siblings together), in order of their first CPU."""
    have = set(cpus)
    seen, groups = set(), []
    for c in sorted(cpus):
        if c in seen:
            continue
        sib = _read(os.path.join(sysfs, "devices", "system", "cpu", f"cpu{c}", "topology", "thread_siblings_list"))
        g = sorted(x for x in (parse_cpulist(sib) if sib else [c]) if x in have) or [c]
        if c not in g:
            g = [c]
        seen.update(g)
        groups.append(g)
    return groups


def _slice(groups: List[List[int]], k: int, m: int) -> List[int]:
    """Slice k of m of the core groups (the first len % m slices one core longer); when
    there are fewer cores than slices, slices share cores round-robin."""
    if not groups:
        return []
    if len(groups) < m:
        return sorted(groups[k % len(groups)])
    q, r = divmod(len(groups), m)
    a = k * q + min(k, r)
    b = a + q + (1 if k < r else 0)
    return sorted(c for g in groups[a:b] for c in g)


def _quota_cpus(sysfs_cgroup: str = "/sys/fs/cgroup/cpu.max") -> Optional[int]:
    txt = _read(sysfs_cgroup)
    if not txt:
        return None
    try:
        q, p = txt.split()[:2]
        return None if q == "max" else max(1, int(q) // int(p))
    except ValueError:
        return None


def plan(local_rank: int, local_world: int, gpu_of_rank: Optional[Sequence[int]] = None, sysfs: str = "/sys",
         env=None, allowed: Optional[Iterable[int]] = None, quota: Optional[int] = -1) -> Dict:
    """The CPU set of rank ``local_rank`` of the ``local_world`` ranks on this node.
    ``gpu_of_rank[r]``: the GPU index rank r drives (default r; all 0 when every rank
    shares one GPU).  ``allowed``: the process affinity (default sched_getaffinity);
    ``quota``: the cgroup CPU quota (-1: read it)."""
    env = os.environ if env is None else env
    if allowed is None:
        allowed = os.sched_getaffinity(0)
    allowed = sorted(set(allowed))
    if quota == -1:
        quota = _quota_cpus(os.path.join(sysfs, "fs", "cgroup", "cpu.max"))
    g_of = list(gpu_of_rank) if gpu_of_rank is not None else list(range(local_world))
    gl = gpus(sysfs, env)
    numa_of = [gl[g]["numa_node"] if 0 <= g < len(gl) else -1 for g in g_of]
    me = g_of[local_rank] if local_rank < len(g_of) else local_rank
    node = numa_of[local_rank] if local_rank < len(numa_of) else -1
    cpus: List[int] = []
    source = "even split"
    if node >= 0:
        ncpu = [c for c in node_cpus(node, sysfs) if c in set(allowed)]
        if ncpu:
            peers = [r for r in range(local_world) if numa_of[r] == node]
            cpus = _slice(_cores(ncpu, sysfs), peers.index(local_rank), len(peers))
            source = "numa"
    if not cpus:
        cpus = _slice(_cores(allowed, sysfs), local_rank, local_world)
    threads = len(cpus)
    if quota:
        threads = min(threads, max(1, quota // max(1, local_world)))
    return {"local_rank": local_rank, "gpu": me, "gpu_bdf": gl[me]["bdf"] if 0 <= me < len(gl) else None,
            "numa_node": node if source == "numa" else None, "cpus": format_cpulist(cpus), "n_cpus": len(cpus),
            "threads": max(1, threads), "source": source, "_cpu_set": cpus}


def bind(local_rank: int, local_world: int, gpu_of_rank: Optional[Sequence[int]] = None, **kw) -> Optional[Dict]:
    """plan() and pin the calling thread (call it before any thread pool or pinned buffer
    exists: threads inherit the mask, first-touch pages follow it).  Returns the plan
    (without the raw set), or None when ``LLFE_NUMA_BIND=0``."""
    if os.environ.get("LLFE_NUMA_BIND", "1") == "0":
        return None
    p = plan(local_rank, local_world, gpu_of_rank, **kw)
    cpus = p.pop("_cpu_set")
    try:
        os.sched_setaffinity(0, cpus)
    except (OSError, AttributeError, ValueError) as e:  # pragma: no cover - restricted hosts
        p["error"] = str(e)
        return p
    os.environ["LLFE_RANK_CPUS"] = str(p["threads"])
    return p
