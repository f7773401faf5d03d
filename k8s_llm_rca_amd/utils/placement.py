"""CPU placement of the per-GPU rank processes (``bench.py --gpus N``).

One engine replica per GPU keeps ~1.75 cores busy (the engine thread plus a
HIP-runtime thread, ``BENCH_r03`` ``host_cpu_s``); eight of them floating over
both sockets of an 8-GPU node share caches and memory controllers with the
wrong GPU's traffic.  Each rank binds itself -- before anything touches the
GPU, so every HIP-runtime and torch thread it starts inherits the mask -- to a
disjoint slice of the CPUs of the NUMA node its GPU hangs off:

* GPU -> NUMA node from the KFD topology (``/sys/class/kfd/kfd/topology``:
  GPU nodes in enumeration order, each with an IO link to its CPU node), with
  ``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES``
  applied; fallback: ranks spread evenly over the NUMA nodes in order.
* the node's CPUs (``/sys/devices/system/node/node*/cpulist``, intersected
  with the process's allowed set) split evenly among the ranks on that node;
  a node with no allowed CPU -> the allowed set split evenly over all ranks.

No exec, no GPU call: :func:`bind_rank` only reads sysfs and calls
``os.sched_setaffinity``.  ``K8SRCA_BIND=0`` disables it.
"""
from __future__ import annotations

from ..knobs import KNOBS
import glob
import os
import re
from typing import Dict, List, Optional, Sequence


def parse_cpulist(text: str) -> List[int]:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]."""
    out: List[int] = []
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def format_cpulist(cpus: Sequence[int]) -> str:
    """[0, 1, 2, 3, 8] -> '0-3,8'."""
    cpus = sorted(set(cpus))
    parts, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        parts.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(parts)


def numa_cpus(root: str = "/sys/devices/system/node") -> Dict[int, List[int]]:
    """NUMA node id -> its CPUs ({} when sysfs has no node directories)."""
    out = {}
    for d in glob.glob(os.path.join(root, "node[0-9]*")):
        m = re.search(r"node(\d+)$", d)
        try:
            with open(os.path.join(d, "cpulist")) as f:
                cpus = parse_cpulist(f.read())
        except OSError:
            continue
        if m and cpus:
            out[int(m.group(1))] = cpus
    return out


def _props(path: str) -> Dict[str, int]:
    out = {}
    try:
        with open(path) as f:
            for line in f:
                k, _, v = line.strip().partition(" ")
                if v.lstrip("-").isdigit():
                    out[k] = int(v)
    except OSError:
        pass
    return out


def gpu_numa_nodes(root: str = "/sys/class/kfd/kfd/topology/nodes") -> List[int]:
    """CPU NUMA node of every GPU in KFD enumeration order ([] if unknown)."""
    nodes = sorted((int(os.path.basename(d)), d) for d in glob.glob(os.path.join(root, "[0-9]*")))
    props = {i: _props(os.path.join(d, "properties")) for i, d in nodes}
    cpu_nodes = [i for i, p in props.items() if p.get("simd_count", 0) == 0 and p.get("cpu_cores_count", 0) > 0]
    out = []
    for i, d in nodes:
        if props[i].get("simd_count", 0) == 0:
            continue
        numa = -1
        for link in sorted(glob.glob(os.path.join(d, "io_links", "*", "properties"))):
            to = _props(link).get("node_to", -1)
            if to in cpu_nodes:
                numa = cpu_nodes.index(to)  # CPU nodes enumerate in NUMA order
                break
        out.append(numa)
    return out if out and all(n >= 0 for n in out) else []


def _visible(n_phys: int) -> List[int]:
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v:
            try:
                ids = [int(x) for x in v.split(",") if x.strip() != ""]
            except ValueError:
                return list(range(n_phys))
            return [i for i in ids if 0 <= i < n_phys]
    return list(range(n_phys))


def rank_cpus(local_rank: int, local_world: int, allowed: Sequence[int], nodes: Dict[int, List[int]],
              gpu_nodes: Sequence[int]) -> tuple:
    """(cpus, numa node or -1, source) of ``local_rank``: disjoint across ranks."""
    allowed = sorted(set(allowed))
    node_of = {}
    if gpu_nodes and len(gpu_nodes) >= local_world:
        node_of = {r: gpu_nodes[r] for r in range(local_world)}
        src = "kfd"
    elif nodes:
        ids = sorted(nodes)
        node_of = {r: ids[r * len(ids) // local_world] for r in range(local_world)}
        src = "even"
    if node_of:
        node = node_of[local_rank]
        peers = [r for r in range(local_world) if node_of[r] == node]
        pool = [c for c in nodes.get(node, []) if c in set(allowed)]
        if len(pool) >= len(peers):
            k = peers.index(local_rank)
            lo, hi = k * len(pool) // len(peers), (k + 1) * len(pool) // len(peers)
            return pool[lo:hi], node, src
    # no usable topology: the allowed set split evenly (one CPU at least, shared only if too few)
    n = len(allowed)
    if n >= local_world:
        lo, hi = local_rank * n // local_world, (local_rank + 1) * n // local_world
        return allowed[lo:hi], -1, "split"
    return [allowed[local_rank % n]] if n else [], -1, "split"


def bind_rank(local_rank: int, local_world: int) -> Optional[dict]:
    """Bind this process to its rank's CPU slice (see the module docstring);
    returns ``{"cpus", "numa", "source"}`` or None when disabled / unsupported."""
    if not KNOBS.bind or local_world <= 1 or not hasattr(os, "sched_setaffinity"):
        return None
    allowed = sorted(os.sched_getaffinity(0))
    gpus = gpu_numa_nodes()
    if gpus:
        vis = _visible(len(gpus))
        gpus = [gpus[i] for i in vis]
    cpus, node, src = rank_cpus(local_rank, local_world, allowed, numa_cpus(), gpus)
    if not cpus:
        return None
    os.sched_setaffinity(0, cpus)
    return {"cpus": format_cpulist(cpus), "numa": node, "source": src}
