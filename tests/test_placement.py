"""Rank CPU placement (utils/placement.py): the ranks of an
8-GPU DP bench bind themselves to disjoint, NUMA-local CPU slices before any
GPU call -- checked on a synthetic 2-socket topology and, in 8 real child
processes, on this machine's own."""
import multiprocessing as mp
import os

import pytest

from k8s_llm_rca_amd.utils import placement as PL


def test_cpulist_roundtrip():
    assert PL.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert PL.format_cpulist([11, 10, 8, 3, 2, 1, 0]) == "0-3,8,10-11"
    assert PL.format_cpulist([]) == ""


def test_kfd_topology_numa_local_disjoint():
    nodes = {0: list(range(0, 64)), 1: list(range(64, 128))}
    gpus = [0, 0, 0, 0, 1, 1, 1, 1]
    allowed = list(range(128))
    seen = set()
    for r in range(8):
        cpus, node, src = PL.rank_cpus(r, 8, allowed, nodes, gpus)
        assert src == "kfd" and node == gpus[r]
        assert len(cpus) == 16 and set(cpus) <= set(nodes[node])
        assert not (set(cpus) & seen)
        seen |= set(cpus)
    # a restricted allowed set (a container cgroup): slices stay inside it
    allowed = list(range(8, 40)) + list(range(72, 104))
    seen = set()
    for r in range(8):
        cpus, node, _ = PL.rank_cpus(r, 8, allowed, nodes, gpus)
        assert len(cpus) == 8 and set(cpus) <= set(allowed) & set(nodes[node]) and not (set(cpus) & seen)
        seen |= set(cpus)


def test_fallbacks_even_and_split():
    nodes = {0: list(range(0, 8)), 1: list(range(8, 16))}
    got = [PL.rank_cpus(r, 4, list(range(16)), nodes, [])[:2] for r in range(4)]
    assert [n for _, n in got] == [0, 0, 1, 1]
    assert sorted(c for cpus, _ in got for c in cpus) == list(range(16))
    # no NUMA information at all: the allowed set split evenly
    got = [PL.rank_cpus(r, 8, list(range(8)), {}, [])[0] for r in range(8)]
    assert got == [[i] for i in range(8)]


def _child(r, n, q):
    os.environ["K8SRCA_BIND"] = "1"
    info = PL.bind_rank(r, n)
    q.put((r, info, sorted(os.sched_getaffinity(0))))


@pytest.mark.skipif(not hasattr(os, "sched_setaffinity"), reason="no sched_setaffinity")
def test_eight_ranks_bind_disjoint_on_this_machine():
    n = 8
    allowed = sorted(os.sched_getaffinity(0))
    if len(allowed) < n:
        pytest.skip("fewer CPUs than ranks")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_child, args=(r, n, q)) for r in range(n)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=60) for _ in range(n))
    for p in ps:
        p.join(30)
    masks = [set(m) for _, _, m in res]
    assert all(info is not None for _, info, _ in res)
    assert all(masks) and sum(len(m) for m in masks) == len(set().union(*masks))  # pairwise disjoint
    assert set().union(*masks) <= set(allowed)
