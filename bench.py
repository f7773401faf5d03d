#!/usr/bin/env python
"""Headline benchmark: RCA analyses/s + p50 latency (Llama-3-8B backend, 10k-node graph).

Contract: ``python bench.py --gpus N --steps K --warmup W``.  Under torchrun
(WORLD_SIZE set) this process is one rank; otherwise ``--gpus N`` > 1 spawns
the N rank processes itself (one per GPU, data-parallel engine replicas).
Rank 0 prints ONE JSON line.  See k8s_llm_rca_amd/bench/rca_bench.py.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
# Kernel arguments in device memory: with it explicitly off the headline drops
# 6.03 -> 5.91 analyses/s (profiles/README.md); pin it on unless the caller says otherwise.
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

from k8s_llm_rca_amd.bench.rca_bench import exit_now, main  # noqa: E402

if __name__ == "__main__":
    exit_now(main())
