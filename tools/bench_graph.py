"""Graph-engine stress (BASELINE config 3: 100k-node synthetic graph, HIP CSR kernels).

Times, host (C++) vs HIP on the HBM mirror:
  * batched CONTAINS: every incident message against every EVENT node (find_srcKind's scan)
  * instance-level metapath walks: all Pods -[*1..3]-> nfs (relationship-unique walks)
  * temporal STATE lookup for every entity on the incidents' paths
"""
import argparse
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from k8s_llm_rca_amd.graph.device import DeviceGraph  # noqa: E402
from k8s_llm_rca_amd.graph import native  # noqa: E402
from k8s_llm_rca_amd.graph.synth import generate_cluster  # noqa: E402
from k8s_llm_rca_amd.graph.store import ts_to_ms  # noqa: E402


def t(fn, n=3):
    fn()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    a = time.perf_counter()
    for _ in range(n):
        r = fn()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return (time.perf_counter() - a) / n * 1e3, r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=100_000)
    ap.add_argument("--incidents", type=int, default=256)
    a = ap.parse_args()
    t0 = time.perf_counter()
    c = generate_cluster(a.nodes, a.incidents, seed=11)
    g = c.stategraph
    gen_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    dg = DeviceGraph(g, "cuda", min_gpu_rows=1)
    up_s = time.perf_counter() - t0
    res = {"nodes": g.num_nodes, "edges": g.num_edges, "gen_s": round(gen_s, 2), "upload_s": round(up_s, 3),
           "hbm_mb": round(dg.bytes / 2**20, 1)}
    ev = g.label_scan("EVENT")
    offs, buf = g.string_heap("message")
    msgs = c.messages
    cpu_ms, _ = t(lambda: [native.substr_mask(offs, buf, ev, m.encode()) for m in msgs], 1)
    gpu_ms, hits = t(lambda: dg.contains_many(ev, "message", msgs))
    res["contains"] = {"needles": len(msgs), "rows": len(ev), "cpu_ms": round(cpu_ms, 2), "gpu_ms": round(gpu_ms, 2),
                       "hits": int(hits.sum())}
    pods = g.label_scan("Pod")
    dev = g.device
    cpu_ms, ref = t(lambda: g.var_length(pods, 1, 3, "out", ["ReferInternal", "UseExternal"], "nfs"), 1)
    gpu_ms, rec = t(lambda: dg.walks(pods, 1, 3, "out", ["ReferInternal", "UseExternal"], "nfs"))
    res["walks_pod_to_nfs"] = {"starts": len(pods), "paths": int(len(rec)), "cpu_ms": round(cpu_ms, 2),
                               "gpu_ms": round(gpu_ms, 2), "match": len(ref) == len(rec)}
    cpu_ms, ref2 = t(lambda: g.var_length(pods, 1, 2, "both", None, None), 1)
    gpu_ms, rec2 = t(lambda: dg.walks(pods, 1, 2, "both", None, None))
    res["walks_pod_undirected_2hop"] = {"paths": int(len(rec2)), "cpu_ms": round(cpu_ms, 2),
                                       "gpu_ms": round(gpu_ms, 2), "match": len(ref2) == len(rec2)}
    ents = np.concatenate([pods, g.label_scan("nfs"), g.label_scan("PersistentVolumeClaim"),
                           g.label_scan("Secret"), g.label_scan("ConfigMap")])
    ts = np.full(len(ents), ts_to_ms("2020-12-12 12:00:00.000"), dtype=np.int64)
    cpu_ms, _ = t(lambda: g.state_lookup(ents, ts, None, "strict", None, 10), 1)
    gpu_ms, _ = t(lambda: dg.state_lookup(ents, ts, None, "strict", None, 10))
    res["state_lookup"] = {"entities": len(ents), "cpu_ms": round(cpu_ms, 2), "gpu_ms": round(gpu_ms, 2)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
