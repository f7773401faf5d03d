"""Roofline accounting of the bench's TIMED WINDOW from a rocprofv3 kernel trace.

    python tools/window_summary.py run_kernel_trace.csv bench.json > summary.txt

``bench.py`` launches a named one-wave marker kernel (``window_mark_kernel``)
right after the timed window's opening barrier and right after its last
analysis completes (``rca_bench._window_mark``).  This tool keeps only the
kernels that ran between the two marks (clipped to them), so warm-up, thread
replay and the no-hints window are excluded, then prices every kernel family
against its ceiling with the work counters of the same window from the bench
JSON line (``engine.*``):

* decode attention: logical KV bytes = decode rows' context tokens x the KV
  bytes per token (shared prompt pages hit L2 / MALL, so the rate can exceed
  the HBM ceiling) against the measured 6.3 TB/s cold-streaming ceiling;
* prefill attention: 4 x heads x head_dim x layers FLOPs per (query, key) pair
  the planner computes (``prefill_attn_pairs``) against 2.5 PFLOP/s dense bf16;
* prefill-size projections (gemm_big + hipBLASLt at M > 256): 2 x dense
  parameters FLOPs per row of the large steps (``big_rows``) plus the LM head's
  sampled rows, against 2.5 PFLOP/s (1.5-1.6 sustained with every CU in MFMA);
* decode-size projections (skinny / mid / stream / grouped kernels, M <= 256):
  the dense weights streamed once per small step (``small_steps``) against
  6.3 TB/s.

The total kernel time of the window against the window's span gives the GPU
busy share (``total ~ span x busy``).
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from tools.kernel_summary import category  # noqa: E402

HBM_TBS = 6.3      # measured cold-streaming ceiling of one MI355X (profiles/r1_hbm_stream_bw.txt)
PEAK_TFS = 2500.0  # dense bf16 MFMA peak


def window(trace_path):
    ks = []
    with open(trace_path) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ks.sort()
    marks = [k for k in ks if "window_mark" in k[2]]
    if len(marks) < 2:
        raise SystemExit(f"{trace_path}: {len(marks)} window marks (run bench.py from this tree)")
    t0, t1 = marks[0][0], marks[-1][1]
    inside = [(max(s, t0), min(e, t1), n) for s, e, n in ks
              if e > t0 and s < t1 and "window_mark" not in n]
    return t0, t1, inside


def model_terms(name):
    from k8s_llm_rca_amd.models.config import get_config
    key = {"Llama-3-8B": "llama3-8b", "Llama-3-70B": "llama3-70b", "Mixtral-8x7B": "mixtral-8x7b"}.get(name, name)
    c = get_config(key)
    h, L = c.hidden, c.n_layers
    dense = L * (h * (c.q_size + 2 * c.kv_size) + c.q_size * h + 3 * h * c.intermediate * max(1, c.top_k or 1))
    return {"kv_bytes_per_token": 2 * L * c.kv_size * 2, "attn_flops_per_pair": 4 * c.n_heads * c.head_dim * L,
            "dense_params": dense, "dense_weight_bytes": 2 * L * (h * (c.q_size + 2 * c.kv_size) + c.q_size * h
                                                                + 3 * h * c.intermediate * max(1, c.n_experts)),
            "lm_head_flops_per_row": 2 * c.vocab_size * h}


def main(trace_path, bench_path):
    t0, t1, ks = window(trace_path)
    span = (t1 - t0) / 1e9
    fam = defaultdict(lambda: [0.0, 0])
    busy, busy_end = 0, t0
    for s, e, n in ks:
        f = fam[category(n)]
        f[0] += (e - s) / 1e9
        f[1] += 1
        # union of kernel intervals = GPU busy time (kernels of side streams overlap)
        if e > busy_end:
            busy += e - max(s, busy_end)
            busy_end = e
    total = sum(v[0] for v in fam.values())
    bench = None
    with open(bench_path) as fh:
        for line in fh:
            if line.startswith('{"metric"'):
                bench = json.loads(line)
    print(f"timed window {span:.2f} s (bench elapsed {bench['ms_per_step'] * bench['steps'] / 1e3:.2f} s), "
          f"{len(ks)} kernels, kernel time {total:.2f} s, GPU busy {busy / 1e9:.2f} s ({100 * busy / 1e9 / span:.1f} %)")
    e = bench["engine"]
    m = model_terms(bench["config"]["model"])
    tok = bench["tokens"]
    work = {
        "attn_decode": ("TB/s", e["decode_ctx_tokens"] * m["kv_bytes_per_token"] / 1e12, HBM_TBS),
        "attn_prefill": ("TFLOP/s", e.get("prefill_attn_pairs", 0) * m["attn_flops_per_pair"] / 1e12, PEAK_TFS),
        "prefill_gemm": ("TFLOP/s", (2 * m["dense_params"] * e.get("big_rows", 0)
                                     + m["lm_head_flops_per_row"] * (tok["sampled"])) / 1e12, PEAK_TFS),
        "decode_gemm": ("TB/s", e.get("small_steps", 0) * m["dense_weight_bytes"] / 1e12, HBM_TBS),
    }
    groups = {"attn_decode": ["attn_decode"], "attn_prefill": ["attn_prefill"],
              "prefill_gemm": ["gemm_big", "gemm_hipblaslt"], "decode_gemm": ["gemm_decode", "gemm_grouped"]}
    print(f"{'family':16s} {'time s':>8s} {'share':>7s} {'calls':>8s}")
    for k, (t, n) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
        print(f"{k:16s} {t:8.2f} {100 * t / total:6.1f}% {n:8d}")
    print("roofline (work from the bench line's window counters):")
    for g, (unit, amount, ceil) in work.items():
        t = sum(fam[c][0] for c in groups[g] if c in fam)
        if t <= 0:
            continue
        rate = amount / t
        print(f"  {g:14s} {amount:10.2f} {'TB' if unit == 'TB/s' else 'TFLOP'} in {t:6.2f} s"
              f" = {rate:8.1f} {unit}  ({100 * rate / ceil:5.1f} % of {ceil:g} {unit})")
    per = defaultdict(lambda: [0.0, 0])
    for s, e_, n in ks:
        nm = re.sub(r"\(.*", "", n)
        nm = re.sub(r"^void ", "", nm)[:80]
        per[nm][0] += (e_ - s) / 1e9
        per[nm][1] += 1
    print("top kernels in the window:")
    for nm, (t, n) in sorted(per.items(), key=lambda kv: -kv[1][0])[:14]:
        print(f"  {t:8.3f} s {100 * t / total:5.1f}% {n:7d} x {1e6 * t / n:8.1f} us  {nm}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
