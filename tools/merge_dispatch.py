"""Merge a fresh decode-GEMM sweep (tools/gemm_mid_sweep.py --emit --out NEW) into
a stored dispatch table: per (shape, M bucket) the faster of the stored and the
new measurement (both cold-weight timings on MI355X; box-to-box noise is a few %).

python tools/merge_dispatch.py NEW.json k8s_llm_rca_amd/data/gemm_dispatch_<model>.json "note"
"""
import json
import sys


def merge(new_path: str, old_path: str, note: str) -> int:
    new = json.load(open(new_path))
    old = json.load(open(old_path))
    changed = 0
    for k, rows in old["shapes"].items():
        nm = {r["m"]: r for r in new["shapes"].get(k, [])}
        out = []
        for r in rows:
            n = nm.get(r["m"])
            same = n is not None and (n["kind"], n.get("cfg"), n.get("splits")) == (r["kind"], r.get("cfg"), r.get("splits"))
            if n is not None and not same and "t_us" in n and "t_us" in r and n["t_us"] < r["t_us"]:
                out.append(n)
                changed += 1
            else:
                out.append(r)
        old["shapes"][k] = out
    for k, rows in new["shapes"].items():  # shapes the stored table did not have
        if k not in old["shapes"]:
            old["shapes"][k] = rows
            changed += len(rows)
    if changed:
        old["note"] = old.get("note", "") + " " + note
    json.dump(old, open(old_path, "w"), indent=1)
    return changed


if __name__ == "__main__":
    print("changed", merge(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else ""))
