"""Instruction mix and wait / barrier skeleton of one kernel in a hipcc -S listing.

usage: python tools/asm_loop.py FILE.s SYMBOL_SUBSTRING [--skeleton N]
"""
import sys


def main():
    path, sym = sys.argv[1], sys.argv[2]
    n_sk = int(sys.argv[4]) if len(sys.argv) > 4 and sys.argv[3] == "--skeleton" else 80
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(sym) or (sym in l and l.endswith(":") is False and l.split(":")[0].endswith(sym)) or (l.startswith("_Z") and sym in l.split(":")[0]))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    cnt = {}
    keep = ("v_mfma", "s_waitcnt", "s_barrier", "global_load_lds", "ds_read", "s_cbranch", "buffer_load",
            "global_load", "global_store", "s_nop", "ds_write", "s_setprio")
    sk = []
    for l in body:
        t = l.strip().split()
        if not t:
            continue
        op = t[0]
        if op.startswith(keep):
            cnt[op] = cnt.get(op, 0) + 1
        if op.startswith(("s_waitcnt", "s_barrier", "s_cbranch")) or l.startswith(".LBB"):
            sk.append(l.strip())
    print(lines[start].split(":")[0], len(body), "lines")
    for k in sorted(cnt):
        print(f"  {k:32s} {cnt[k]}")
    print("\n".join(sk[:n_sk]))


if __name__ == "__main__":
    main()
