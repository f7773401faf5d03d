"""Decode work-list planning on the host (no GPU): multi-token items."""
import pytest
import numpy as np

from k8s_llm_rca_amd.ops import attention as A


def _coverage(items, ctx, part):
    """(row, key) pairs each row's items cover, with the partition index the
    row's split-KV reduce expects for every key."""
    cov = {}
    for seq, p, k1, w in items.tolist():
        nt = (w >> 24) + 1
        assert (w & 0xFFFFFF) == seq  # q rows are the row indices here
        k0 = 0 if p < 0 else p * part
        for qi in range(nt):
            r = seq + qi
            lim = min(k1, ctx[r])
            n_row = -(-ctx[r] // part)
            assert (p < 0) == (n_row == 1)  # whole-row items only for one-partition rows
            for k in range(k0, lim):
                assert (r, k) not in cov
                cov[(r, k)] = p
    return cov


def test_multi_token_items_cover_every_row_once():
    rng = np.random.default_rng(0)
    for trial in range(20):
        ctx, chain = [], []
        for _ in range(rng.integers(1, 12)):
            c0, q = int(rng.integers(1, 3000)), int(rng.integers(1, 9))
            for j in range(q):
                ctx.append(c0 + j + 1)
                chain.append(j > 0)
        part = int(rng.choice([256, 320, 512, 1024]))
        for gmax in (1, 2, 4):
            items = A.build_decode_items(ctx, np.arange(len(ctx)), part, np.asarray(chain), gmax)
            cov = _coverage(items, ctx, part)
            assert len(cov) == sum(ctx)
            nts = (items[:, 3] >> 24) + 1
            assert nts.max() <= gmax
            if gmax == 1:
                assert (nts == 1).all()


def test_groups_break_on_partition_count_and_sequence():
    ctx = [255, 256, 257, 258, 10, 11]
    chain = np.array([0, 1, 1, 1, 0, 1], bool)
    lead, nt = A.decode_groups(ctx, np.arange(6), chain, 4, part=256)
    assert lead.tolist() == [0, 2, 4] and nt.tolist() == [2, 2, 2]
    lead, nt = A.decode_groups(ctx, np.arange(6), chain, 4)
    assert lead.tolist() == [0, 4] and nt.tolist() == [4, 2]
    lead, nt = A.decode_groups(ctx, np.arange(6), None, 4)
    assert nt.tolist() == [1] * 6


def test_prefill_plan_caps_w8_items_at_lds_page_table(monkeypatch, knob):
    """with the 8-wave prefill kernel every work item spans at
    most PF8_MAXP key pages (the kernel's LDS page table), whatever the block
    table width; each tile's items tile its key range exactly once."""
    knob("pf_w8", 2)
    for ctx, qlen, known in (([70_000, 500], [96, 40], True), ([66_000, 300], [66_000, 300], False)):
        qs = [0]
        for n in qlen:
            qs.append(qs[-1] + n)
        plan = A.plan_prefill(qs, 4, 64, list(ctx) if known else None, nkv=8)
        spans = {}
        for s, t, n, k0, k1, sl in zip(plan.seq, plan.tok0, plan.length, plan.kv0, plan.kv1, plan.slot):
            assert k1 - k0 <= A.PF8_MAXP or k1 >= 1 << 30
            spans.setdefault((s, t), []).append((k0, k1, sl))
        for (s, t), sp in spans.items():
            sp.sort()
            base = ctx[s] - qlen[s]
            end_pages = -(-(base + (t - qs[s]) + min(64, qs[s + 1] - t)) // 64)
            if len(sp) > 1:
                assert sp[0][0] == 0 and all(a[1] == b[0] for a, b in zip(sp, sp[1:]))
                assert sp[-1][1] >= min(end_pages, sp[-1][1])
    # the 4-wave kernel has no page table: no cap without a split plan
    knob("pf_w8", 0)
    plan = A.plan_prefill([0, 66_000], 4, 64, None, nkv=8)
    assert plan.n_merge == 0


def test_prefill_makespan_planner_covers_keys_and_balances(monkeypatch, knob):
    """The makespan split choice (K8S_PF_OVERHEAD_PAGES > 0): every tile's items
    still tile its key range exactly once, the slot budget holds, and on a
    200-700-token extend over a ~5k context (7 tiles x 8 heads of ~83 pages) it
    picks a split whose round count is full rather than a few items over a
    multiple of the CU slots."""
    knob("pf_w8", 1)
    monkeypatch.setattr(A, "PF_OVERHEAD_PAGES", 3.0)
    monkeypatch.setattr(A, "PF_MAKESPAN_ALL", True)
    ctx, q = [5277], [437]
    plan = A.plan_prefill([0, q[0]], 4, 64, ctx, nkv=8)
    spans = {}
    for t, k0, k1 in zip(plan.tok0, plan.kv0, plan.kv1):
        spans.setdefault(t, []).append((k0, k1))
    for t, sp in spans.items():
        sp.sort()
        assert sp[0][0] == 0 and all(a[1] == b[0] for a, b in zip(sp, sp[1:]))
        assert sp[-1][1] == -(-(ctx[0] - q[0] + t + min(64, q[0] - t)) // 64)
    n_wg = plan.n_tiles * 8
    rounds = -(-n_wg // A.PF_CU_SLOTS)
    assert n_wg > (rounds - 1) * A.PF_CU_SLOTS + A.PF_CU_SLOTS // 2  # the last round is at least half full
    assert sum(plan.m_np) <= A.PF_MAX_SLOTS
    # a fresh 8k prompt: 32 causal tiles x 8 heads fill the CUs once, but the
    # tiles run 1..128 pages -- the longest ones are split so the launch is not
    # twice its average work (the fixed-target rule leaves them whole)
    plan = A.plan_prefill([0, 8192], 4, 64, [8192], nkv=8)
    longest = max(b - a for a, b in zip(plan.kv0, plan.kv1))
    assert plan.n_merge > 0 and longest < 128
    monkeypatch.setattr(A, "PF_OVERHEAD_PAGES", 0.0)
    assert A.plan_prefill([0, 8192], 4, 64, [8192], nkv=8).n_merge == 0
    # the default (makespan only where the fixed rule splits) leaves it whole too
    monkeypatch.setattr(A, "PF_OVERHEAD_PAGES", 8.0)
    monkeypatch.setattr(A, "PF_MAKESPAN_ALL", False)
    assert A.plan_prefill([0, 8192], 4, 64, [8192], nkv=8).n_merge == 0


def test_fit_slots_clamps_non_power_of_two_part():
    """a makespan part such as 768 must clamp its doubling at
    max_part (1024) instead of jumping to 1536 and failing a plan that fits."""
    from k8s_llm_rca_amd.ops import attention as A
    pages = [1024 * 3] * 4                   # 12 slots at part 1024, 16 at 768
    assert A._fit_slots(pages, 768, 1024, 12) == 1024
    assert A._fit_slots(pages, 384, 1024, 12) == 1024
    assert A._fit_slots(pages, 256, None, 12) == 1024
    with pytest.raises(ValueError):
        A._fit_slots(pages, 768, 1024, 11)   # max_part itself overflows


@pytest.mark.parametrize("rows,ctx,want", [(1, 2048, 64), (1, 5000, 128), (2, 5000, 192), (2, 8000, 256),
                                           (4, 2048, 128), (4, 8000, 512), (8, 2048, 256)])
def test_low_batch_decode_split_targets_wave_count(rows, ctx, want):
    """One-round decode steps take the fewest keys per item that keep the
    launch at <= DECODE_LOW_UNITS (item, kv head) waves -- the measured best of
    tools/decode_part_sweep.py at these shapes -- capped by the graph buffers'
    partition count; big batches keep the makespan planner (>= 256 keys)."""
    nkv = 8
    n, P = A.plan_decode_split([ctx] * rows, nkv)
    assert P == want and n == -(-ctx // P)
    assert nkv * rows * n <= A.DECODE_LOW_UNITS
    # the buffer cap: at most 32 partitions (an 8k window at 256 keys) -> P >= ctx / 32
    n2, P2 = A.plan_decode_split([ctx] * rows, nkv, max_parts=32)
    assert n2 <= 32 and P2 >= P
    # a headline-size step: many rows, several rounds -> the makespan planner's part sizes
    _, Pb = A.plan_decode_split([5000] * 100, nkv)
    assert Pb in A.DECODE_PARTS


def test_low_batch_rule_off(monkeypatch):
    monkeypatch.setattr(A, "DECODE_LOW_UNITS", 0)
    _, P = A.plan_decode_split([5000], 8)
    assert P == min(A.DECODE_PARTS)
