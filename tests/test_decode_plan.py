"""Decode work-list planning on the host (no GPU): multi-token items."""
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
