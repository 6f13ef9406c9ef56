"""Sparse data parallelism kernels (csrc/kernels/embedding.hip fm_sdp_*) against a float64 torch
oracle: coalescing a replica's lookups into (unique row, summed gradient) payloads, and applying
the gathered segments in rank order (no dense table gradient anywhere)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _oracle(idx, dy, rows, lo, scale):
    B, bag = idx.shape
    li = idx.long().reshape(-1) - lo
    ok = (li >= 0) & (li < rows)
    g = (dy.double() * scale).repeat_interleave(bag, 0)[ok]
    uniq, inv = torch.unique(li[ok], return_inverse=True)
    s = torch.zeros(uniq.numel(), dy.shape[1], dtype=torch.float64, device=dy.device).index_add_(0, inv, g)
    return uniq, s


@pytest.mark.parametrize("dy_dtype", [torch.float32, torch.bfloat16])
def test_sdp_coalesce_and_apply(dy_dtype):
    from flexmi.ops import _kernels as K
    dev = torch.device("cuda")
    torch.manual_seed(0)
    B = 1024
    # (rows held, D, bag, first row, index width): a large mostly-unique table, a tiny table with
    # thousands of duplicates per row, a bag-2 table, a row shard that sees out-of-shard lookups
    specs = [(50000, 128, 1, 0, torch.int64), (3, 64, 1, 0, torch.int32), (700, 32, 2, 0, torch.int64),
             (400, 128, 1, 300, torch.int64)]
    W, idx, dy, slot, cid, ids, g, cnt, lo, scale = [], [], [], [], [], [], [], [], [], []
    for rows, D, bag, l0, it in specs:
        W.append(torch.randn(rows, D, device=dev))
        hi = rows + l0 + (200 if l0 else 0)
        idx.append(torch.randint(0, hi, (B, bag), device=dev, dtype=it))
        dy.append(torch.randn(B, D, device=dev).to(dy_dtype))
        slot.append(torch.full((rows,), -1, dtype=torch.int32, device=dev))
        cid.append(torch.empty(B * bag, dtype=torch.int32, device=dev))
        ids.append(torch.zeros(B * bag, dtype=torch.int32, device=dev))
        g.append(torch.zeros(B * bag * D, dtype=torch.float32, device=dev))
        cnt.append(torch.zeros(1, dtype=torch.int32, device=dev))
        lo.append(l0)
        scale.append(0.5 if bag == 2 else 1.0)
    K.C().sdp_coalesce(W, idx, dy, [d.stride(0) for d in dy], scale, lo, slot, cid, ids, g, cnt)
    torch.cuda.synchronize()
    for k, (rows, D, bag, l0, _) in enumerate(specs):
        uniq, s = _oracle(idx[k], dy[k], rows, l0, scale[k])
        n = int(cnt[k].item())
        assert n == uniq.numel(), (k, n, uniq.numel())
        got_ids = ids[k][:n].long()
        order = torch.argsort(got_ids)
        assert torch.equal(got_ids[order], uniq)
        got = g[k][:n * D].view(n, D)[order].double()
        # fp32 sums in atomic (run-dependent) order: the 3-row table folds ~340 duplicates per row,
        # whose rounding reached 1.3e-5 absolute in one run -- bound it by the duplicate count
        dup = B * bag / max(1, uniq.numel())
        torch.testing.assert_close(got, s, rtol=1e-5, atol=1e-5 * max(1.0, dup ** 0.5))
    # apply two segments in order: own (0) and a peer's payload with unique rows
    lr = torch.tensor([0.05], device=dev)
    seg1_ids, seg1_g, seg1_cnt = [], [], []
    for rows, D, bag, l0, _ in specs:
        m = min(rows, 257)
        seg1_ids.append(torch.cat([torch.randperm(rows, device=dev)[:m].int(),
                                   torch.zeros(B * bag - m, dtype=torch.int32, device=dev)]))
        seg1_g.append(torch.randn(B * bag * D, device=dev))
        seg1_cnt.append(torch.tensor([m], dtype=torch.int32, device=dev))
    exp = []
    for k, (rows, D, bag, l0, _) in enumerate(specs):
        w = W[k].double().clone()
        n = int(cnt[k].item())
        w.index_add_(0, ids[k][:n].long(), -0.05 * g[k][:n * D].view(n, D).double())
        m = int(seg1_cnt[k].item())
        w.index_add_(0, seg1_ids[k][:m].long(), -0.05 * seg1_g[k][:m * D].view(m, D).double())
        exp.append(w)
    K.C().sdp_apply(W, ids + seg1_ids, g + seg1_g, cnt + seg1_cnt, slot, cnt, 2, 0, lr)
    torch.cuda.synchronize()
    for k in range(len(specs)):
        torch.testing.assert_close(W[k].double(), exp[k], rtol=1e-5, atol=1e-5)
        assert int((slot[k] != -1).sum().item()) == 0, "claim slots not released"
        assert int(cnt[k].item()) == 0, "own count not reset for the next step"


def test_sdp_step_is_repeatable():
    """Two consecutive coalesce+apply rounds on the same buffers (slots / counts recycled)."""
    from flexmi.ops import _kernels as K
    dev = torch.device("cuda")
    rows, D, B = 5000, 128, 2048
    W = torch.randn(rows, D, device=dev)
    slot = torch.full((rows,), -1, dtype=torch.int32, device=dev)
    cid = torch.empty(B, dtype=torch.int32, device=dev)
    ids = torch.zeros(B, dtype=torch.int32, device=dev)
    g = torch.zeros(B * D, dtype=torch.float32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    lr = torch.tensor([0.1], device=dev)
    w_ref = W.double().clone()
    for step in range(2):
        idx = torch.randint(0, rows, (B, 1), device=dev)
        dy = torch.randn(B, D, device=dev)
        uniq, s = _oracle(idx, dy, rows, 0, 1.0)
        w_ref.index_add_(0, uniq, -0.1 * s)
        K.C().sdp_coalesce([W], [idx], [dy], [D], [1.0], [0], [slot], [cid], [ids], [g], [cnt])
        K.C().sdp_apply([W], [ids], [g], [cnt], [slot], [cnt], 1, 0, lr)
    torch.cuda.synchronize()
    torch.testing.assert_close(W.double(), w_ref, rtol=1e-5, atol=1e-5)
