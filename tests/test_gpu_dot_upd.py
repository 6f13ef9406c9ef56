"""Embedding sparse-SGD update fused into the fp32 interaction backward (csrc/kernels/interaction.hip
fm_dot_interaction_bwd_f32_upd + the count pass fm_embedding_count): against a float64 oracle of
the interaction backward followed by W[idx] -= lr * scale * dZ, over tables updated through the
count slots (rows hit once: plain store; repeated rows: atomics), slot-less tables (atomics),
tables left to their own backward (dZ written), the dense feature with its activation backward,
two steps (the slots must be re-armed to -1), int32 and int64 indices."""
import pytest
import torch

from tests.test_gpu_fp32 import rel_err

pytestmark = pytest.mark.gpu


def _oracle_dz(zs, dy, selfi):
    F = len(zs)
    D = zs[0].shape[1]
    B = zs[0].shape[0]
    Z = torch.stack([z.double() for z in zs], 1)
    li, lj = zip(*[(i, j) for i in range(F) for j in range(i + (1 if selfi else 0))])
    npairs = len(li)
    dG = torch.zeros(B, F, F, dtype=torch.float64, device=zs[0].device)
    dG[:, li, lj] = dy[:, D:D + npairs].double()
    dZ = (dG + dG.transpose(1, 2)) @ Z
    dZ[:, 0] += dy[:, :D].double()
    return dZ


@pytest.mark.parametrize("B,i64", [(8192, True), (1000, False)])
def test_fused_update_matches_oracle(gpu, B, i64):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(B)
    D, F = 128, 27
    # per table feature: (rows, mode) -- mode "count" (slots), "atomic" (no slots), "dz" (unfused)
    spec = [(40000, "count"), (3000, "count"), (12000, "count"), (500, "atomic"), (90, "atomic"), (7, "dz"),
            (64, "dz"), (200000, "count"), (1500, "count")] * 3
    spec = spec[:F - 1]
    idt = torch.int64 if i64 else torch.int32
    lr = torch.tensor([0.05], device=gpu)
    tables, idxs, slots, owns, W0 = [], [], [], [], []
    for rows, mode in spec:
        w = torch.randn(rows, D, device=gpu) * 0.1
        tables.append(w)
        W0.append(w.double().clone())
        slots.append(torch.full((rows,), -1, dtype=torch.int32, device=gpu) if mode == "count" else None)
        owns.append(torch.zeros(B, dtype=torch.int32, device=gpu) if mode == "count" else None)
    x = torch.randn(B, D, device=gpu)
    dzs = [torch.zeros(B, D, device=gpu) for _ in range(F)]
    scales = [1.0 if k % 2 else 0.5 for k in range(F - 1)]
    for step in range(2):
        idxs = []
        for rows, _ in spec:
            # skewed: hot rows repeat (atomics), the tail stays mostly unique (plain stores)
            hot = torch.randint(0, max(1, rows // 50), (B,), device=gpu)
            cold = torch.randint(0, rows, (B,), device=gpu)
            pick = torch.rand(B, device=gpu) < 0.3
            idxs.append(torch.where(pick, hot, cold).to(idt).view(B, 1).contiguous())
        # the forward's lookups (the interaction inputs are the looked-up rows)
        zs = [x] + [t[ix.view(-1).long()].clone() for t, ix in zip(tables, idxs)]
        npairs = F * (F - 1) // 2
        W = D + npairs
        dy = torch.randn(B, (W + 3) // 4 * 4, device=gpu)
        dZ = _oracle_dz(zs, dy, False)
        dZ[:, 0] *= (zs[0].double() > 0)      # act0 = relu on the dense feature
        exp = []
        for k, (t, ix) in enumerate(zip(W0, idxs)):
            if spec[k][1] == "dz":
                exp.append(t)
                continue
            t = t.clone()
            t.index_add_(0, ix.view(-1).long(), -0.05 * scales[k] * dZ[:, k + 1])
            exp.append(t)
        cnt = [k for k, (_, m) in enumerate(spec) if m == "count"]
        Kk.C().embedding_count([idxs[k] for k in cnt], [0] * len(cnt), [spec[k][0] for k in cnt], [slots[k] for k in cnt],
                               [owns[k] for k in cnt])
        # the descriptor holds the index pointers: rebuilt for this step's index tensors
        desc = Kk.C().dot_upd_desc([None] + [t if m != "dz" else None for t, (_, m) in zip(tables, spec)],
                                   [None] + [ix if m != "dz" else None for ix, (_, m) in zip(idxs, spec)],
                                   [None] + slots, [None] + owns, [0] * F, [1.0] + scales, lr)
        ok = Kk.C().dot_bwd_upd(zs, D, dy, dy.shape[1], dzs, D, D, False, 11, desc)
        assert ok
        torch.cuda.synchronize()
        assert rel_err(dzs[0], dZ[:, 0]) < 1e-5
        errs = []
        for k, (rows, mode) in enumerate(spec):
            ids = idxs[k].view(-1).long()
            cnt_ = torch.bincount(ids, minlength=rows)
            once = (cnt_ == 1).nonzero().view(-1)
            many = (cnt_ > 1).nonzero().view(-1)
            untouched = (cnt_ == 0).nonzero().view(-1)
            e1 = rel_err(tables[k][once], exp[k][once]) if once.numel() else 0.0
            e2 = rel_err(tables[k][many], exp[k][many]) if many.numel() else 0.0
            e0 = rel_err(tables[k][untouched], exp[k][untouched]) if untouched.numel() else 0.0
            errs.append((k, mode, round(e1, 7), round(e2, 7), round(e0, 7)))
        print("per-table errors (once, repeated, untouched):", errs)
        for k, (rows, mode) in enumerate(spec):
            assert rel_err(tables[k], exp[k]) < 1e-5, (step, k, mode)
            if mode == "dz":
                assert rel_err(dzs[k + 1], dZ[:, k + 1]) < 1e-5, (step, k)
            if mode == "count":
                assert bool((slots[k] == -1).all()), ("slots not re-armed", step, k)
        W0 = [t.double().clone() for t in tables]
