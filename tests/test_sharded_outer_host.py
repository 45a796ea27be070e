"""Host logic of the sample-sharded outer objective (no GPU): the sample
split, the per-rank noise slices in the reference draw order and the softmax
coefficients (checked against autograd of PSVI.psvi_elbo's combine,
psvi_classes.py:463-481)."""
import numpy as np
import pytest
import torch

from psvi.runtime.sharded import local_eps, outer_coefficients, pack_coef, sample_split


def test_sample_split():
    assert sample_split(128, 8) == [(16 * r, 16) for r in range(8)]
    assert sample_split(32, 5) == [(0, 7), (7, 7), (14, 6), (20, 6), (26, 6)]
    assert sum(c for _, c in sample_split(257, 8)) == 257


@pytest.mark.parametrize("family,layers", [
    ("meanfield", [(3, 4), (4, 2)]),
    ("fullcov", [(3, 4), (4, 2)]),
    ("lenet", [(25, 6), (150, 16), (400, 120), (120, 84), (84, 10)]),
])
def test_local_eps_is_a_sample_slice(family, layers):
    S = 5
    per_layer = []                  # draw order: per layer, the S-batched blocks
    for l, (din, dout) in enumerate(layers):
        if family == "fullcov":
            per_layer.append([torch.randn(S, din * dout + dout)])
        elif family == "lenet" and l == len(layers) - 1:
            per_layer.append([torch.randn(1, din * dout + dout)])   # one shared draw
        else:
            per_layer.append([torch.randn(S, dout, din), torch.randn(S, dout)])
    eps = torch.cat([b.reshape(-1) for blocks in per_layer for b in blocks])
    for off, cnt in sample_split(S, 2):
        got = local_eps(family, layers, S, off, cnt, eps)
        want = torch.cat([(b if b.shape[0] == 1 else b[off:off + cnt]).reshape(-1)
                          for blocks in per_layer for b in blocks])
        assert torch.equal(got, want)


def test_outer_coefficients_are_the_loss_derivatives():
    g = torch.Generator().manual_seed(0)
    terms = (torch.randn(37, 3, generator=g, dtype=torch.float64) * 3).requires_grad_()
    loss, cp, cd, ck = outer_coefficients(terms)
    # PSVI.psvi_elbo: lw = nkl - pseudo; W = softmax(lw); loss = sum W (data - pseudo) - mean lw
    pseudo, data, nkl = terms.unbind(1)
    lw = nkl - pseudo
    ref = (torch.softmax(lw, 0) * (data - pseudo)).sum() - lw.mean()
    assert abs(loss.item() - ref.item()) < 1e-12
    gr, = torch.autograd.grad(ref, terms)
    np.testing.assert_allclose(torch.stack([cp, cd, ck], 1).detach(), gr, rtol=1e-10,
                               atol=1e-12)
    c = pack_coef(cp.detach(), cd.detach(), ck.detach(), 10, 4)
    assert c.dtype == torch.float32 and c.numel() == 13
    np.testing.assert_allclose(c[8:12], ck.detach()[10:14].float())
    assert abs(c[12].item() - ck.detach()[10:14].sum().item()) < 1e-6
