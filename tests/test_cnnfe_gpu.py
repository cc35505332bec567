"""GPU parity of the HIP CNN front end (srf_cnnfe_fwd/bwd through the C ABI)
against a float64 torch-autograd restatement of CapsulationLayer
(sequence_router.py:44-82).  Dropout masks are regenerated on the host from the
same counter-based RNG (tests/torch_ref.dropout_mult_pair: both maxout branches from one hash).

Tolerances: output |err| <= 2e-4 * (1 + |ref|) (fp32 conv + BN normalisation
vs fp64); parameter gradients |err| <= 2e-3 * max|ref| (fp32 reductions over
up to 1e5 positions, rare maxout near-ties)."""
import numpy as np
import pytest
import torch

from tests import torch_ref as tr

pytestmark = pytest.mark.gpu

CASES = [  # B, T, lengths, dropout
    (3, 37, [37, 30, 21], 0.0),
    (2, 40, [40, 33], 0.2),
    (4, 64, [64, 64, 50, 7], 0.0),
]


def _params(seed, dtype=torch.float64):
    g = torch.Generator().manual_seed(seed)
    P = {}
    cin = 1
    for k in range(2):
        for ab in 'ab':
            lim = (6.0 / (9 * cin + 9 * 64)) ** 0.5
            P[f'conv{k}{ab}_kernel'] = (torch.rand(3, 3, cin, 64, generator=g, dtype=dtype) * 2 - 1) * lim
            P[f'conv{k}{ab}_bias'] = 0.05 * torch.randn(64, generator=g, dtype=dtype)
        P[f'bn{k}_gamma'] = 1 + 0.1 * torch.randn(64, generator=g, dtype=dtype)
        P[f'bn{k}_beta'] = 0.1 * torch.randn(64, generator=g, dtype=dtype)
        cin = 64
    return P


@pytest.mark.parametrize('case', CASES)
def test_cnnfe_forward_backward(cuda, case):
    from srf_amd import ops
    B, T, lens, p = case
    seed = 77
    P = _params(5)
    rng = np.random.default_rng(9)
    feats = rng.standard_normal((B, T, 123))
    for b, l in enumerate(lens):
        feats[b, l:] = 0
    inp_len = np.array(lens, dtype=np.int32)
    T1, F1 = -(-T // 2), 62
    T2, F2 = -(-T1 // 2), 31
    drop = None
    if p > 0:
        drop = {}
        for k, (Tk, Fk) in enumerate(((T1, F1), (T2, F2))):
            ma, mb = tr.dropout_mult_pair(seed, tr.STREAMS[f'conv{k}a'], (B, Tk, Fk, 64), p)
            drop[f'conv{k}a'] = torch.tensor(ma)
            drop[f'conv{k}b'] = torch.tensor(mb)
    # reference (fp64, CPU)
    Pr = {k: v.clone().requires_grad_() for k, v in P.items()}
    ref = tr.cnnfe(torch.tensor(feats), torch.tensor(inp_len), Pr, drop)
    gout = torch.tensor(rng.standard_normal(ref.shape))
    (ref * gout).sum().backward()
    # HIP
    Pg = {k: v.float().to(cuda).requires_grad_() for k, v in P.items()}
    moving = [torch.zeros(64, device=cuda), torch.ones(64, device=cuda), torch.zeros(64, device=cuda),
              torch.ones(64, device=cuda)]
    out = ops.cnnfe(torch.tensor(feats, dtype=torch.float32, device=cuda), torch.tensor(inp_len, device=cuda),
                    [Pg[k] for k in ops.CNNFE_PARAMS], moving, True, p, seed)
    got = out.detach().cpu().double().numpy()
    r = ref.detach().numpy()
    assert got.shape == r.shape
    assert np.all(np.abs(got - r) <= 2e-4 * (1 + np.abs(r))), np.abs(got - r).max()
    (out * gout.float().to(cuda)).sum().backward()
    bad = []
    for k in ops.CNNFE_PARAMS:
        gr = Pr[k].grad.numpy()
        gg = Pg[k].grad.detach().cpu().double().numpy()
        err = np.abs(gg - gr).max()
        if err > 2e-3 * np.abs(gr).max() + 1e-6:
            bad.append((k, err, np.abs(gr).max()))
    assert not bad, bad
    # moving statistics: 0.99 * init + 0.01 * batch statistic (unbiased variance)
    assert torch.all(moving[0].abs() > 0) and torch.all(moving[1] != 1.0)


def test_cnnfe_inference_uses_moving_stats(cuda):
    from srf_amd import ops
    P = _params(6)
    rng = np.random.default_rng(10)
    B, T = 2, 24
    feats = rng.standard_normal((B, T, 123))
    inp_len = np.array([24, 24], dtype=np.int32)
    mm = [0.1 * torch.randn(64, dtype=torch.float64), 1 + 0.2 * torch.rand(64, dtype=torch.float64)] * 2
    # reference with fixed statistics
    x = torch.tensor(feats).unsqueeze(-1)
    for k in range(2):
        y = torch.maximum(tr.conv2d_same(x, P[f'conv{k}a_kernel'], P[f'conv{k}a_bias'], 2),
                          tr.conv2d_same(x, P[f'conv{k}b_kernel'], P[f'conv{k}b_bias'], 2))
        x = (y - mm[2 * k]) / torch.sqrt(mm[2 * k + 1] + 1e-3) * P[f'bn{k}_gamma'] + P[f'bn{k}_beta']
    moving = [t.float().to(cuda) for t in mm]
    out = ops.cnnfe(torch.tensor(feats, dtype=torch.float32, device=cuda), torch.tensor(inp_len, device=cuda),
                    [P[k].float().to(cuda) for k in ops.CNNFE_PARAMS], moving, False, 0.2, 1)
    assert np.abs(out.cpu().double().numpy() - x.numpy()).max() < 2e-4 * (1 + np.abs(x.numpy()).max())
    assert torch.allclose(moving[0].cpu().double(), mm[0].float().double())   # untouched



def test_cnnfe_wgrad_side_stream_bitwise(cuda):
    """ops.CNNFE_WGRAD_SIDE: srf_cnnfe_bwd_parts PREP + DATA on the backward's stream and
    WGRAD deferred onto the side stream (joined by the end-of-backward callback) gives
    the gradients of the one-call srf_cnnfe_bwd bit for bit (same kernels, same inputs),
    read right after backward() without an explicit join."""
    from srf_amd import ops
    B, T, lens, p = CASES[1]
    P = _params(5)
    rng = np.random.default_rng(11)
    feats = torch.tensor(rng.standard_normal((B, T, 123)), dtype=torch.float32, device=cuda)
    inp_len = torch.tensor(lens, dtype=torch.int32, device=cuda)
    grads = []
    for side in (False, True):
        ops.CNNFE_WGRAD_SIDE = side
        try:
            Pg = {}
            for k, v in P.items():
                t = v.float().to(cuda).requires_grad_()
                t.grad = torch.full_like(t, float('nan'))   # written in place (flat-buffer views in the model)
                t._srf_flat = True
                Pg[k] = t
            moving = [torch.zeros(64, device=cuda), torch.ones(64, device=cuda)] * 2
            out = ops.cnnfe(feats, inp_len, [Pg[k] for k in ops.CNNFE_PARAMS], moving, True, p, 77)
            g = torch.tensor(rng.standard_normal(out.shape) if not grads else gout, dtype=torch.float32)
            gout = g.numpy()
            (out * g.to(cuda)).sum().backward()
            grads.append({k: Pg[k].grad.cpu().clone() for k in ops.CNNFE_PARAMS})
        finally:
            ops.CNNFE_WGRAD_SIDE = True
    for k in ops.CNNFE_PARAMS:
        assert torch.isfinite(grads[1][k]).all(), k
        assert torch.equal(grads[0][k], grads[1][k]), (k, (grads[0][k] - grads[1][k]).abs().max())
