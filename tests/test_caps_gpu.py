"""GPU parity of the capsule glue kernels (primary capsules, per-layer LN +
dropout, output head) and of the CTC kernel, through the C ABI, against float64
torch-autograd restatements (tests/torch_ref.py) with bit-identical dropout
masks.  Tolerances: values |err| <= 1e-4 * (1 + |ref|); gradients
|err| <= 1e-3 * max|ref| + 1e-6; CTC NLL within 1e-4 relative."""
import numpy as np
import pytest
import torch

from tests import torch_ref as tr

pytestmark = pytest.mark.gpu


def _cmp(got, ref, rtol):
    g = got.detach().cpu().double().numpy()
    r = ref.detach().cpu().double().numpy()
    return np.abs(g - r).max() <= rtol * (1 + np.abs(r).max()), np.abs(g - r).max()


@pytest.mark.parametrize('PH,PD,p', [(8, 16, 0.0), (8, 16, 0.2), (4, 8, 0.1), (16, 32, 0.2)])
def test_primary_caps(cuda, PH, PD, p):
    from srf_amd import ops
    B, T, F2, C = 3, 11, 31, 64
    rng = np.random.default_rng(PH + PD)
    X = rng.standard_normal((B, T, F2, C))
    inp_len = np.array([44, 37, 20], dtype=np.int32)   # -> 11, 10, 5 valid frames
    g = torch.Generator().manual_seed(1)
    P = {'proj_kernel': torch.randn(F2 * C, PH, generator=g, dtype=torch.float64) * 0.05,
         'proj_bias': torch.randn(PH, generator=g, dtype=torch.float64) * 0.1,
         'encaps1_kernel': torch.randn(3, 3, 1, PD, generator=g, dtype=torch.float64) * 0.3,
         'encaps1_bias': torch.randn(PD, generator=g, dtype=torch.float64) * 0.1,
         'encaps2_kernel': torch.randn(3, 3, 1, PD, generator=g, dtype=torch.float64) * 0.3,
         'encaps2_bias': torch.randn(PD, generator=g, dtype=torch.float64) * 0.1,
         'ln_input_gamma': 1 + 0.1 * torch.randn(PH * PD, generator=g, dtype=torch.float64),
         'ln_input_beta': 0.1 * torch.randn(PH * PD, generator=g, dtype=torch.float64)}
    seed = 99
    drop = None
    if p > 0:
        drop = {'encaps1': torch.tensor(tr.dropout_mult(seed, 4, (B, T, PH, PD), 0.2)),
                'encaps2': torch.tensor(tr.dropout_mult(seed, 5, (B, T, PH, PD), 0.2)),
                'input': torch.tensor(tr.dropout_mult(seed, 6, (B, T, PH * PD), p))}
    Pr = {k: v.clone().requires_grad_() for k, v in P.items()}
    Xr = torch.tensor(X, requires_grad=True)
    ref = tr.primary_caps(Xr, torch.tensor(inp_len), Pr, PH, PD, drop)
    gz = torch.tensor(rng.standard_normal(ref.shape))
    (ref * gz).sum().backward()
    Pg = {k: v.float().to(cuda).requires_grad_() for k, v in P.items()}
    Xg = torch.tensor(X, dtype=torch.float32, device=cuda, requires_grad=True)
    z = ops.primary_caps(Xg, torch.tensor(inp_len, device=cuda), PH, PD, True, 0.2 if p > 0 else 0.0, p, seed,
                         [Pg[k] for k in ops.CAPS_PARAMS])
    ok, err = _cmp(z, ref, 1e-4)
    assert ok, err
    (z * gz.float().to(cuda)).sum().backward()
    for name, got, want in [('X', Xg.grad, Xr.grad)] + [(k, Pg[k].grad, Pr[k].grad) for k in ops.CAPS_PARAMS]:
        e = (got.cpu().double() - want).abs().max().item()
        assert e <= 1e-3 * want.abs().max().item() + 1e-6, (name, e)


@pytest.mark.parametrize('head,J,D', [(False, 8, 16), (True, 63, 16),
                                      # the wave-per-row kernels: rows of 256, 512, 1024 values
                                      (False, 16, 16), (False, 16, 32), (False, 32, 32),
                                      (True, 16, 16), (True, 32, 32)])
@pytest.mark.parametrize('p', [0.0, 0.1])
def test_capsnorm_and_head(cuda, head, J, D, p):
    from srf_amd import ops
    B, T = 2, 9   # 18 rows: the last four-row workgroup of the wave kernels is partial
    rng = np.random.default_rng(3)
    v = rng.standard_normal((B, T, J, D)) * 0.3
    g = torch.Generator().manual_seed(2)
    gm = 1 + 0.1 * torch.randn(J * D, generator=g, dtype=torch.float64)
    bm = 0.1 * torch.randn(J * D, generator=g, dtype=torch.float64)
    go = 1 + 0.1 * torch.randn(J, generator=g, dtype=torch.float64)
    bo = 0.1 * torch.randn(J, generator=g, dtype=torch.float64)
    seed, layer = 5, 2
    drop = torch.tensor(tr.dropout_mult(seed, 7 + layer, (B, T, J * D), p)) if p > 0 else None
    ts = [torch.tensor(v, requires_grad=True)] + [t.clone().requires_grad_() for t in (gm, bm, go, bo)]
    tg = [t.detach().float().to(cuda).requires_grad_() for t in ts]
    if head:
        ref = tr.caps_head(*ts, drop)
        out = ops.CapsHead.apply(*tg, True, p, seed, layer)
    else:
        ref = tr.capsnorm(ts[0], ts[1], ts[2], drop)
        out = ops.CapsNorm.apply(tg[0], tg[1], tg[2], True, p, seed, layer)
    ok, err = _cmp(out, ref, 1e-4)
    assert ok, err
    w = torch.tensor(rng.standard_normal(ref.shape))
    (ref * w).sum().backward()
    (out * w.float().to(cuda)).sum().backward()
    n = 5 if head else 3
    for i in range(n):
        e = (tg[i].grad.cpu().double() - ts[i].grad).abs().max().item()
        assert e <= 1e-3 * ts[i].grad.abs().max().item() + 1e-6, (i, e)


def test_ctc_matches_torch(cuda):
    from srf_amd import ops
    B, T, C = 4, 23, 9
    rng = np.random.default_rng(4)
    logits = rng.standard_normal((B, T, C)) * 2
    labels = np.array([[1, 1, 2, 3, 0], [4, 5, 5, 6, 7], [2, 0, 0, 0, 0], [3, 3, 3, 3, 3]], dtype=np.int32)
    lab_len = np.array([4, 5, 1, 5], dtype=np.int32)
    logit_len = np.array([23, 17, 3, 9], dtype=np.int32)   # utt 3: 5 repeats need 9 frames (feasible)
    lr = torch.tensor(logits, requires_grad=True)
    ref = torch.nn.functional.ctc_loss(torch.log_softmax(lr, -1).transpose(0, 1), torch.tensor(labels).long(),
                                       torch.tensor(logit_len).long(), torch.tensor(lab_len).long(), blank=C - 1,
                                       reduction='none')
    ref.sum().backward()
    lg = torch.tensor(logits, dtype=torch.float32, device=cuda, requires_grad=True)
    nll = ops.ctc_loss(lg, torch.tensor(labels, device=cuda), torch.tensor(lab_len, device=cuda),
                       torch.tensor(logit_len, device=cuda), C - 1)
    assert np.allclose(nll.detach().cpu().numpy(), ref.detach().numpy(), rtol=1e-4, atol=1e-4)
    nll.sum().backward()
    # fp32 recursions over 90-420 frames: gradient entries agree to 5e-4 absolute
    e = (lg.grad.cpu().double() - lr.grad).abs().max().item()
    assert e < 1e-4, e


def test_ctc_infeasible_is_inf_with_zero_grad(cuda):
    from srf_amd import ops
    lg = torch.zeros(1, 4, 5, device=cuda, requires_grad=True)
    nll = ops.ctc_loss(lg, torch.tensor([[1, 1, 1]], device=cuda), torch.tensor([3], device=cuda),
                       torch.tensor([4], device=cuda), 4)
    assert torch.isinf(nll).all()
    nll.sum().backward()
    assert torch.count_nonzero(lg.grad) == 0


@pytest.mark.parametrize('B,T,C,L', [(3, 150, 12, 70), (2, 420, 32, 200), (2, 90, 63, 40),
                                     (1, 2100, 32, 1000),    # block loop; gradient stages 4 frames per block
                                     (1, 11300, 8, 5600)])   # gradient reads alpha/beta from HBM
def test_ctc_long_labels_cross_state_groups(cuda, B, T, C, L):
    """Extended-label lengths past 64 states exercise the group boundaries of the
    wave-resident recursion (KM = 4, 8); past 512 states the block loop runs.  The
    longest cases exceed the gradient kernel's 16-frame LDS staging (fewer frames
    per block, then no staging)."""
    from srf_amd import ops
    rng = np.random.default_rng(B * 1000 + T)
    logits = rng.standard_normal((B, T, C)) * 2
    lab_len = rng.integers(L // 2, L + 1, size=B).astype(np.int32)
    lab_len[0] = L
    labels = rng.integers(0, C - 1, size=(B, L)).astype(np.int32)
    logit_len = np.array([T] + [int(rng.integers(2 * L + 1, T + 1)) for _ in range(B - 1)], dtype=np.int32)
    lr = torch.tensor(logits, requires_grad=True)
    ref = torch.nn.functional.ctc_loss(torch.log_softmax(lr, -1).transpose(0, 1), torch.tensor(labels).long(),
                                       torch.tensor(logit_len).long(), torch.tensor(lab_len).long(), blank=C - 1,
                                       reduction='none')
    ref.sum().backward()
    lg = torch.tensor(logits, dtype=torch.float32, device=cuda, requires_grad=True)
    nll = ops.ctc_loss(lg, torch.tensor(labels, device=cuda), torch.tensor(lab_len, device=cuda),
                       torch.tensor(logit_len, device=cuda), C - 1)
    got = nll.detach().cpu().double().numpy()
    assert np.all(np.abs(got - ref.detach().numpy()) <= 1e-4 * np.maximum(1, np.abs(ref.detach().numpy()))), got
    nll.sum().backward()
    # fp32 log-space recursions over T frames: gradient entries agree to 2e-6 * T
    # absolute, or to twice the error of torch's own fp32 CTC (whose rounding grows
    # with the log-likelihood's magnitude over very long utterances)
    lr32 = torch.tensor(logits, dtype=torch.float32, requires_grad=True)
    torch.nn.functional.ctc_loss(torch.log_softmax(lr32, -1).transpose(0, 1), torch.tensor(labels).long(),
                                 torch.tensor(logit_len).long(), torch.tensor(lab_len).long(), blank=C - 1,
                                 reduction='none').sum().backward()
    e32 = (lr32.grad.double() - lr.grad).abs().max().item()
    e = (lg.grad.cpu().double() - lr.grad).abs().max().item()
    assert e < max(2e-6 * T, 2 * e32), (e, e32)
