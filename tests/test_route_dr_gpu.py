"""GPU parity of the fused window+pose+DR layer (srf_route_dr_fwd/bwd, through
the C ABI) against the CPU oracle.

Forward: numpy float64 restatement of sequence_router_naive.py:150-185.
Backward: float64 autograd of the op-for-op torch mirror (oracle/naive_mirror).
Tolerances (fp32 kernel vs fp64 oracle): forward |err| <= 2e-5 * (1 + |ref|),
gradients |err| <= 1e-4 * max|ref| (fp32 reassociation over up to in_n*J terms).
"""
import numpy as np
import pytest
import torch

from oracle import srf_oracle as so
from oracle import naive_mirror as nm

pytestmark = pytest.mark.gpu

CASES = [
    # B, T, N, D, lpad, rpad, J, iters, mask_first
    (2, 13, 8, 16, 4, 4, 8, 3, False),    # C2 layers 1-2 shape (short)
    (2, 11, 8, 16, 4, 4, 63, 3, True),    # C2 last layer (short)
    (1, 7, 4, 8, 0, 0, 63, 1, True),      # C1 single layer
    (3, 9, 16, 32, 2, 2, 16, 3, False),   # C3/C4 inner layer
    (2, 6, 16, 32, 2, 2, 32, 3, True),    # C3/C4 last layer
    (1, 5, 3, 16, 1, 2, 5, 2, True),      # ragged odd sizes
    (1, 5, 2, 64, 1, 1, 4, 2, True),      # C5-width capsules (DIM=64)
    (2, 7, 4, 8, 1, 1, 6, 5, False),      # 5 routing iterations
    (3, 37, 8, 16, 4, 4, 63, 3, True),    # several 32-frame tiles, ragged last tile
    (2, 21, 4, 8, 2, 1, 12, 3, False),    # din 8 -> dout 8 with a partial 32-row tile
    # din = dout = 32 on the split-fp16 gx / gW passes (route_gux16 / route_gw16s): two
    # iterations, J not a multiple of a workgroup's 4 output capsules, partial frame tiles
    (1, 35, 8, 32, 1, 2, 8, 2, True),
    (2, 17, 4, 32, 1, 1, 6, 3, True),
    (3, 61, 8, 32, 2, 2, 12, 3, False),
]


def _mk(case, seed):
    B, T, N, D, lp, rp, J, it, mf = case
    rng = np.random.default_rng(seed)
    in_n = N * (lp + rp + 1)
    emb = rng.standard_normal((B, T, N, D)) * 0.5
    W = rng.standard_normal((in_n, J, D, D)) * 0.1
    bias = rng.standard_normal((in_n, J, D)) * 0.1
    return emb, W, bias


def _run_gpu(case, emb, W, bias, dev, n_chunks=0, store_couplings=True):
    from srf_amd.ops import RouteGeom, dynamic_routing
    B, T, N, D, lp, rp, J, it, mf = case
    g = RouteGeom(B, T, N, D, lp, rp, J, D, it, mf, n_chunks)
    g.store_couplings = store_couplings
    te = torch.tensor(emb, dtype=torch.float32, device=dev, requires_grad=True)
    tW = torch.tensor(W, dtype=torch.float32, device=dev, requires_grad=True)
    tb = torch.tensor(bias, dtype=torch.float32, device=dev, requires_grad=True)
    v = dynamic_routing(te, tW, tb, g)
    return te, tW, tb, v


@pytest.mark.parametrize('case', CASES)
def test_route_dr_forward(cuda, case):
    emb, W, bias = _mk(case, 1)
    _, _, _, v = _run_gpu(case, emb, W, bias, cuda)
    B, T, N, D, lp, rp, J, it, mf = case
    ref = so.dynamic_routing(so.pose(so.window(emb, lp, rp), W, bias), it, mf)
    got = v.detach().cpu().double().numpy()
    assert np.all(np.abs(got - ref) <= 2e-5 * (1 + np.abs(ref))), np.abs(got - ref).max()


@pytest.mark.parametrize('case', CASES)
def test_route_dr_backward(cuda, case):
    emb, W, bias = _mk(case, 2)
    te, tW, tb, v = _run_gpu(case, emb, W, bias, cuda)
    rng = np.random.default_rng(3)
    gv = rng.standard_normal(v.shape)
    v.backward(torch.tensor(gv, dtype=torch.float32, device=cuda))
    B, T, N, D, lp, rp, J, it, mf = case
    ce = torch.tensor(emb, requires_grad=True)
    cW = torch.tensor(W, requires_grad=True)
    cb = torch.tensor(bias, requires_grad=True)
    ep = torch.nn.functional.pad(ce, (0, 0, 0, 0, lp, rp))
    xw = torch.cat([ep[:, w:w + T] for w in range(lp + rp + 1)], dim=2)
    vr = nm.dynamic_routing(nm.pose_tiled(xw, cW, cb), it, mf)
    vr.backward(torch.tensor(gv))
    for name, got, ref in (('g_emb', te.grad, ce.grad), ('g_W', tW.grad, cW.grad), ('g_bias', tb.grad, cb.grad)):
        got = got.cpu().double().numpy()
        ref = ref.numpy()
        err = np.abs(got - ref).max()
        assert err <= 1e-4 * max(1.0, np.abs(ref).max()), (name, err, np.abs(ref).max())


@pytest.mark.parametrize('case,chunks', [((2, 11, 8, 16, 4, 4, 63, 3, True), (1, 5, 72)),
                                         ((2, 40, 16, 32, 2, 2, 16, 3, False), (1, 3, 80))])
def test_route_dr_chunking_invariant(cuda, case, chunks):
    """The i-chunk split (RouteGeom n_chunks, an explicit plan argument) is a pure
    work decomposition: forward and gradients agree for any chunk count."""
    emb, W, bias = _mk(case, 4)
    gv = torch.tensor(np.random.default_rng(5).standard_normal(case[:2] + (case[6], case[3])), dtype=torch.float32,
                      device=cuda)
    outs = []
    for nc in chunks:
        te, tW, tb, v = _run_gpu(case, emb, W, bias, cuda, nc)
        v.backward(gv)
        outs.append([v.detach().cpu().double().numpy()] + [t.grad.cpu().double().numpy() for t in (te, tW, tb)])
    for o in outs[1:]:
        assert np.abs(outs[0][0] - o[0]).max() < 1e-5
        for a, b in zip(outs[0][1:], o[1:]):
            assert np.abs(a - b).max() <= 2e-5 * max(1.0, np.abs(a).max())


@pytest.mark.parametrize('case', [(3, 37, 8, 16, 4, 4, 63, 3, True), (2, 19, 8, 16, 4, 4, 8, 3, False),
                                  (2, 21, 4, 8, 2, 1, 12, 3, False), (2, 7, 4, 8, 1, 1, 6, 5, False),
                                  (2, 40, 16, 32, 2, 2, 16, 3, False), (2, 23, 16, 32, 2, 2, 32, 3, True),
                                  (1, 9, 4, 32, 1, 1, 8, 5, False)])
def test_route_dr_backward_from_stored_couplings(cuda, case):
    """The backward routing passes that read the forward's stored couplings
    (route_bwd32_kernel and the passes behind it) against the ones that recompute the
    logits (route_pass_kernel: a forward that stores no couplings, RouteGeom
    store_couplings=False): same gradients to fp32 accuracy."""
    emb, W, bias = _mk(case, 6)
    gv = torch.tensor(np.random.default_rng(7).standard_normal(case[:2] + (case[6], case[3])), dtype=torch.float32,
                      device=cuda)
    grads = []
    for flag in (True, False):
        te, tW, tb, v = _run_gpu(case, emb, W, bias, cuda, store_couplings=flag)
        v.backward(gv)
        grads.append([t.grad.detach().cpu().double().numpy() for t in (te, tW, tb)])
    for a, b, name in zip(grads[0], grads[1], ('g_emb', 'g_W', 'g_bias')):
        assert np.abs(a - b).max() <= 2e-5 * max(1.0, np.abs(b).max()), (name, np.abs(a - b).max())


@pytest.mark.parametrize('case', [(2, 37, 8, 16, 4, 4, 63, 3, True), (2, 23, 16, 32, 2, 2, 16, 3, False),
                                  (2, 21, 4, 8, 2, 1, 12, 3, False)])
def test_route_dr_skewed_operand_magnitudes(cuda, case):
    """The split-fp16 pose scales each operand tensor by one power of two
    (route_fwd32.hip prep32_kernel), so rows far below the tensor's maximum land in
    fp16's subnormal range.  W rows (per input capsule i, output capsule j) and
    emb frames spanning 2^-20 .. 2^4, with all-zero padded frames, against the
    fp64 oracle: forward and gradients at the layer tests' tolerances."""
    B, T, N, D, lp, rp, J, it, mf = case
    emb, W, bias = _mk(case, 12)
    rng = np.random.default_rng(13)
    W = W * np.exp2(rng.uniform(-20, 4, size=W.shape[:2]))[:, :, None, None]
    emb = emb * np.exp2(rng.uniform(-20, 4, size=(B, T)))[:, :, None, None]
    emb[:, T - 3:] = 0.0                               # padded frames
    emb[0, 1] *= 0.0
    te, tW, tb, v = _run_gpu(case, emb, W, bias, cuda)
    ref = so.dynamic_routing(so.pose(so.window(emb, lp, rp), W, bias), it, mf)
    got = v.detach().cpu().double().numpy()
    assert np.all(np.abs(got - ref) <= 2e-5 * (1 + np.abs(ref))), np.abs(got - ref).max()
    gv = rng.standard_normal(v.shape)
    v.backward(torch.tensor(gv, dtype=torch.float32, device=cuda))
    ce, cW, cb = (torch.tensor(a, requires_grad=True) for a in (emb, W, bias))
    ep = torch.nn.functional.pad(ce, (0, 0, 0, 0, lp, rp))
    xw = torch.cat([ep[:, w:w + T] for w in range(lp + rp + 1)], dim=2)
    nm.dynamic_routing(nm.pose_tiled(xw, cW, cb), it, mf).backward(torch.tensor(gv))
    for name, g, r in (('g_emb', te.grad, ce.grad), ('g_W', tW.grad, cW.grad), ('g_bias', tb.grad, cb.grad)):
        g, r = g.cpu().double().numpy(), r.numpy()
        err = np.abs(g - r).max()
        assert err <= 1e-4 * max(1.0, np.abs(r).max()), (name, err, np.abs(r).max())
