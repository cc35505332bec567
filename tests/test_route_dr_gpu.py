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
]


def _mk(case, seed):
    B, T, N, D, lp, rp, J, it, mf = case
    rng = np.random.default_rng(seed)
    in_n = N * (lp + rp + 1)
    emb = rng.standard_normal((B, T, N, D)) * 0.5
    W = rng.standard_normal((in_n, J, D, D)) * 0.1
    bias = rng.standard_normal((in_n, J, D)) * 0.1
    return emb, W, bias


def _run_gpu(case, emb, W, bias, dev, n_chunks=0):
    from srf_amd.ops import RouteGeom, dynamic_routing
    B, T, N, D, lp, rp, J, it, mf = case
    g = RouteGeom(B, T, N, D, lp, rp, J, D, it, mf, n_chunks)
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


def test_route_dr_chunking_invariant(cuda):
    """The i-chunk split is a pure work decomposition: results must agree."""
    case = (2, 11, 8, 16, 4, 4, 63, 3, True)
    emb, W, bias = _mk(case, 4)
    outs = []
    for nc in (1, 5, 72):
        _, _, _, v = _run_gpu(case, emb, W, bias, cuda, nc)
        outs.append(v.detach().cpu().numpy())
    assert np.abs(outs[0] - outs[1]).max() < 1e-5
    assert np.abs(outs[0] - outs[2]).max() < 1e-5


@pytest.mark.parametrize('case', [(3, 37, 8, 16, 4, 4, 63, 3, True), (2, 19, 8, 16, 4, 4, 8, 3, False),
                                  (1, 33, 4, 8, 0, 0, 63, 1, True), (2, 40, 16, 32, 2, 2, 16, 3, False),
                                  (2, 23, 16, 32, 2, 2, 32, 3, True)])
def test_route_dr_fwd32_matches_fp32_mfma_path(cuda, case, monkeypatch):
    """The split-fp16 32x32 forward (route_fwd32.hip) against the exact-fp32
    16x16x4 MFMA forward (route_pass_kernel): same routing to fp32 accuracy."""
    emb, W, bias = _mk(case, 5)
    _, _, _, v32 = _run_gpu(case, emb, W, bias, cuda)
    monkeypatch.setenv('SRF_ROUTE_FWD32', '0')
    _, _, _, v16 = _run_gpu(case, emb, W, bias, cuda)
    a = v32.detach().cpu().double().numpy()
    b = v16.detach().cpu().double().numpy()
    assert np.all(np.abs(a - b) <= 1e-5 * (1 + np.abs(b))), np.abs(a - b).max()


@pytest.mark.parametrize('case', [(3, 37, 8, 16, 4, 4, 63, 3, True), (2, 19, 8, 16, 4, 4, 8, 3, False),
                                  (2, 21, 4, 8, 2, 1, 12, 3, False), (2, 7, 4, 8, 1, 1, 6, 5, False),
                                  (2, 40, 16, 32, 2, 2, 16, 3, False), (2, 23, 16, 32, 2, 2, 32, 3, True),
                                  (1, 9, 4, 32, 1, 1, 8, 5, False)])
def test_route_dr_backward_from_stored_couplings(cuda, case, monkeypatch):
    """The backward routing passes that read the forward's stored couplings
    (route_bwd32_kernel) against the ones that recompute the logits
    (route_pass_kernel, SRF_ROUTE_COUPLINGS=0): same gradients to fp32 accuracy."""
    emb, W, bias = _mk(case, 6)
    gv = torch.tensor(np.random.default_rng(7).standard_normal(case[:2] + (case[6], case[3])), dtype=torch.float32,
                      device=cuda)
    grads = []
    for flag in ('1', '0'):
        monkeypatch.setenv('SRF_ROUTE_COUPLINGS', flag)
        te, tW, tb, v = _run_gpu(case, emb, W, bias, cuda)
        v.backward(gv)
        grads.append([t.grad.detach().cpu().double().numpy() for t in (te, tW, tb)])
    for a, b, name in zip(grads[0], grads[1], ('g_emb', 'g_W', 'g_bias')):
        assert np.abs(a - b).max() <= 2e-5 * max(1.0, np.abs(b).max()), (name, np.abs(a - b).max())


@pytest.mark.parametrize('case', [(3, 37, 8, 16, 4, 4, 63, 3, True), (2, 19, 8, 16, 4, 4, 8, 3, False),
                                  (1, 5, 3, 16, 1, 2, 5, 2, True)])
def test_split_passes_match(cuda, case, monkeypatch):
    """The opt-in split routing passes (SRF_FWD32_SPLIT=1: route_logit_kernel,
    route_lse_kernel, route_acc_kernel) against route_fwd32_kernel: same routing to
    fp32 accuracy, and the backward from the couplings they store agrees too."""
    emb, W, bias = _mk(case, 8)
    gv = torch.tensor(np.random.default_rng(9).standard_normal(case[:2] + (case[6], case[3])), dtype=torch.float32,
                      device=cuda)
    outs = []
    for flag in ('1', '0'):
        monkeypatch.setenv('SRF_FWD32_SPLIT', flag)
        te, tW, tb, v = _run_gpu(case, emb, W, bias, cuda)
        v.backward(gv)
        outs.append([v.detach().cpu().double().numpy()] + [t.grad.detach().cpu().double().numpy() for t in (te, tW, tb)])
    a, b = outs[0][0], outs[1][0]
    assert np.all(np.abs(a - b) <= 1e-5 * (1 + np.abs(b))), np.abs(a - b).max()
    for x, y, name in zip(outs[0][1:], outs[1][1:], ('g_emb', 'g_W', 'g_bias')):
        assert np.abs(x - y).max() <= 2e-5 * max(1.0, np.abs(y).max()), (name, np.abs(x - y).max())


@pytest.mark.parametrize('case,var', [((2, 40, 16, 32, 2, 2, 16, 3, False), 'SRF_FWD32_TW32'),
                                      ((1, 35, 8, 32, 1, 2, 8, 2, True), 'SRF_FWD32_TW32'),
                                      ((2, 45, 8, 16, 4, 4, 8, 3, False), 'SRF_FWD32_TW16'),
                                      ((2, 21, 4, 8, 2, 1, 12, 3, False), 'SRF_FWD32_TW16')])
def test_row_tiles_per_wave_plans_match(cuda, case, var, monkeypatch):
    """Row tiles per wave are a plan choice: din 32 runs 2 (J*dout <= 512) unless
    SRF_FWD32_TW32=4; small din <= 16 layers run 4 unless SRF_FWD32_TW16=2.  Both
    plans (and their coupling layouts) give the same routing and gradients."""
    emb, W, bias = _mk(case, 10)
    gv = torch.tensor(np.random.default_rng(11).standard_normal(case[:2] + (case[6], case[3])), dtype=torch.float32,
                      device=cuda)
    outs = []
    for tw in ('2', '4'):
        monkeypatch.setenv(var, tw)
        te, tW, tb, v = _run_gpu(case, emb, W, bias, cuda)
        v.backward(gv)
        outs.append([v.detach().cpu().double().numpy()] + [t.grad.detach().cpu().double().numpy() for t in (te, tW, tb)])
    a, b = outs[0][0], outs[1][0]
    assert np.all(np.abs(a - b) <= 1e-5 * (1 + np.abs(b))), np.abs(a - b).max()
    for x, y, name in zip(outs[0][1:], outs[1][1:], ('g_emb', 'g_W', 'g_bias')):
        assert np.abs(x - y).max() <= 2e-5 * max(1.0, np.abs(y).max()), (name, np.abs(x - y).max())


@pytest.mark.parametrize('case', [(2, 40, 16, 32, 2, 2, 16, 3, False), (2, 23, 16, 32, 2, 2, 32, 3, True),
                                  (1, 35, 8, 32, 1, 2, 8, 2, True), (1, 9, 4, 32, 1, 1, 8, 4, False),
                                  (2, 17, 4, 32, 1, 1, 6, 3, True), (3, 61, 8, 32, 2, 2, 12, 3, False)])
@pytest.mark.parametrize('var,on', [('SRF_GUX16', '1'), ('SRF_GUX16', '2'), ('SRF_GW16', '1'), ('SRF_GW_XCD', '1')])
def test_split16_grad_passes_match_fp32(cuda, case, var, on, monkeypatch):
    """The split-fp16 32x32 gradient passes for din = dout = 32 -- gx
    (route_gux16_kernel, SRF_GUX16) and gW / gbias (route_gw16_kernel, SRF_GW16) --
    against the exact-fp32 16x16x4 ones (route_gux_kernel / route_gw3_kernel, the
    switch at 0; SRF_GUX16=2: the gx pass as 2R-1 products on pre-split frame
    vectors): the same gradients to fp32 accuracy, including J not a multiple of
    the workgroup's 4 output capsules, partial last frame tiles and several frame
    splits of the gW pass (route_gw16_kernel stops at 3 iterations)."""
    emb, W, bias = _mk(case, 14)
    gv = torch.tensor(np.random.default_rng(15).standard_normal(case[:2] + (case[6], case[3])), dtype=torch.float32,
                      device=cuda)
    outs = []
    for flag in (on, '0'):
        monkeypatch.setenv(var, flag)
        te, tW, tb, v = _run_gpu(case, emb, W, bias, cuda)
        v.backward(gv)
        outs.append([t.grad.detach().cpu().double().numpy() for t in (te, tW, tb)])
    for x, y, name in zip(outs[0], outs[1], ('g_emb', 'g_W', 'g_bias')):
        assert np.abs(x - y).max() <= 2e-5 * max(1.0, np.abs(y).max()), (name, np.abs(x - y).max())


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
