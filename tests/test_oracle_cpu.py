"""CPU checks of the oracle itself (no GPU): the numpy float64 restatement and
the torch mirror must reproduce the committed golden fixtures and each other,
the CTC restatement must match torch's, and the backward of the mirror must
match finite differences."""
import numpy as np
import pytest
import torch

from oracle import naive_mirror as nm
from oracle import srf_oracle as so
from tests.helpers import load_model_fixture


@pytest.mark.parametrize('name', ['c1_mini', 'c2_mini', 'c3_mini_sdr', 'c2_mini_einsum', 'c2_mini_lowmemory',
                                  'c3_mini_sdr_lowmemory'])
def test_oracle_reproduces_fixture(name):
    kw, sh, P, z = load_model_fixture(name)
    logits = so.srf_forward(P, sh, z['feats'], z['inp_len'])
    assert np.abs(logits - z['logits']).max() < 1e-9
    nll = so.ctc_batch(logits, z['labels'], z['inp_len'], z['tar_len'], sh.class_n)
    assert np.abs(nll - z['nll']).max() < 1e-8
    assert so.greedy_decode(logits, np.ceil(z['inp_len'] / 4).astype(int), sh.class_n - 1) == z['greedy']


@pytest.mark.parametrize('caps_type', ['naive', 'einsum', 'lowmemory'])
def test_mirror_matches_oracle_sdr_and_dr(caps_type):
    for ctx in (False, True):
        sh = so.SrfShape(enc_num=2, iters=2, lpad=1, rpad=2, ph=4, pd=8, ch=4, cd=8, vd=8, class_n=9, context=ctx,
                         caps_type=caps_type)
        P = so.init_params(sh, seed=5)
        rng = np.random.default_rng(6)
        feats = rng.standard_normal((2, 23, 123))
        inp_len = np.array([23, 17])
        feats[1, 17:] = 0
        a = so.srf_forward(P, sh, feats, inp_len)
        b = nm.NaiveMirror(sh, P)(torch.tensor(feats), torch.tensor(inp_len)).detach().numpy()
        assert np.abs(a - b).max() < 1e-10


def test_same_padding_rule():
    # TF 'SAME': pad_before = total // 2
    assert so.same_pad(123, 3, 2) == (62, 1, 1)
    assert so.same_pad(62, 3, 2) == (31, 0, 1)
    assert so.same_pad(320, 3, 2) == (160, 0, 1)
    assert so.same_pad(37, 3, 2) == (19, 1, 1)
    assert so.same_pad(80, 3, 1) == (80, 1, 1)


def test_dr_mask_makes_capsule0_exactly_zero():
    rng = np.random.default_rng(0)
    u = rng.standard_normal((1, 3, 5, 4, 8))
    v = so.dynamic_routing(u, 3, True)
    assert np.all(v[..., 0, :] == 0.0)


def test_ctc_oracle_matches_torch_with_repeats_and_blank_last():
    rng = np.random.default_rng(1)
    C, T = 7, 12
    logits = rng.standard_normal((2, T, C))
    labels = np.array([[1, 1, 2, 3], [4, 5, 5, 0]])
    tl = np.array([4, 3])
    il = np.array([T * 4, 9 * 4])
    ours = so.ctc_batch(logits, labels, il, tl, C)
    ref = nm.ctc_per_utt(torch.tensor(logits), torch.tensor(labels), torch.tensor(il), torch.tensor(tl), C).numpy()
    assert np.abs(ours - ref).max() < 1e-10


def test_ctc_infeasible_is_inf():
    logits = np.zeros((3, 5))
    assert np.isinf(so.ctc_nll(logits, np.array([1, 1, 1]), 4))   # needs >= 5 frames


def test_mirror_gradient_finite_difference():
    sh = so.SrfShape(enc_num=1, iters=2, lpad=1, rpad=0, ph=2, pd=8, ch=2, cd=8, vd=8, class_n=5, nfilt=4)
    P = so.init_params(sh, seed=3)
    rng = np.random.default_rng(4)
    feats = rng.standard_normal((1, 9, 123))
    inp_len = np.array([9])
    m = nm.NaiveMirror(sh, P)
    out = m(torch.tensor(feats), torch.tensor(inp_len))
    wvec = torch.tensor(rng.standard_normal(out.shape))
    (out * wvec).sum().backward()
    g = m.P('W0').grad.numpy().copy()
    idx = (1, 3, 2, 5)
    eps = 1e-6
    for sgn in (1, -1):
        P2 = dict(P)
        P2['W0'] = P['W0'].copy()
        P2['W0'][idx] += sgn * eps
        val = (so.srf_forward(P2, sh, feats, inp_len) * wvec.numpy()).sum()
        if sgn == 1:
            plus = val
        else:
            minus = val
    fd = (plus - minus) / (2 * eps)
    assert abs(fd - g[idx]) < 1e-6 * max(1.0, abs(fd))


def test_pos_enc_matches_closed_form():
    """get_pos_enc (model_helper.py:30-58): row 0 is [0..0 | 1..1]; float32 values
    agree with the float64 closed form to float32 rounding of t * inv_k."""
    pe = so.pos_enc(200, 16)
    assert pe.dtype == np.float32 and pe.shape == (200, 16)
    assert np.all(pe[0, :8] == 0) and np.all(pe[0, 8:] == 1)
    t = np.arange(200)[:, None]
    inv = np.exp(-np.arange(8) * np.log(1e4) / 7)[None, :]
    ref = np.concatenate([np.sin(t * inv), np.cos(t * inv)], 1)
    assert np.abs(pe - ref).max() < 5e-5


def test_lowmemory_routes_once_and_ignores_W_in_dr():
    """lowmemory: --model-caps-iter is ignored (lowmemory:107-109,190) and its DR
    layers do not read W / bias (lowmemory:162-164)."""
    rng = np.random.default_rng(3)
    feats = rng.standard_normal((2, 21, 123))
    inp_len = np.array([21, 16])
    outs = []
    for iters in (1, 3):
        sh = so.SrfShape(enc_num=2, iters=iters, lpad=1, rpad=1, ph=4, pd=8, ch=4, cd=8, vd=8, class_n=9,
                         caps_type='lowmemory')
        P = so.init_params(sh, seed=7)
        outs.append(so.srf_forward(P, sh, feats, inp_len))
    assert np.abs(outs[0] - outs[1]).max() == 0
    P2 = dict(P, W0=P['W0'] * 3.0, b1=P['b1'] + 1.0)
    assert np.abs(so.srf_forward(P2, sh, feats, inp_len) - outs[1]).max() == 0
    sh_n = so.SrfShape(enc_num=2, iters=3, lpad=1, rpad=1, ph=4, pd=8, ch=4, cd=8, vd=8, class_n=9)
    assert np.abs(so.srf_forward(P, sh_n, feats, inp_len) - outs[1]).max() > 1e-3


def test_dr_layer_chunked_matches_mirror_autograd():
    """The chunked float64 DR layer (used at C4 bench size) equals the numpy oracle's
    forward and the tiled mirror's autograd gradients on a small ragged case."""
    rng = np.random.default_rng(0)
    B, T, N, D, lp, rp, J = 2, 9, 3, 8, 2, 1, 5
    emb = rng.standard_normal((B, T, N, D))
    W = rng.standard_normal((N * 4, J, D, D)) * 0.1
    b = rng.standard_normal((N * 4, J, D)) * 0.1
    gv = rng.standard_normal((B, T, J, D))
    v, ge, gW, gb = nm.dr_layer_chunked(emb, W, b, lp, rp, 3, True, gv, frames_per_chunk=5)
    assert np.abs(v.numpy() - so.dynamic_routing(so.pose(so.window(emb, lp, rp), W, b), 3, True)).max() < 1e-13
    ce, cW, cb = (torch.tensor(a, requires_grad=True) for a in (emb, W, b))
    ep = torch.nn.functional.pad(ce, (0, 0, 0, 0, lp, rp))
    xw = torch.cat([ep[:, w:w + T] for w in range(lp + rp + 1)], 2)
    nm.dynamic_routing(nm.pose_tiled(xw, cW, cb), 3, True).backward(torch.tensor(gv))
    for got, ref in ((ge, ce), (gW, cW), (gb, cb)):
        assert (got - ref.grad).abs().max().item() < 1e-12


def test_sdr_stack_frames_matches_oracle_and_tiled_mirror():
    """The frame-by-frame float64 SDR stack (used at C3 / C5 bench size) equals the
    numpy oracle's layer-by-layer forward and the tiled mirror's autograd gradients on
    a small ragged 2-layer case with LN between the layers; its fp8 pose is the
    oracle's ``pose_fp8``."""
    rng = np.random.default_rng(2)
    B, T, N, D, lp, rp, J = 2, 7, 3, 8, 2, 1, 4
    I = N * (lp + rp + 1)
    emb = rng.standard_normal((B, T, N, D))
    Ws = [rng.standard_normal((I, N, D, D)) * 0.3, rng.standard_normal((I, J, D, D)) * 0.3]
    bs = [rng.standard_normal((I, N, D)) * 0.1, rng.standard_normal((I, J, D)) * 0.1]
    gam, bet = [1 + 0.1 * rng.standard_normal(N * D)], [0.1 * rng.standard_normal(N * D)]
    gv = rng.standard_normal((B, T, J, D))
    v, ge, gW, gb, gg, gbt = nm.sdr_stack_frames(emb, Ws, bs, gam, bet, lp, rp, 3, gv)
    x = emb
    for l in range(2):
        y = so.sequential_routing(so.pose(so.window(x, lp, rp), Ws[l], bs[l]), 3, l == 1)
        if l == 0:
            x = so.layer_norm(y.reshape(B, T, -1), gam[0], bet[0]).reshape(B, T, N, D)
    assert np.abs(v.numpy() - y).max() < 1e-13
    ce = torch.tensor(emb, requires_grad=True)
    cW = [torch.tensor(w, requires_grad=True) for w in Ws]
    cb = [torch.tensor(b, requires_grad=True) for b in bs]
    cg, cbt = torch.tensor(gam[0], requires_grad=True), torch.tensor(bet[0], requires_grad=True)
    x = ce
    for l in range(2):
        ep = torch.nn.functional.pad(x, (0, 0, 0, 0, lp, rp))
        xw = torch.cat([ep[:, w:w + T] for w in range(lp + rp + 1)], 2)
        y = nm.sequential_routing(nm.pose_tiled(xw, cW[l], cb[l]), 3, l == 1)
        if l == 0:
            x = nm.layer_norm(y.reshape(B, T, -1), cg, cbt).reshape(B, T, N, D)
    y.backward(torch.tensor(gv))
    pairs = [(ge, ce), (gW[0], cW[0]), (gW[1], cW[1]), (gb[0], cb[0]), (gb[1], cb[1]), (gg[0], cg), (gbt[0], cbt)]
    for got, ref in pairs:
        assert (got - ref.grad).abs().max().item() < 1e-12
    # fp8 pose, bf16 u on the first layer
    v8 = nm.sdr_stack_frames(emb, Ws, bs, gam, bet, lp, rp, 3, gv, fp8_pose=[True, False])[0]
    x = emb
    for l in range(2):
        y = so.sequential_routing(so.pose_fp8(so.window(x, lp, rp), Ws[l], bs[l], l == 0), 3, l == 1)
        if l == 0:
            x = so.layer_norm(y.reshape(B, T, -1), gam[0], bet[0]).reshape(B, T, N, D)
    assert np.abs(v8.numpy() - y).max() < 1e-12


def test_sdr_teacher_forced_is_one_step_of_the_recurrence():
    """sdr_layer_teacher_forced fed a float64 run's own output reproduces it (to float64 rounding);
    fed a float32 run's output it stays at rounding level while the free-running float32
    run has drifted (reference init: the recurrence amplifies rounding along the frames)."""
    rng = np.random.default_rng(3)
    B, T, N, D, lp = 4, 60, 16, 32, 2   # the C3 layer shape
    I = N * (2 * lp + 1)
    emb = rng.standard_normal((B, T, N, D))
    W, b = rng.standard_normal((I, 16, D, D)) * 0.1, rng.standard_normal((I, 16, D)) * 0.1
    gv = rng.standard_normal((B, T, 16, D))
    v64 = nm.sdr_stack_frames(emb, [W], [b], [], [], lp, lp, 3, gv, mask_last=False)[0]
    v32 = nm.sdr_stack_frames(emb, [W], [b], [], [], lp, lp, 3, gv, dtype=torch.float32, mask_last=False)[0]
    v32 = v32.double()
    assert (nm.sdr_layer_teacher_forced(emb, W, b, v64, lp, lp, 3, False, frames_per_chunk=7) - v64).abs().max() < 1e-14
    tf = nm.sdr_layer_teacher_forced(emb, W, b, v32, lp, lp, 3, False)
    assert ((tf - v32).abs() / (1 + v32.abs())).max() < 2e-6
    assert ((v32 - v64).abs() / (1 + v64.abs())).max() > 1e-5


@pytest.mark.parametrize('masked', [False, True])
def test_sdr_backward_teacher_forced_is_one_frame_of_the_adjoint(masked):
    """sdr_layer_backward_teacher_forced, fed a float64 run's own v and, per frame, the
    total dL/dv_t of a float64 autograd backward through the whole recurrence (loss
    gradient plus the carry from frame t + 1), reproduces that backward's pose gradient
    for every frame and its carry into frame t - 1 (to float64 rounding)."""
    import torch.nn.functional as F
    rng = np.random.default_rng(1)
    B, T, N, D, J, Dv, lp, rp, iters = 2, 6, 3, 4, 5, 4, 1, 1, 3
    I = N * (lp + rp + 1)
    emb = torch.tensor(rng.standard_normal((B, T, N, D)))
    W = torch.tensor(rng.standard_normal((I, J, Dv, D)) * 0.3)
    bias = torch.tensor(rng.standard_normal((I, J, Dv)) * 0.1)
    g_v = torch.tensor(rng.standard_normal((B, T, J, Dv)))
    ep = F.pad(emb, (0, 0, 0, 0, lp, rp))
    xw = torch.cat([ep[:, w:w + T] for w in range(lp + rp + 1)], 2)            # [B, T, I, D]
    u = (torch.einsum('ijek,btik->btije', W, xw) + bias).requires_grad_(True)   # [B, T, I, J, Dv]
    v = torch.zeros(B, J, Dv, dtype=torch.float64)
    m = torch.zeros(B, I, J, dtype=torch.float64)
    if masked:
        m[..., 0] = -1e9
    vs = []
    for t in range(T):
        b = torch.zeros(B, I, J, dtype=torch.float64)
        for _ in range(iters):
            b = b + torch.sum(u[:, t] * v.unsqueeze(1), -1) + m
            v = nm.squash(torch.sum(torch.softmax(b, 2).unsqueeze(-1) * u[:, t], 1), -1)
        v.retain_grad()
        vs.append(v)
    sum((vs[t] * g_v[:, t]).sum() for t in range(T)).backward()
    g_bar = torch.stack([x.grad for x in vs], 1)
    gu, gvp = nm.sdr_layer_backward_teacher_forced(emb, W, bias, torch.stack([x.detach() for x in vs], 1), g_bar,
                                                   lp, rp, iters, masked, frames_per_chunk=4)
    assert (gu - u.grad).abs().max() < 1e-13
    assert (gvp[:, 1:] - (g_bar - g_v)[:, :-1]).abs().max() < 1e-13


def test_e4m3_and_bf16_emulation_match_torch_casts():
    """The fp8-pose restatement's rounding (srf_oracle.e4m3_round / bf16_round) equals
    torch's float8_e4m3fn / bfloat16 casts (round to nearest even, e4m3 subnormals),
    and the per-vector scale puts every absmax in (224, 448]."""
    rng = np.random.default_rng(1)
    a = (rng.standard_normal(100000) * np.exp2(rng.uniform(-12, 8, 100000))).astype(np.float32)
    a = np.clip(a, -448, 448).astype(np.float64)
    ref = torch.tensor(a, dtype=torch.float32).to(torch.float8_e4m3fn).to(torch.float64).numpy()
    assert np.array_equal(so.e4m3_round(a), ref)
    b = rng.standard_normal(10000).astype(np.float32)
    assert np.array_equal(so.bf16_round(b), torch.tensor(b).to(torch.bfloat16).double().numpy())
    am = (np.abs(rng.standard_normal(10000)) * np.exp2(rng.integers(-30, 30, 10000))).astype(np.float32)
    s = am.astype(np.float64) * np.exp2(so.e4m3_scale_exp(am))
    assert s.min() > 224 and s.max() <= 448
    assert so.e4m3_scale_exp(np.float32(0)) == 0


def test_fp8_pose_error_within_declared_bound():
    """pose_fp8 against the exact pose: |u - u_exact| <= 0.13 sum_k |W||x| + fp32
    (the bound include/srf.h states for srf_route_sdr_pose_n modes 1 and 2)."""
    rng = np.random.default_rng(2)
    x = rng.standard_normal((2, 3, 5, 32)) * np.exp2(rng.uniform(-10, 4, (2, 3, 5, 1)))
    W = rng.standard_normal((5, 4, 8, 32)) * 0.1
    bias = rng.standard_normal((5, 4, 8)) * 0.1
    exact = so.pose(x, W, bias)
    bound = 0.13 * np.einsum('ijde,btie->btijd', np.abs(W), np.abs(x)) + 1e-6 * (1 + np.abs(exact))
    for bf in (False, True):
        err = np.abs(so.pose_fp8(x, W, bias, bf) - exact)
        assert np.all(err <= bound + (np.abs(exact) * 2.0 ** -8 if bf else 0))
