"""SDR parity at the sizes and plans the bench runs (round-4 verdict, item 1), against
the float64 CPU oracle -- every frame of v and the FULL parameter / input gradients,
not samples.

* C3 slice: two inner J = 16 layers feeding the masked J = 32 layer at B = 28,
  T' = 200, through ``ops.SdrStack`` with the bench's own plan (20 frame ranges of 10,
  the inner layers' ranges batched per anti-diagonal, the last layer's backward on
  G = 2 workgroups per utterance), u kept from the forward and recomputed per range.
  W x 0.5 (the ``c3_real`` fixture's scale): there fp32 tracks float64 (the float32
  mirror of this slice is within 3.4e-7 of it in v, 1.3e-6 in the gradients), so the
  layer tests' bounds apply.
* C5 pair: an inner streamed layer (in_n = 656, D = 64, 5 iterations) feeding the
  masked last layer, B = 2, T' = 200, W x 0.25, at the bench's G = 2 and at the
  plan's own G.
* Reference init (W ~ N(0, 0.1), naive:97-103): the recurrence itself amplifies fp32
  rounding along the frames (two fp32 runs of ONE C3 layer drift apart from 1e-7 at
  frame 0 to ~0.3 by frame 180), so no fp32 run tracks a free-running float64 oracle.
  Each frame is checked instead as one step from the run's own previous output
  (``oracle.naive_mirror.sdr_layer_teacher_forced``), every layer of the slice, at the
  layer bound 2e-5 (1 + |ref|), and the LN between layers against float64 LN of the
  run's own v.  Likewise the first C5 layer, with the fp32 pose and with the opt-in
  fp8 pose (bf16 u on and off) against its emulation.

References: sequence_router_naive.py:162-170 (frame loop), :212-245 (body_context,
pad_body_context), :187-191 (LN between layers).
"""
import numpy as np
import pytest
import torch

from oracle import naive_mirror as nm

pytestmark = pytest.mark.gpu

V_TOL = 2e-5     # |v - ref| <= V_TOL (1 + |ref|), the routing-layer bound
G_TOL = 1e-4     # |g - ref| <= G_TOL max(1, max|ref|) per tensor


def _f32(a):
    return a.astype(np.float32).astype(np.float64)   # the values the GPU holds


def _params(rng, layers, lpad, rpad, w_scale):
    win = lpad + rpad + 1
    Ws, bs, gam, bet = [], [], [], []
    for l, (N, din, J, D, mf) in enumerate(layers):
        Ws.append(rng.standard_normal((N * win, J, D, din)) * 0.1 * w_scale)
        bs.append(rng.standard_normal((N * win, J, D)) * 0.1)
        if l < len(layers) - 1:
            gam.append(1 + 0.1 * rng.standard_normal(J * D))
            bet.append(0.1 * rng.standard_normal(J * D))
    return [_f32(w) for w in Ws], [_f32(b) for b in bs], [_f32(g) for g in gam], [_f32(b) for b in bet]


def _run_stack(dev, emb, Ws, bs, gam, bet, plan, g_v):
    """ops.SdrStack forward + backward.  Returns (v, grads..., the forward's saved layer
    inputs and outputs)."""
    from srf_amd import ops
    L = plan.L
    te = torch.tensor(emb, dtype=torch.float32, device=dev, requires_grad=True)
    params = []
    for l in range(L):
        params += [torch.tensor(Ws[l], dtype=torch.float32, device=dev, requires_grad=True),
                   torch.tensor(bs[l], dtype=torch.float32, device=dev, requires_grad=True)]
    for l in range(L - 1):
        params += [torch.tensor(gam[l], dtype=torch.float32, device=dev, requires_grad=True),
                   torch.tensor(bet[l], dtype=torch.float32, device=dev, requires_grad=True)]
    v = ops.sdr_stack(te, plan, False, 0.0, 0, params)
    saved = v.grad_fn.saved_tensors
    embs = [s.detach().cpu().double() for s in saved[:L]]
    vs = [s.detach().cpu().double() for s in saved[L:2 * L]]
    v.backward(torch.tensor(g_v, dtype=torch.float32, device=dev))
    torch.cuda.synchronize()
    grads = [te.grad] + [p.grad for p in params]
    return v.detach().cpu().double(), [g.cpu().double() for g in grads], embs, vs


def _check(got, ref, what):
    got, ref = torch.as_tensor(got).double(), torch.as_tensor(ref).double()
    bad = (got - ref).abs() > V_TOL * (1 + ref.abs())
    print(what, 'max |err| / (1 + |ref|) = %.3g' % float(((got - ref).abs() / (1 + ref.abs())).max()))
    assert not bad.any(), (what, int(bad.sum()), bad.nonzero()[:6].tolist(), float((got - ref).abs().max()))


def _check_grads(grads, ref, L):
    """grads: [g_emb, gW0, gb0, ..., gamma0, beta0, ...]; ref: sdr_stack_frames' tuple."""
    names = ['g_emb'] + [f'g_{w}{l}' for l in range(L) for w in ('W', 'b')] + \
            [f'g_{t}{l}' for l in range(L - 1) for t in ('gamma', 'beta')]
    rf = [ref[1]] + [x for l in range(L) for x in (ref[2][l], ref[3][l])] + \
         [x for l in range(L - 1) for x in (ref[4][l], ref[5][l])]
    bad = []
    for n, g, r in zip(names, grads, rf):
        err, scale = float((g - r).abs().max()), float(r.abs().max())
        print(n, 'max |err| / max(1, max|ref|) = %.3g' % (err / max(1.0, scale)))
        if err > G_TOL * max(1.0, scale):
            bad.append((n, err, scale))
    assert not bad, bad


# --------------------------------------------------------------------------- C3 slice
C3_SLICE = [(16, 32, 16, 32, 0), (16, 32, 16, 32, 0), (16, 32, 32, 32, 1)]


@pytest.fixture(scope='module')
def c3_slice():
    rng = np.random.default_rng(305)
    B, T = 28, 200
    Ws, bs, gam, bet = _params(rng, C3_SLICE, 2, 2, 0.5)
    emb = _f32(rng.standard_normal((B, T, 16, 32)))     # the primary capsules' LN output scale
    g_v = rng.standard_normal((B, T, 32, 32))
    ref = nm.sdr_stack_frames(emb, Ws, bs, gam, bet, 2, 2, 3, g_v)
    return emb, Ws, bs, gam, bet, g_v, ref


@pytest.mark.parametrize('store_u', [None, 0], ids=['u_kept', 'u_recomputed'])
def test_c3_sdr_slice_at_bench_size(cuda, c3_slice, store_u):
    """Every frame of the last layer's v and the full g_emb / g_W / g_bias / g_gamma /
    g_beta of a 3-layer C3 slice at B = 28, T' = 200 against the float64 frame-by-frame
    mirror, on the bench's plan (asserted)."""
    from srf_amd import ops
    emb, Ws, bs, gam, bet, g_v, ref = c3_slice
    plan = ops.SdrStackPlan(28, 200, C3_SLICE, 2, 2, 3, store_u_bytes=store_u)
    assert plan.S == 10 and sum(plan.fwd[0][k + 1] > plan.fwd[0][k] for k in range(plan.K)) == 20, \
        'the bench cuts 200 frames into 20 ranges of 10'
    assert any(all(0 <= d - l < plan.K and plan.fwd[l][d - l] < plan.fwd[l][d - l + 1] for l in range(2))
               for d in range(plan.K + 1)), 'the inner layers share batched launches'
    assert plan.group(2, cuda, backward=True) == 2 and plan.group(2, cuda) == 1, 'last backward on G = 2'
    assert plan.streamed == [False, False, False], 'C3 layers run the register recurrence'
    v, grads, _, _ = _run_stack(cuda, emb, Ws, bs, gam, bet, plan, g_v)
    _check(v, ref[0], 'v')
    _check_grads(grads, ref, 3)


def test_c3_reference_init_every_frame_teacher_forced(cuda):
    """The same slice at the reference init W ~ N(0, 0.1): every frame of every layer
    against one float64 step from the run's own previous frame, and the LN between
    layers against float64 LN of the run's own v."""
    from srf_amd import ops
    rng = np.random.default_rng(306)
    B, T = 28, 200
    Ws, bs, gam, bet = _params(rng, C3_SLICE, 2, 2, 1.0)
    emb = _f32(rng.standard_normal((B, T, 16, 32)))
    g_v = rng.standard_normal((B, T, 32, 32))
    plan = ops.SdrStackPlan(B, T, C3_SLICE, 2, 2, 3)
    _, _, embs, vs = _run_stack(cuda, emb, Ws, bs, gam, bet, plan, g_v)
    assert torch.equal(embs[0], torch.tensor(emb, dtype=torch.float32).double())
    for l, (N, din, J, D, mf) in enumerate(C3_SLICE):
        ref = nm.sdr_layer_teacher_forced(embs[l], Ws[l], bs[l], vs[l], 2, 2, 3, bool(mf))
        _check(vs[l], ref, f'layer {l} v')
        if l < 2:
            ln = nm.layer_norm(vs[l].reshape(B, T, J * D), torch.tensor(gam[l]), torch.tensor(bet[l]))
            _check(embs[l + 1], ln.reshape(B, T, J, D), f'LN after layer {l}')


# --------------------------------------------------------------------------- C5
C5_PAIR = [(16, 64, 16, 64, 0), (16, 64, 32, 64, 1)]


@pytest.fixture(scope='module')
def c5_pair():
    rng = np.random.default_rng(505)
    B, T = 2, 200
    Ws, bs, gam, bet = _params(rng, C5_PAIR, 20, 20, 0.25)
    emb = _f32(rng.standard_normal((B, T, 16, 64)))
    g_v = rng.standard_normal((B, T, 32, 64))
    ref = nm.sdr_stack_frames(emb, Ws, bs, gam, bet, 20, 20, 5, g_v)
    return emb, Ws, bs, gam, bet, g_v, ref


@pytest.mark.parametrize('group', [2, None], ids=['G2_bench', 'G_auto'])
def test_c5_sdr_pair_at_bench_length(cuda, c5_pair, group):
    """A C5 inner streamed layer feeding the masked last layer (in_n = 656, D = 64,
    5 iterations) at B = 2, T' = 200: every frame of v and the full gradients against
    the float64 frame-by-frame mirror.  The last layer's recurrence on G = 2
    workgroups per utterance (the bench's G at B = 28) and on the plan's own choice."""
    from srf_amd import ops
    emb, Ws, bs, gam, bet, g_v, ref = c5_pair
    plan = ops.SdrStackPlan(2, 200, C5_PAIR, 20, 20, 5, last_group=group)
    assert plan.streamed == [True, True], 'C5 layers stream u_t from HBM'
    if group is None:
        assert plan.group(1, cuda) > 2
    v, grads, _, _ = _run_stack(cuda, emb, Ws, bs, gam, bet, plan, g_v)
    _check(v, ref[0], 'v')
    _check_grads(grads, ref, 2)


# fp8 pose against its emulation: the MFMA's e4m3 block sums are not the exact sums of
# the same products (up to 2^-12 sum|W_q||x_q| on the kernel test,
# tests/test_route_sdr_gpu.py::test_sdr_pose_fp8_matches_emulation), and with bf16 u an
# element within that distance of a bf16 rounding boundary rounds the other way
# (2^-8 of |u|).  Both enter v through a softmax-weighted sum over 656 capsules.
FP8_V_TOL = 2e-3


@pytest.mark.parametrize('pose', ['fp32', 'fp8_bf16u', 'fp8_fp32u'])
def test_c5_first_layer_reference_init_teacher_forced(cuda, pose):
    """The first C5 layer at the reference init, B = 2, T' = 200, where the recurrence
    amplifies rounding along the frames as in C3 (fp32 and float64 runs 1.7e-5 apart by
    frame 6, 0.17 by frame 30): every frame against one float64 step from the run's own
    previous frame -- fp32 pose at the layer bound; the opt-in fp8 pose (BASELINE
    configs[4]) against the emulated e4m3 pose (``srf_oracle.pose_fp8`` quantisation),
    bf16 u on and off, at FP8_V_TOL."""
    from srf_amd import ops
    rng = np.random.default_rng(507)
    B, T = 2, 200
    layers = [(16, 64, 16, 64, 0)]
    Ws, bs, _, _ = _params(rng, layers, 20, 20, 1.0)
    emb = _f32(rng.standard_normal((B, T, 16, 64)))
    fp8, bf16_u = pose != 'fp32', pose == 'fp8_bf16u'
    plan = ops.SdrStackPlan(B, T, layers, 20, 20, 5, pose_fp8=fp8, u_bf16=bf16_u)
    assert plan.ubf == [bf16_u]
    _, _, embs, vs = _run_stack(cuda, emb, Ws, bs, [], [], plan, rng.standard_normal((B, T, 16, 64)))
    ref = nm.sdr_layer_teacher_forced(embs[0], Ws[0], bs[0], vs[0], 20, 20, 5, False,
                                      fp8_bf16=bf16_u if fp8 else None)
    if not fp8:
        _check(vs[0], ref, 'v')
    else:
        err = ((vs[0] - ref).abs() / (1 + ref.abs())).max()
        print(pose, 'max |err| / (1 + |ref|) = %.3g' % float(err))
        assert err <= FP8_V_TOL, float(err)


# --------------------------------------------------------------------------- reference-init backward
@pytest.mark.parametrize('layer,group', [((16, 32, 16, 32, 0), 1), ((16, 32, 32, 32, 1), 2)],
                         ids=['c3_inner', 'c3_last_G2'])
def test_c3_reference_init_backward_teacher_forced(cuda, layer, group):
    """The backward of a C3 layer at the reference init W ~ N(0, 0.1), B = 28 (the
    bench's batch), frame by frame: the recurrence backward runs one frame per launch
    (srf_route_sdr_recur_bwd_n, the last layer on G = 2 workgroups per utterance as the
    bench runs it), so the carry the GPU hands each frame (dL/dv_t from frame t + 1) is
    read back, and every frame's full pose gradient g_u_t and its carry into frame t - 1
    are checked against the float64 adjoint of that one frame given the run's own
    v_{t-1} and that carry (``oracle.naive_mirror.sdr_layer_backward_teacher_forced``)
    at the routing-layer gradient bound.  Then gx (window adjoint of W^T g_u) and
    gW / gbias (sum over frames of g_u x^T, g_u) of the fused contraction
    (srf_route_sdr_gx_gw_n) against float64 contractions of the GPU's own g_u.  At this
    init a free-running float32 mirror drifts from float64 by 6e-5 in v and 8e-4 in
    the gradients within 10 frames, so per-frame teacher forcing is what makes a tight
    full-gradient check possible (the scaled-init stack test covers the plan's ranges)."""
    import ctypes
    from srf_amd import _lib
    L = _lib.lib()
    N, din, J, D, mf = layer
    lp = rp = 2
    B, T, iters = 28, 64, 3
    in_n, JD = N * (lp + rp + 1), J * D
    rng = np.random.default_rng(308 + J)
    Ws, bs, _, _ = _params(rng, [layer], lp, rp, 1.0)
    W64, b64 = Ws[0], bs[0]
    emb = _f32(rng.standard_normal((B, T, N, din)))
    g_v = _f32(rng.standard_normal((B, T, J, D)))
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    te = torch.tensor(emb, dtype=torch.float32, device=cuda)
    tW = torch.tensor(W64, dtype=torch.float32, device=cuda)              # [in_n, J, D, din] = [in_n][J*D][din]
    tb = torch.tensor(b64, dtype=torch.float32, device=cuda)
    tg = torch.tensor(g_v, dtype=torch.float32, device=cuda)
    u = torch.zeros(B * T * in_n * JD, device=cuda)
    v = torch.zeros(B, T, JD, device=cuda)
    ncs = L.srf_route_sdr_coupling_floats(in_n, J, D, iters)
    assert ncs > 0 and not L.srf_route_sdr_couplings_required(in_n, J, D, iters), 'C3: register recurrence'
    cs = torch.zeros(B * T * ncs, device=cuda)
    ws_n = L.srf_route_sdr_recur_workspace(B, in_n, J, D, iters)
    ws = torch.zeros(max(ws_n // 4, 4) + 4, device=cuda)
    r = _lib.SdrRange(t0=0, t1=T, emb=p(te), W=p(tW), bias=p(tb), u=p(u), v0=0, vn=T, v=p(v), couplings=p(cs),
                      workspace=p(ws), workspace_bytes=ws.numel() * 4)
    _lib.check(L.srf_route_sdr_pose_n((_lib.SdrRange * 1)(r), 1, B, T, N, din, lp, rp, J, D, 0, st), 'pose')
    _lib.check(L.srf_route_sdr_recur_fwd_n((_lib.SdrRange * 1)(r), 1, B, T, in_n, J, D, iters, mf, st), 'fwd')
    gu = torch.zeros(B * T * in_n * JD, device=cuda)
    carry = torch.zeros(B, JD, device=cuda)
    c_in = torch.zeros(B, T, JD, device=cuda)
    c_out = torch.zeros(B, T, JD, device=cuda)
    for t in range(T - 1, -1, -1):   # one frame per launch: the carry between frames is read back
        c_in[:, t] = carry
        rt = _lib.SdrRange(t0=t, t1=t + 1, u=p(u), v0=0, vn=T, v=p(v), couplings=p(cs), workspace=p(ws),
                           workspace_bytes=ws.numel() * 4, g_v=p(tg), carry=p(carry), gu=p(gu), g0=0, gn=T,
                           group=group)
        _lib.check(L.srf_route_sdr_recur_bwd_n((_lib.SdrRange * 1)(rt), 1, B, T, in_n, J, D, iters, mf, st), 'bwd')
        c_out[:, t] = carry
    torch.cuda.synchronize()
    v_run = v.cpu().double().reshape(B, T, J, D)
    g_bar = torch.tensor(g_v) + c_in.cpu().double().reshape(B, T, J, D)
    ref_gu, ref_gvp = nm.sdr_layer_backward_teacher_forced(emb, W64, b64, v_run, g_bar, lp, rp, iters, bool(mf))
    got_gu = gu.cpu().double().reshape(B, T, in_n, J, D)
    for name, got, ref in (('g_u', got_gu, ref_gu), ('carry', c_out.cpu().double().reshape(B, T, J, D), ref_gvp)):
        err, scale = float((got - ref).abs().max()), float(ref.abs().max())
        print(name, 'max |err| / max(1, max|ref|) = %.3g' % (err / max(1.0, scale)), 'max|ref| %.3g' % scale)
        assert scale > 0 and err <= G_TOL * max(1.0, scale), (name, err, scale)
    # the contractions of the GPU's own g_u: gx through the window adjoint, gW, gbias
    WT = tW.reshape(in_n, JD, din).permute(0, 2, 1).contiguous()
    g_emb = torch.zeros_like(te)
    gW = torch.zeros(in_n, JD, din, device=cuda)
    gb = torch.zeros(in_n, JD, device=cuda)
    rg = _lib.SdrRange(t0=0, t1=T, emb=p(te), W=p(tW), WT=p(WT), gu=p(gu), g0=0, gn=T, g_emb=p(g_emb), g_W=p(gW),
                       g_bias=p(gb), accumulate=0)
    _lib.check(L.srf_route_sdr_gx_gw_n((_lib.SdrRange * 1)(rg), 1, B, T, N, din, lp, rp, J, D, st), 'gx_gw')
    torch.cuda.synchronize()
    gu64 = got_gu.reshape(B, T, in_n, JD)
    xw = torch.nn.functional.pad(torch.tensor(emb), (0, 0, 0, 0, lp, rp))
    xw = torch.cat([xw[:, w:w + T] for w in range(lp + rp + 1)], 2)                  # [B, T, in_n, din]
    ref_gW = torch.einsum('btir,btik->irk', gu64, xw)
    ref_gb = gu64.sum((0, 1))
    gxw = torch.einsum('btir,irk->btik', gu64, torch.tensor(W64).reshape(in_n, JD, din))   # [B, T, in_n, din]
    ref_ge = torch.zeros(B, T + lp + rp, N, din, dtype=torch.float64)
    for w in range(lp + rp + 1):
        ref_ge[:, w:w + T] += gxw[:, :, w * N:(w + 1) * N]
    ref_ge = ref_ge[:, lp:lp + T]
    for name, got, ref in (('g_emb', g_emb, ref_ge), ('g_W', gW, ref_gW), ('g_bias', gb, ref_gb)):
        got = got.cpu().double().reshape(ref.shape)
        err, scale = float((got - ref).abs().max()), float(ref.abs().max())
        print(name, 'max |err| / max(1, max|ref|) = %.3g' % (err / max(1.0, scale)))
        assert err <= G_TOL * max(1.0, scale), (name, err, scale)
