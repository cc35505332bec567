"""GPU parity of the sequential dynamic routing layer (srf_route_sdr_fwd/bwd,
through the C ABI) against the CPU oracle.

Forward: numpy float64 restatement of sequence_router_naive.py:162-170 with
body_context :231-245 / pad_body_context :212-229 (oracle/srf_oracle.py).
Backward: float64 autograd of the op-for-op torch mirror (oracle/naive_mirror.py).
Tolerances (fp32 kernel vs fp64 oracle): forward |err| <= 2e-5 * (1 + |ref|),
gradients |err| <= 1e-4 * max(1, max|ref|) -- the carried agreement vector makes
later frames depend on all earlier ones, so fp32 reassociation accumulates
along the utterance.
"""
import numpy as np
import pytest
import torch

from oracle import srf_oracle as so
from oracle import naive_mirror as nm

pytestmark = pytest.mark.gpu

CASES = [
    # B, T, N, D, lpad, rpad, J, iters, mask_first
    (2, 9, 4, 16, 1, 1, 5, 3, True),      # small, last-layer mask
    (1, 7, 8, 8, 2, 2, 16, 3, False),     # D = 8
    (3, 6, 16, 32, 2, 2, 16, 3, False),   # C3 inner layer shape (short)
    (2, 5, 16, 32, 2, 2, 32, 3, True),    # C3 last layer shape (short)
    (2, 8, 3, 16, 0, 1, 7, 1, False),     # one iteration, asymmetric window
    (1, 6, 2, 16, 1, 0, 4, 5, True),      # five iterations
    (2, 16, 16, 32, 2, 2, 16, 3, False),  # C3 inner layer shape, 16 frames of recurrence
    (1, 10, 8, 16, 4, 4, 63, 3, True),    # TIMIT-sized last layer: J = 63 (padded to 64), in_n = 72
    (2, 6, 4, 8, 0, 0, 3, 2, True),       # J = 3 (padded to 4), D = 8, no window
]
# shapes outside the register-resident (dout 8 | 16 | 32) and streaming (dout 32 | 64)
# kernels' cases, which run on the general LDS-state recurrence kernels (one workgroup
# per utterance); the optional last element is dout (default: = din)
LEGACY = [
    (2, 9, 4, 16, 1, 1, 5, 3, True, 12),
    (1, 7, 8, 8, 2, 2, 16, 3, False, 4),
    (2, 6, 4, 32, 2, 2, 6, 5, True, 20),
]
# ... and one whose frame state (in_n = 656 capsules x 8, five iterations) exceeds one
# CU's LDS: the same kernels keep it in the global workspace
GSTATE = [(1, 4, 16, 8, 20, 20, 8, 5, True, 4)]
# shapes of the streaming recurrence (route_sdr_stream.hip: dout 32 | 64, J*dout in
# {512, 1024, 2048}) that the register path does not take
STREAM = [
    (1, 3, 16, 64, 20, 20, 16, 5, False),  # C5 inner layer: in_n = 656, J*D = 1024, five iterations
    (2, 6, 4, 64, 2, 2, 16, 3, True),      # in_n = 20, last-layer mask
    (2, 5, 8, 32, 12, 12, 16, 3, False),   # D = 32, in_n = 200 (beyond the register path)
    (1, 4, 4, 64, 1, 1, 8, 2, True),       # J*D = 512
    (1, 3, 4, 32, 2, 2, 32, 4, False),     # D = 32, J = 32
    (2, 4, 3, 64, 1, 2, 32, 1, True),      # one iteration, J*D = 2048, in_n = 12 (ragged wave tail)
]


def _dims(case):
    B, T, N, D, lp, rp, J, it, mf = case[:9]
    return B, T, N, D, lp, rp, J, it, mf, (case[9] if len(case) > 9 else D)


def _mk(case, seed):
    B, T, N, D, lp, rp, J, it, mf, Do = _dims(case)
    rng = np.random.default_rng(seed)
    in_n = N * (lp + rp + 1)
    emb = rng.standard_normal((B, T, N, D)) * 0.5
    W = rng.standard_normal((in_n, J, Do, D)) * 0.1
    bias = rng.standard_normal((in_n, J, Do)) * 0.1
    return emb, W, bias


def _run_gpu(case, emb, W, bias, dev):
    from srf_amd.ops import RouteGeom, sequential_routing
    B, T, N, D, lp, rp, J, it, mf, Do = _dims(case)
    g = RouteGeom(B, T, N, D, lp, rp, J, Do, it, mf)
    te = torch.tensor(emb, dtype=torch.float32, device=dev, requires_grad=True)
    tW = torch.tensor(W, dtype=torch.float32, device=dev, requires_grad=True)
    tb = torch.tensor(bias, dtype=torch.float32, device=dev, requires_grad=True)
    return te, tW, tb, sequential_routing(te, tW, tb, g)


def _check_forward(case, dev):
    emb, W, bias = _mk(case, 11)
    _, _, _, v = _run_gpu(case, emb, W, bias, dev)
    B, T, N, D, lp, rp, J, it, mf, Do = _dims(case)
    ref = so.sequential_routing(so.pose(so.window(emb, lp, rp), W, bias), it, mf)
    got = v.detach().cpu().double().numpy()
    assert np.all(np.abs(got - ref) <= 2e-5 * (1 + np.abs(ref))), np.abs(got - ref).max()


@pytest.mark.parametrize('case', CASES)
def test_route_sdr_forward(cuda, case):
    _check_forward(case, cuda)


@pytest.mark.parametrize('case', LEGACY)
def test_route_sdr_legacy_kernels(cuda, case):
    """The LDS-state recurrence kernels (the general path for capsule widths the
    register-resident and streaming kernels do not cover)."""
    _check_forward(case, cuda)
    _check_backward(case, cuda)


@pytest.mark.parametrize('case', STREAM)
def test_route_sdr_stream_kernels(cuda, case):
    """The streaming recurrence (u_t re-read per iteration, stored couplings for the
    backward): forward and backward against the oracle."""
    _check_forward(case, cuda)
    _check_backward(case, cuda)


@pytest.mark.parametrize('case', CASES)
def test_route_sdr_backward(cuda, case):
    _check_backward(case, cuda)


def _check_backward(case, cuda):
    emb, W, bias = _mk(case, 12)
    te, tW, tb, v = _run_gpu(case, emb, W, bias, cuda)
    gv = np.random.default_rng(13).standard_normal(v.shape)
    v.backward(torch.tensor(gv, dtype=torch.float32, device=cuda))
    B, T, N, D, lp, rp, J, it, mf, Do = _dims(case)
    ce = torch.tensor(emb, requires_grad=True)
    cW = torch.tensor(W, requires_grad=True)
    cb = torch.tensor(bias, requires_grad=True)
    ep = torch.nn.functional.pad(ce, (0, 0, 0, 0, lp, rp))
    xw = torch.cat([ep[:, w:w + T] for w in range(lp + rp + 1)], dim=2)
    vr = nm.sequential_routing(nm.pose_tiled(xw, cW, cb), it, mf)
    vr.backward(torch.tensor(gv))
    for name, got, ref in (('g_emb', te.grad, ce.grad), ('g_W', tW.grad, cW.grad), ('g_bias', tb.grad, cb.grad)):
        got = got.cpu().double().numpy()
        ref = ref.numpy()
        err = np.abs(got - ref).max()
        assert err <= 1e-4 * max(1.0, np.abs(ref).max()), (name, err, np.abs(ref).max())


@pytest.mark.parametrize('case', GSTATE)
def test_route_sdr_global_state_kernels(cuda, case):
    """The LDS-state kernels with their frame state in the global-memory workspace
    (shapes whose state exceeds one CU's LDS)."""
    _check_forward(case, cuda)
    _check_backward(case, cuda)


def test_route_sdr_c5_last_layer_shape(cuda):
    """BASELINE C5's last layer (in_n = 16*41 = 656, J = 32, D = 64, 5 iterations,
    lpad = rpad = 20): u_t (5.4 MB) exceeds a workgroup's registers, so it runs on
    the streaming recurrence.  Two frames, forward and backward against the oracle."""
    case = (1, 2, 16, 64, 20, 20, 32, 5, True)
    _check_forward(case, cuda)
    _check_backward(case, cuda)


@pytest.mark.parametrize('din,J,D', [(64, 16, 64), (64, 32, 64), (32, 16, 32)])
def test_sdr_pose_fp8_bound(cuda, din, J, D):
    """srf_route_sdr_pose_fp8 (opt-in e4m3 pose, BASELINE C5) against the float64 pose
    (sequence_router_naive.py:154-159): per element |u - ref| <= 0.13 sum_k |W||x|
    (each operand rounded to e4m3, 2^-4 relative, after a per-row / per-frame
    power-of-two scale) + fp32 rounding, on operands whose rows and frames span
    2^-20 .. 2^4 with zero (padded) frames.  The median error must stay at e4m3
    level (not merely inside the bound)."""
    import ctypes
    from srf_amd import _lib
    B, T, N, lp, rp = 2, 9, 3, 2, 1
    t0, t1 = 2, 8
    in_n, JD = N * (lp + rp + 1), J * D
    rng = np.random.default_rng(21)
    emb = rng.standard_normal((B, T, N, din)) * 2.0 ** rng.uniform(-20, 4, (B, T, N, 1))
    emb[1, 4] = 0.0
    W = rng.standard_normal((in_n, JD, din)) * 0.1 * 2.0 ** rng.uniform(-20, 4, (in_n, JD, 1))
    bias = rng.standard_normal((in_n, JD)) * 0.1
    L = _lib.lib()
    te = torch.tensor(emb, dtype=torch.float32, device=cuda)
    tW = torch.tensor(W, dtype=torch.float32, device=cuda)
    tb = torch.tensor(bias, dtype=torch.float32, device=cuda)
    nt = t1 - t0
    u = torch.full((B, nt, in_n, JD), float('nan'), device=cuda)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(L.srf_route_sdr_pose_fp8(p(te), p(tW), p(tb), B, T, N, din, lp, rp, J, D, t0, t1, p(u), t0, nt, st),
               'pose_fp8')
    torch.cuda.synchronize()
    e32 = te.double().cpu().numpy()   # the fp32 operands the kernel saw
    W32 = tW.double().cpu().numpy()
    b32 = tb.double().cpu().numpy()
    x = so.window(e32, lp, rp)[:, t0:t1]                      # [B, nt, in_n, din]
    ref = np.einsum('irk,btik->btir', W32, x) + b32[None, None]
    mag = np.einsum('irk,btik->btir', np.abs(W32), np.abs(x))
    got = u.cpu().double().numpy()
    err = np.abs(got - ref)
    assert np.all(err <= 0.13 * mag + 1e-6 * (np.abs(ref) + 1e-30)), (err - 0.13 * mag).max()
    rel = err[mag > 0] / mag[mag > 0]
    assert np.median(rel) < 0.02, np.median(rel)


@pytest.mark.parametrize('din,J,D', [(64, 16, 64), (32, 16, 32)])
def test_sdr_pose_fp8_matches_emulation(cuda, din, J, D):
    """The fp8 pose kernel (pose_n mode 1: fp32 u; mode 2: bf16 u) computes exactly the
    quantisation oracle/srf_oracle.pose_fp8 restates (per-vector power-of-two scales,
    e4m3 round to nearest even, exact products, fp32 bias, bf16 rounding of u), with
    operands spanning 2^-20 .. 2^4 and zero frames.  The emulation sums exactly; the
    fp8 MFMA does not accumulate its K block in full fp32: measured on gfx950 (r04g
    dump, both din) its sums differ from the exact sum of the same e4m3 products by
    up to 2^-14.3 sum_k |W_q||x_q| (2^-12.3 of the largest single product).  The bound
    is 2^-12 sum_k |W_q||x_q| + 2 fp32 ulps of u (+ one bf16 ulp, 2^-7 |u|, in mode 2:
    a sum that differs in its last fp32 bits may round to the other bf16 neighbour): one
    wrongly rounded or wrongly scaled operand of weight above 2^-8 of the sum fails it."""
    import ctypes
    from srf_amd import _lib
    L = _lib.lib()
    B, T, N, lp, rp = 2, 7, 3, 1, 2
    in_n, JD = N * (lp + rp + 1), J * D
    rng = np.random.default_rng(31)
    emb = (rng.standard_normal((B, T, N, din)) * 2.0 ** rng.uniform(-20, 4, (B, T, N, 1))).astype(np.float32)
    emb[0, 3] = 0.0
    W = (rng.standard_normal((in_n, JD, din)) * 0.1 * 2.0 ** rng.uniform(-20, 4, (in_n, JD, 1))).astype(np.float32)
    bias = (rng.standard_normal((in_n, JD)) * 0.1).astype(np.float32)
    x = so.window(emb.astype(np.float64), lp, rp)                                   # [B, T, in_n, din]
    Wr = W.astype(np.float64).reshape(in_n, J, D, din)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    te, tW, tb = (torch.tensor(a, device=cuda) for a in (emb, W, bias))
    ex = so.e4m3_scale_exp(np.abs(x).max(-1))
    ew = so.e4m3_scale_exp(np.abs(Wr).max(-1))
    xq = so.e4m3_round(x * np.exp2(ex)[..., None]) * np.exp2(-ex)[..., None]
    wq = so.e4m3_round(Wr * np.exp2(ew)[..., None]) * np.exp2(-ew)[..., None]
    mag = np.einsum('ijdk,btik->btijd', np.abs(wq), np.abs(xq)).reshape(B, T, in_n, JD)
    for mode in (1, 2):
        ref = so.pose_fp8(x, Wr, bias.astype(np.float64).reshape(in_n, J, D), bf16_u=(mode == 2))
        ref = ref.reshape(B, T, in_n, JD)
        if mode == 1:
            u = torch.full((B * T * in_n * JD,), float('nan'), device=cuda)
        else:
            u = torch.zeros(B * T * in_n * JD, device=cuda, dtype=torch.bfloat16)
        r = _lib.SdrRange(t0=0, t1=T, emb=p(te), W=p(tW), bias=p(tb), u=p(u), v0=0, vn=T, u_bf16=int(mode == 2))
        _lib.check(L.srf_route_sdr_pose_n((_lib.SdrRange * 1)(r), 1, B, T, N, din, lp, rp, J, D, mode, st), 'pose')
        torch.cuda.synchronize()
        got = u.float().cpu().double().numpy().reshape(B, T, in_n, JD)
        tol = 2.0 ** -12 * mag + 2.0 ** -22 * np.abs(ref) + (2.0 ** -7 * np.abs(ref) if mode == 2 else 0.0)
        err = np.abs(got - ref)
        assert np.all(err <= tol), (mode, (err - tol).max(), np.argwhere(err > tol)[:4].tolist())


@pytest.mark.parametrize('J,D,iters,mf', [(16, 64, 5, False), (32, 64, 3, True)])
def test_sdr_stream_bf16_u_equals_fp32(cuda, J, D, iters, mf):
    """The streaming recurrence reading u stored in bf16 (the fp8 C5 variant) computes
    exactly what the fp32 kernels compute from the same, bf16-representable u:
    forward v, couplings and backward gu / carry to fp32 rounding (the widening is
    exact).  And the fp8 pose storing bf16 (pose_n mode 2) writes the fp32-output
    fp8 pose (mode 1) rounded to nearest even."""
    import ctypes
    from srf_amd import _lib
    L = _lib.lib()
    B, T, N, lp, rp = 2, 5, 8, 4, 4
    in_n, JD = N * (lp + rp + 1), J * D
    rng = torch.Generator().manual_seed(5)
    u32 = (torch.randn(B * T * in_n * JD, generator=rng) * 0.3).to(torch.bfloat16)
    u16 = u32.to(cuda)
    u32 = u32.float().to(cuda)
    ncs = L.srf_route_sdr_coupling_floats(in_n, J, D, iters)
    ws_n = L.srf_route_sdr_recur_workspace(B, in_n, J, D, iters)
    assert ncs > 0 and L.srf_route_sdr_couplings_required(in_n, J, D, iters)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g_v = torch.randn(B, T, JD, generator=rng).to(cuda)
    outs = []
    for u, bf in ((u32, 0), (u16, 1)):
        v = torch.zeros(B, T, JD, device=cuda)
        cs = torch.zeros(B * T * ncs, device=cuda)
        ws = torch.zeros(max(ws_n // 4, 4), device=cuda)
        r = _lib.SdrRange(t0=0, t1=T, u=p(u), v0=0, vn=T, v=p(v), couplings=p(cs), workspace=p(ws),
                          workspace_bytes=ws.numel() * 4, u_bf16=bf)
        _lib.check(L.srf_route_sdr_recur_fwd_n((_lib.SdrRange * 1)(r), 1, B, T, in_n, J, D, iters, int(mf), st), 'fwd')
        gu = torch.zeros(B * T * in_n * JD, device=cuda)
        carry = torch.zeros(B, JD, device=cuda)
        r.g_v, r.carry, r.gu, r.g0, r.gn = p(g_v), p(carry), p(gu), 0, T
        _lib.check(L.srf_route_sdr_recur_bwd_n((_lib.SdrRange * 1)(r), 1, B, T, in_n, J, D, iters, int(mf), st), 'bwd')
        torch.cuda.synchronize()
        outs.append((v, cs, gu, carry))
    for a, b in zip(*outs):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6), (a - b).abs().max().item()
    # pose_n mode 2 == mode 1 rounded to bf16
    din = 64
    emb = torch.randn(B, T, N, din, generator=rng).to(cuda)
    W = (torch.randn(in_n, JD, din, generator=rng) * 0.1).to(cuda)
    bias = (torch.randn(in_n, JD, generator=rng) * 0.1).to(cuda)
    uf = torch.zeros(B * T * in_n * JD, device=cuda)
    ub = torch.zeros(B * T * in_n * JD, device=cuda, dtype=torch.bfloat16)
    for buf, mode in ((uf, 1), (ub, 2)):
        r = _lib.SdrRange(t0=0, t1=T, emb=p(emb), W=p(W), bias=p(bias), u=p(buf), v0=0, vn=T, u_bf16=int(mode == 2))
        _lib.check(L.srf_route_sdr_pose_n((_lib.SdrRange * 1)(r), 1, B, T, N, din, lp, rp, J, D, mode, st), 'pose')
    torch.cuda.synchronize()
    assert torch.equal(uf.to(torch.bfloat16), ub)


@pytest.mark.parametrize('J,D,iters,mf,N,lp,rp', [
    (16, 64, 5, False, 16, 20, 20),   # streaming: C5 inner layer
    (32, 64, 3, True, 8, 4, 4),       # streaming: J * D = 2048
    (16, 64, 2, False, 3, 1, 1),      # streaming: in_n = 9 (members without capsules)
    (32, 32, 3, True, 16, 2, 2),      # register kernels: C3 last layer (G = 2: three rows per lane)
    (16, 32, 3, False, 16, 2, 2),     # register kernels: C3 inner layer
    (16, 16, 5, True, 4, 1, 1),       # register kernels: five iterations, in_n = 12
])
def test_sdr_groups_match_one_workgroup(cuda, J, D, iters, mf, N, lp, rp):
    """srf_sdr_range.group > 1 splits each utterance's input capsules over G workgroups
    that add their per-iteration partial sums inside the launch (srf_group.h; the
    streaming and the register-resident recurrence kernels).  Forward v / couplings and
    backward gu / carry equal the one-workgroup launch up to the reassociation of the
    partial sums, for groups of 2, 3 and 8 (members without capsules included), over
    two frame ranges, and no member gave up waiting (the timeout word stays 0); every
    launch leaves the workspace's group counters zero (three launches reuse each)."""
    import ctypes
    from srf_amd import _lib
    L = _lib.lib()
    B, T = 3, 6
    in_n, JD = N * (lp + rp + 1), J * D
    rng = torch.Generator().manual_seed(7)
    u = (torch.randn(B * T * in_n * JD, generator=rng) * 0.3).to(cuda)
    g_v = torch.randn(B, T, JD, generator=rng).to(cuda)
    ncs = L.srf_route_sdr_coupling_floats(in_n, J, D, iters)
    ws_n = L.srf_route_sdr_recur_workspace(B, in_n, J, D, iters)
    streamed = bool(L.srf_route_sdr_couplings_required(in_n, J, D, iters))
    assert ncs > 0
    # srf_group.h coff: the stream backward's gL scratch first, then the counters and the timeout word
    coff = -(-B * iters * in_n * J // 64) * 64 if streamed else 0
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    outs = []
    for G in (1, 2, 3, 8):
        v = torch.zeros(B, T, JD, device=cuda)
        cs = torch.zeros(B * T * ncs, device=cuda)
        gu = torch.zeros(B * T * in_n * JD, device=cuda)
        carry = torch.zeros(B, JD, device=cuda)
        wss = [torch.zeros(ws_n // 4 + 4, device=cuda) for _ in range(2)]
        cut = 2
        rr = []
        for k, (t0, t1) in enumerate(((0, cut), (cut, T))):
            rr.append(_lib.SdrRange(t0=t0, t1=t1, u=p(u), v0=0, vn=T, v=p(v), couplings=p(cs), workspace=p(wss[k]),
                                    workspace_bytes=ws_n, group=G, g_v=p(g_v), carry=p(carry), gu=p(gu), g0=0, gn=T))
        # the forward's ranges in order (range 1 starts from range 0's v), the backward's in reverse
        for k in (0, 1):
            _lib.check(L.srf_route_sdr_recur_fwd_n((_lib.SdrRange * 1)(rr[k]), 1, B, T, in_n, J, D, iters, int(mf),
                                                   st), 'fwd')
        for k in (1, 0):
            _lib.check(L.srf_route_sdr_recur_bwd_n((_lib.SdrRange * 1)(rr[k]), 1, B, T, in_n, J, D, iters, int(mf),
                                                   st), 'bwd')
        # and both ranges' forward in one two-item launch, each into a v buffer of its own
        # (range 1 then starts from a zero v_{t0-1}): per-item counters, against G = 1
        v2 = torch.zeros(2, B, T, JD, device=cuda)
        r2 = [_lib.SdrRange(t0=t0, t1=t1, u=p(u), v0=0, vn=T, v=p(v2[k]), workspace=p(wss[k]), workspace_bytes=ws_n,
                            group=G) for k, (t0, t1) in enumerate(((0, cut), (cut, T)))]
        _lib.check(L.srf_route_sdr_recur_fwd_n((_lib.SdrRange * 2)(*r2), 2, B, T, in_n, J, D, iters, int(mf), st),
                   'fwd2')
        torch.cuda.synchronize()
        if G > 1:
            for w in wss:
                assert w[coff + B].view(torch.int32).item() == 0, 'a group member timed out'
                # each launch left its arrival / departure counters zero for the next one
                # (srf_group.h depart: no memset per launch)
                assert w[coff:coff + 2 * B + 1].view(torch.int32).abs().sum().item() == 0, 'counters left set'
        outs.append((G, v, cs, gu, carry, v2))
    # reassociated fp32 sums, carried through the frames: 1e-5 of each output's magnitude
    for G, *got in outs[1:]:
        for name, a, b in zip(('v', 'cs', 'gu', 'carry', 'v2'), outs[0][1:], got):
            err, mag = (a - b).abs().max().item(), a.abs().max().item()
            assert err <= 1e-5 * mag + 1e-7, (G, name, err, mag)


@pytest.mark.gpu
@pytest.mark.parametrize('J,N,lp,rp', [(16, 16, 2, 2), (32, 16, 2, 2), (8, 3, 1, 1)])
def test_sdr_gx_gw_fused_matches_separate(cuda, J, N, lp, rp):
    """srf_route_sdr_gx_gw_n (din 32: one pass over gu, sdr_gxw32_kernel) computes what
    srf_route_sdr_gx_n + srf_route_sdr_gw_n compute on the same ranges: g_emb through the
    window adjoint (added), gW / gbias overwritten by a range with accumulate == 0
    (also an empty one) and added by the next; C3's inner and last layer shapes and one
    with idle waves (J*dout = 256 < 512 rows per workgroup).  Both sum in fp32 in
    different orders (and g_emb by atomics): 1e-5 of each output's magnitude."""
    import ctypes
    from srf_amd import _lib
    L = _lib.lib()
    din, D, B, T = 32, 32, 3, 9
    in_n, JD = N * (lp + rp + 1), J * D
    g = torch.Generator().manual_seed(11)
    emb = torch.randn(B, T, N, din, generator=g).to(cuda)
    W = (torch.randn(in_n, JD, din, generator=g) * 0.1).to(cuda)
    WT = W.permute(0, 2, 1).contiguous()
    gu = torch.randn(B * T * in_n * JD, generator=g).to(cuda)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    init_W, init_b = torch.randn(in_n, JD, din, generator=g).to(cuda), torch.randn(in_n, JD, generator=g).to(cuda)
    outs = []
    for fused in (False, True):
        g_emb = torch.zeros_like(emb)
        gW, gb = init_W.clone(), init_b.clone()
        for t0, t1, acc in ((0, 0, 0), (0, 4, 1), (4, 9, 1), (9, 9, 1)):
            r = _lib.SdrRange(t0=t0, t1=t1, emb=p(emb), W=p(W), WT=p(WT), gu=p(gu), g0=0, gn=T, g_emb=p(g_emb),
                              g_W=p(gW), g_bias=p(gb), accumulate=acc)
            rr = (_lib.SdrRange * 1)(r)
            args = (rr, 1, B, T, N, din, lp, rp, J, D, st)
            if fused:
                _lib.check(L.srf_route_sdr_gx_gw_n(*args), 'gx_gw_n')
            else:
                if t1 > t0:
                    _lib.check(L.srf_route_sdr_gx_n(*args), 'gx_n')
                _lib.check(L.srf_route_sdr_gw_n(*args), 'gw_n')
        torch.cuda.synchronize()
        outs.append((g_emb, gW, gb))
    for name, a, b in zip(('g_emb', 'gW', 'gbias'), *outs):
        err, mag = (a - b).abs().max().item(), a.abs().max().item()
        assert mag > 0 and err <= 1e-5 * mag, (name, err, mag)


@pytest.mark.gpu
@pytest.mark.parametrize('din,J,D', [(32, 16, 32), (32, 32, 32), (64, 16, 64)])
def test_sdr_pose_fp32_accuracy(cuda, din, J, D):
    """The fp32 pose (pose_n mode 0; din 32 / 64 on bf16 MFMA with three-term split
    operands, sdr_pose3b_kernel) against u = W x + b in float64: fp32-level error,
    |u - u64| <= 2^-18 (sum_k |W||x| + |b|) -- the accumulator starts at the bias and
    each MFMA rounds the running sum in fp32 (a one-term bf16 split would miss the bound
    by 2^10) -- with operands spanning 2^-20 .. 2^4, a zero frame and the window's edge
    frames."""
    import ctypes
    from srf_amd import _lib
    L = _lib.lib()
    B, T, N, lp, rp = 2, 7, 3, 1, 2
    in_n, JD = N * (lp + rp + 1), J * D
    rng = np.random.default_rng(5)
    emb = (rng.standard_normal((B, T, N, din)) * 2.0 ** rng.uniform(-20, 4, (B, T, N, 1))).astype(np.float32)
    emb[0, 3] = 0.0
    W = (rng.standard_normal((in_n, JD, din)) * 0.1 * 2.0 ** rng.uniform(-20, 4, (in_n, JD, 1))).astype(np.float32)
    bias = (rng.standard_normal((in_n, JD)) * 0.1).astype(np.float32)
    x = so.window(emb.astype(np.float64), lp, rp)                                   # [B, T, in_n, din]
    ref = np.einsum('ijk,btik->btij', W.astype(np.float64), x) + bias.astype(np.float64)
    mag = np.einsum('ijk,btik->btij', np.abs(W.astype(np.float64)), np.abs(x))
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    te, tW, tb = (torch.tensor(a, device=cuda) for a in (emb, W, bias))
    u = torch.full((B * T * in_n * JD,), float('nan'), device=cuda)
    r = _lib.SdrRange(t0=0, t1=T, emb=p(te), W=p(tW), bias=p(tb), u=p(u), v0=0, vn=T)
    _lib.check(L.srf_route_sdr_pose_n((_lib.SdrRange * 1)(r), 1, B, T, N, din, lp, rp, J, D, 0, st), 'pose')
    torch.cuda.synchronize()
    got = u.double().cpu().numpy().reshape(B, T, in_n, JD)
    err = np.abs(got - ref)
    tol = 2.0 ** -18 * (mag + np.abs(bias.astype(np.float64)))
    assert np.all(err <= tol), ((err - tol).max(), np.argwhere(err > tol)[:4].tolist())
