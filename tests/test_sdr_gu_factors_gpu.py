"""The SDR backward through gu factors (srf_sdr_range.gu_factored) against gu itself.

With the forward's couplings, the register recurrence backward can store per frame
gL^r [R][in_n][JP], gs^r and Vc^r [R][J*dout] (srf_route_sdr_fact_floats) instead of
gu [in_n][J*dout], and srf_route_sdr_gx_gw_fact_n forms
gu_ij = sum_r c^r_ij gs^r_j + gL^r_ij Vc^r_j inside the fused gx / gW pass
(sdr_gxw32f_kernel).  Same inputs through both paths: the carry is bit-identical (the
recurrence's arithmetic does not change), g_emb / gW / gbias agree to fp32 reassociation
(1e-5 of each output's magnitude).  Cases: the C3 inner and last layer shapes (J = 16, 32;
the last masked, its recurrence ungrouped and grouped in two), two and three iterations,
two frame ranges run in reverse with the carry, an empty first range that starts the gW
sum, frame counts not a multiple of the 16-frame tile, one- and two-item launches.

Reference: sequence_router_naive.py:212-245 (the frame loop whose autodiff this is).
"""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [
    # J, N, lpad, rpad, iters, mask_first, group
    (16, 16, 2, 2, 3, False, 1),   # C3 inner layer
    (32, 16, 2, 2, 3, True, 1),    # C3 last layer
    (32, 16, 2, 2, 3, True, 2),    # C3 last layer, backward grouped as the stack runs it
    (16, 4, 1, 1, 2, False, 1),    # two iterations, in_n = 12
]


@pytest.mark.parametrize('J,N,lp,rp,iters,mf,G', CASES)
def test_sdr_gu_factors_match_gu(cuda, J, N, lp, rp, iters, mf, G):
    from srf_amd import _lib
    L = _lib.lib()
    din, D, B, T, cut = 32, 32, 3, 9, 4
    in_n, JD = N * (lp + rp + 1), J * D
    g = torch.Generator().manual_seed(5)
    u = (torch.randn(B * T * in_n * JD, generator=g) * 0.3).to(cuda)
    g_v = torch.randn(B, T, JD, generator=g).to(cuda)
    emb = torch.randn(B, T, N, din, generator=g).to(cuda)
    W = (torch.randn(in_n, JD, din, generator=g) * 0.1).to(cuda)
    WT = W.permute(0, 2, 1).contiguous()
    ncs = L.srf_route_sdr_coupling_floats(in_n, J, D, iters)
    nff = L.srf_route_sdr_fact_floats(in_n, J, D, iters)
    JP = max(4, 1 << (J - 1).bit_length())
    assert ncs > 0 and nff == iters * (in_n * JP + 2 * JD) and nff < in_n * JD
    ws_n = L.srf_route_sdr_recur_workspace(B, in_n, J, D, iters)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    v = torch.zeros(B, T, JD, device=cuda)
    cs = torch.zeros(B * T * ncs, device=cuda)
    ws = torch.zeros(ws_n // 4 + 4, device=cuda)
    ranges = ((0, cut), (cut, T))
    for t0, t1 in ranges:
        r = _lib.SdrRange(t0=t0, t1=t1, u=p(u), v0=0, vn=T, v=p(v), couplings=p(cs), workspace=p(ws),
                          workspace_bytes=ws_n)
        _lib.check(L.srf_route_sdr_recur_fwd_n((_lib.SdrRange * 1)(r), 1, B, T, in_n, J, D, iters, int(mf), st), 'fwd')
    init_W = torch.randn(in_n, JD, din, generator=g).to(cuda)
    init_b = torch.randn(in_n, JD, generator=g).to(cuda)
    outs = {}
    for fact in (False, True):
        gu = torch.full((B * T * (nff if fact else in_n * JD),), float('nan'), device=cuda)
        carry = torch.zeros(B, JD, device=cuda)

        def rng(t0, t1, acc=1):
            return _lib.SdrRange(t0=t0, t1=t1, emb=p(emb), W=p(W), WT=p(WT), u=p(u), v0=0, vn=T, v=p(v),
                                 couplings=p(cs), workspace=p(ws), workspace_bytes=ws_n, g_v=p(g_v), carry=p(carry),
                                 gu=p(gu), g0=0, gn=T, group=G, gu_factored=int(fact), accumulate=acc)
        for t0, t1 in reversed(ranges):
            rr = (_lib.SdrRange * 1)(rng(t0, t1))
            _lib.check(L.srf_route_sdr_recur_bwd_n(rr, 1, B, T, in_n, J, D, iters, int(mf), st), 'bwd')
        for items in ([[(0, 0, 0)], [(cut, T, 1)], [(0, cut, 1)]],        # one range per launch
                      [[(cut, T, 0), (0, 0, 1)], [(0, cut, 1)]]):          # two-item launches
            g_emb = torch.zeros_like(emb)
            gW, gb = init_W.clone(), init_b.clone()
            for launch in items:
                rr = (_lib.SdrRange * len(launch))(*[rng(t0, t1, acc) for t0, t1, acc in launch])
                for r in rr:
                    r.g_emb, r.g_W, r.g_bias = p(g_emb), p(gW), p(gb)
                if fact:
                    _lib.check(L.srf_route_sdr_gx_gw_fact_n(rr, len(launch), B, T, N, din, lp, rp, J, D, iters, st),
                               'gx_gw_fact_n')
                else:
                    _lib.check(L.srf_route_sdr_gx_gw_n(rr, len(launch), B, T, N, din, lp, rp, J, D, st), 'gx_gw_n')
            torch.cuda.synchronize()
            outs[(fact, len(items))] = (carry.clone(), g_emb, gW, gb)
    for n_launch in (3, 2):
        ref, got = outs[(False, n_launch)], outs[(True, n_launch)]
        assert torch.equal(ref[0], got[0]), 'carry'
        for name, a, b in zip(('g_emb', 'gW', 'gbias'), ref[1:], got[1:]):
            assert torch.isfinite(b).all(), name
            err, mag = (a - b).abs().max().item(), a.abs().max().item()
            assert mag > 0 and err <= 1e-5 * mag, (n_launch, name, err, mag)


def test_gx_gw_n_refuses_factors(cuda):
    """srf_route_sdr_gx_gw_n reads gu: a range marked gu_factored is refused (error, no
    launch) rather than read as gu."""
    from srf_amd import _lib
    L = _lib.lib()
    B, T, N, din, J, D = 2, 4, 4, 32, 16, 32
    in_n = N * 5
    buf = torch.zeros(B * T * in_n * J * D, device=cuda)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    r = _lib.SdrRange(t0=0, t1=T, emb=p(buf), W=p(buf), WT=p(buf), gu=p(buf), g0=0, gn=T, g_emb=p(buf), g_W=p(buf),
                      g_bias=p(buf), gu_factored=1)
    rc = L.srf_route_sdr_gx_gw_n((_lib.SdrRange * 1)(r), 1, B, T, N, din, 2, 2, J, D,
                                 ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc != 0 and b'gx_gw_fact_n' in L.srf_last_error()
