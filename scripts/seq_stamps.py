"""Per-frame time and phase shares of the register SDR recurrence (one layer, C3 shapes).

    python scripts/seq_stamps.py                      # timing with the shipped library
    SRF_LIB_PATH=ab/stamp.so python scripts/seq_stamps.py   # + phase cycle shares
                                                      # (bash scripts/build_ab.sh stamp
                                                      #  "route_sdr_seq.hip route_sdr_seq_bwd.hip" -DSRF_SEQ_STAMP=1)

Stamp builds are diagnostic: read their shares, not their length.
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from srf_amd import _lib  # noqa: E402

FWD_PH = ['logits+softmax+partials', 'barrier A', 'wave sums+squash', 'barrier B']
BWD_PH = ['loads v,g_v,c + barrier', 's loads + Vc', 'squash adjoint + barrier', 'adjoint dots/partials',
          'barrier', 'gVc sums', 'gu', 'next rows + barrier']


def vp(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def run(name, B, T, in_n, J, D, R, mf, frames):
    L = _lib.lib()
    dev = torch.device('cuda:0')
    JD = J * D
    g = torch.Generator(device=dev).manual_seed(0)
    u = torch.randn(B, T, in_n, JD, device=dev, generator=g) * 0.1
    v = torch.empty(B, T, JD, device=dev)
    ncs = L.srf_route_sdr_coupling_floats(in_n, J, D, R)
    cs = torch.empty(B * T * ncs, device=dev)
    wsb = L.srf_route_sdr_recur_workspace(B, in_n, J, D, R)
    ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device=dev)
    g_v = torch.randn(B, T, JD, device=dev, generator=g) * 0.01
    carry = torch.zeros(B, JD, device=dev)
    gu = torch.empty_like(u)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    t0, t1 = T - frames, T

    def fwd(a, b):
        _lib.check(L.srf_route_sdr_recur_fwd(vp(u), 0, T, B, T, in_n, J, D, R, mf, a, b, vp(v), vp(cs), vp(ws),
                                             ws.numel(), st), 'recur_fwd')

    def bwd(a, b):
        _lib.check(L.srf_route_sdr_recur_bwd(vp(u), 0, T, vp(v), vp(cs), vp(g_v), B, T, in_n, J, D, R, mf, a, b,
                                             vp(carry), vp(gu), 0, T, vp(ws), ws.numel(), st), 'recur_bwd')

    fwd(0, T)   # every frame's v and couplings
    torch.cuda.synchronize()
    stamps = {}
    for which, fn, phases in (('fwd', fwd, FWD_PH), ('bwd', bwd, BWD_PH)):
        buf = torch.zeros(B * 2 * 8, dtype=torch.int64, device=dev)
        setter = _stamp_setter(which)
        if setter:
            setter(ctypes.c_void_p(buf.data_ptr()))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn(t0, t1)   # warm
        torch.cuda.synchronize()
        e0.record()
        fn(t0, t1)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / frames
        line = f'{name} {which}: {us:.2f} us/frame ({frames} frames, B={B})'
        if setter:
            c = buf.view(B, 2, 8).double().mean(0) / frames   # cycles per frame, waves 0 / 15
            tot = c.sum(1)
            line += '\n' + '\n'.join(f'    {p:28s} w0 {c[0, i]:9.0f} cyc {100 * c[0, i] / tot[0]:5.1f}%   '
                                     f'w15 {c[1, i]:9.0f} {100 * c[1, i] / tot[1]:5.1f}%'
                                     for i, p in enumerate(phases))
            setter(None)
        print(line, flush=True)
        stamps[which] = us
    return stamps


def _stamp_setter(which):
    try:
        f = getattr(ctypes.CDLL(_lib.LIB_PATH), f'srf_seq_{which}_stamp_buffer')
    except AttributeError:
        return None
    f.argtypes = [ctypes.c_void_p]
    f.restype = ctypes.c_int
    return f


if __name__ == '__main__':
    B = int(os.environ.get('B', 28))
    T = int(os.environ.get('T', 200))
    frames = int(os.environ.get('FRAMES', 20))
    run('inner (80x16x32)', B, T, 80, 16, 32, 3, 0, frames)
    run('last (80x32x32)', B, T, 80, 32, 32, 3, 1, frames)
