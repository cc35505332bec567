"""Per-frame time of one SDR recurrence layer, forward and backward, against the
workgroup-group size G (srf_sdr_range.group), the layer alone on the GPU.

    python scripts/sdr_group_frames.py            # C3 last (80x32x32) and inner (80x16x32)

Each (layer, G) line: us per frame of the forward and of the backward over FRAMES
frames of B utterances (HIP events around one launch, after a warm launch).
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from srf_amd import _lib  # noqa: E402


def run(name, B, T, in_n, J, D, R, mf, frames, groups):
    L = _lib.lib()
    dev = torch.device('cuda:0')
    JD = J * D
    g = torch.Generator(device=dev).manual_seed(0)
    u = torch.randn(B * T * in_n * JD, device=dev, generator=g) * 0.1
    g_v = torch.randn(B, T, JD, device=dev, generator=g) * 0.01
    ncs = L.srf_route_sdr_coupling_floats(in_n, J, D, R)
    ws_n = L.srf_route_sdr_recur_workspace(B, in_n, J, D, R)
    v = torch.zeros(B, T, JD, device=dev)
    cs = torch.zeros(B * T * ncs, device=dev)
    gu = torch.empty_like(u)
    carry = torch.zeros(B, JD, device=dev)
    ws = torch.zeros(ws_n // 4 + 4, device=dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    t0 = T - frames
    for G in groups:
        full = _lib.SdrRange(t0=0, t1=T, u=p(u), v0=0, vn=T, v=p(v), couplings=p(cs), workspace=p(ws),
                             workspace_bytes=ws_n, group=1)
        rr = _lib.SdrRange(t0=t0, t1=T, u=p(u), v0=0, vn=T, v=p(v), couplings=p(cs), workspace=p(ws),
                           workspace_bytes=ws_n, group=G, g_v=p(g_v), carry=p(carry), gu=p(gu), g0=0, gn=T)
        try:
            _lib.check(L.srf_route_sdr_recur_fwd_n((_lib.SdrRange * 1)(full), 1, B, T, in_n, J, D, R, mf, st), 'f')
        except _lib.SrfError as e:
            print(f'{name} G={G}: {e}', flush=True)
            continue

        def fwd():
            _lib.check(L.srf_route_sdr_recur_fwd_n((_lib.SdrRange * 1)(rr), 1, B, T, in_n, J, D, R, mf, st), 'fwd')

        def bwd():
            _lib.check(L.srf_route_sdr_recur_bwd_n((_lib.SdrRange * 1)(rr), 1, B, T, in_n, J, D, R, mf, st), 'bwd')

        res = []
        for fn in (fwd, bwd):
            try:
                fn()
            except _lib.SrfError as e:
                res.append(f'n/a ({e})')
                continue
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            res.append(f'{e0.elapsed_time(e1) * 1e3 / frames:8.2f} us/frame')
        print(f'{name} G={G}: fwd {res[0]}  bwd {res[1]}  ({frames} frames, B={B})', flush=True)


if __name__ == '__main__':
    B = int(os.environ.get('B', 28))
    T = int(os.environ.get('T', 200))
    frames = int(os.environ.get('FRAMES', 20))
    groups = [int(x) for x in os.environ.get('SDR_GROUPS', '1,2,4,8').split(',')]
    run('last (80x32x32)', B, T, 80, 32, 32, 3, 1, frames, groups)
    run('inner (80x16x32)', B, T, 80, 16, 32, 3, 0, frames, groups)
