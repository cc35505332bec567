"""Times the SDR layer's frame-parallel contractions (srf_route_sdr_pose / _gx / _gw)
on one frame range of the C3 / C5 stack, alone on the GPU (the kernel family the
library picks per din; A/B other families with SRF_LIB_PATH=ab/x.so builds).
    python scripts/bench_sdr_gemm.py [--shapes c3,c5] [--reps 20]"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from srf_amd import _lib  # noqa: E402

SHAPES = {   # B, T, N, din, lpad, rpad, J, dout, frames per range
    'c3': (28, 200, 16, 32, 2, 2, 16, 32, 20),
    'c5': (28, 200, 16, 64, 20, 20, 16, 64, 20),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--shapes', default='c3,c5')
    ap.add_argument('--reps', type=int, default=20)
    a = ap.parse_args()
    L = _lib.lib()
    dev = torch.device('cuda:0')
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    for name in a.shapes.split(','):
        B, T, N, din, lp, rp, J, D, nt = SHAPES[name]
        in_n, JD = N * (lp + rp + 1), J * D
        t0, t1 = 80, 80 + nt
        emb = torch.randn(B, T, N, din, device=dev) * 0.5
        W = torch.randn(in_n, JD, din, device=dev) * 0.1
        bias = torch.randn(in_n, JD, device=dev) * 0.1
        u = torch.empty(B * nt * in_n * JD, device=dev)
        WT = torch.empty_like(W)
        gW = torch.zeros_like(W)
        gb = torch.zeros_like(bias)
        gemb = torch.zeros_like(emb)
        _lib.check(L.srf_route_sdr_transpose_w(p(W), in_n, J, D, din, p(WT), st), 'tw')
        flop = 2.0 * B * nt * in_n * JD * din
        calls = {
            'pose': lambda: L.srf_route_sdr_pose(p(emb), p(W), p(bias), B, T, N, din, lp, rp, J, D, t0, t1, p(u), t0,
                                                 nt, st),
            'gx': lambda: L.srf_route_sdr_gx(p(u), t0, nt, p(WT), B, T, N, din, lp, rp, J, D, t0, t1, p(gemb), st),
            'gw': lambda: L.srf_route_sdr_gw(p(u), t0, nt, p(emb), B, T, N, din, lp, rp, J, D, t0, t1, 1, p(gW),
                                             p(gb), st),
        }
        for lib_path in (_lib.LIB_PATH,):
            res = {}
            for k, fn in calls.items():
                _lib.check(fn(), k)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    _lib.check(fn(), k)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / a.reps
                res[k] = {'us': round(us, 1), 'tflops': round(flop / us / 1e6, 1)}
            print(json.dumps({'shape': name, 'lib': lib_path, 'gflop': round(flop / 1e9, 2), **res}), flush=True)


if __name__ == '__main__':
    main()
