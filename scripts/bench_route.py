"""Microbenchmark of one DR routing layer (forward + backward) through the C ABI.

    python scripts/bench_route.py [--layer 3] [--chunks 0,3,8] [--iters 20]

Times srf_route_dr_fwd / srf_route_dr_bwd with HIP events (torch.cuda.Event on
the launch stream) at the BASELINE C2 shapes (B=17, T'=80)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from srf_amd.ops import RouteGeom, dynamic_routing  # noqa: E402

SHAPES = {  # (N, D, lpad, rpad, J, iters, mask_first)
    1: (8, 16, 4, 4, 8, 3, False),
    3: (8, 16, 4, 4, 63, 3, True),
    'c4': (16, 32, 2, 2, 16, 3, False),
    'c4last': (16, 32, 2, 2, 32, 3, True),
}


def run(layer, chunks, iters, B, T):
    N, D, lp, rp, J, it, mf = SHAPES[layer]
    dev = torch.device('cuda')
    in_n = N * (lp + rp + 1)
    emb = (torch.randn(B, T, N, D, device=dev) * 0.5).requires_grad_()
    W = (torch.randn(in_n, J, D, D, device=dev) * 0.1).requires_grad_()
    b = (torch.randn(in_n, J, D, device=dev) * 0.1).requires_grad_()
    g = RouteGeom(B, T, N, D, lp, rp, J, D, it, mf, chunks)
    gv = torch.randn(B, T, J, D, device=dev)
    for _ in range(3):
        v = dynamic_routing(emb, W, b, g)
        v.backward(gv)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    fw = bw = 0.0
    for _ in range(iters):
        e[0].record()
        v = dynamic_routing(emb, W, b, g)
        e[1].record()
        v.backward(gv)
        e[2].record()
        torch.cuda.synchronize()
        fw += e[0].elapsed_time(e[1])
        bw += e[1].elapsed_time(e[2])
    F = B * T
    pose = 2.0 * F * in_n * J * D * D
    print(f'layer {layer} chunks={g.n_chunks:3d}: fwd {fw / iters * 1e3:8.1f} us  bwd {bw / iters * 1e3:8.1f} us  '
          f'(executed pose MFMA per fwd pass {pose / 1e9:.2f} GF -> {pose * it / (fw / iters * 1e-3) / 1e12:.1f} TF/s)')


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--layers', default='1,3')
    ap.add_argument('--chunks', default='0')
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--B', type=int, default=17)
    ap.add_argument('--T', type=int, default=80)
    a = ap.parse_args()
    for layer in a.layers.split(','):
        layer = int(layer) if layer.isdigit() else layer
        for c in a.chunks.split(','):
            run(layer, int(c), a.iters, a.B, a.T)
