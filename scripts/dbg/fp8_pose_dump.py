"""Dump the fp8 pose kernel's output next to its inputs (the case of
tests/test_route_sdr_gpu.py test_sdr_pose_fp8_matches_emulation) for offline
comparison with oracle/srf_oracle.pose_fp8:  python scripts/dbg/fp8_pose_dump.py OUT.npz"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from srf_amd import _lib  # noqa: E402

out = sys.argv[1]
dev = torch.device('cuda:0')
L = _lib.lib()
res = {}
for din, J, D in ((64, 16, 64), (32, 16, 32)):
    B, T, N, lp, rp = 2, 7, 3, 1, 2
    in_n, JD = N * (lp + rp + 1), J * D
    rng = np.random.default_rng(31)
    emb = (rng.standard_normal((B, T, N, din)) * 2.0 ** rng.uniform(-20, 4, (B, T, N, 1))).astype(np.float32)
    emb[0, 3] = 0.0
    W = (rng.standard_normal((in_n, JD, din)) * 0.1 * 2.0 ** rng.uniform(-20, 4, (in_n, JD, 1))).astype(np.float32)
    bias = (rng.standard_normal((in_n, JD)) * 0.1).astype(np.float32)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    te, tW, tb = (torch.tensor(a, device=dev) for a in (emb, W, bias))
    u = torch.full((B * T * in_n * JD,), float('nan'), device=dev)
    r = _lib.SdrRange(t0=0, t1=T, emb=p(te), W=p(tW), bias=p(tb), u=p(u), v0=0, vn=T, u_bf16=0)
    _lib.check(L.srf_route_sdr_pose_n((_lib.SdrRange * 1)(r), 1, B, T, N, din, lp, rp, J, D, 1, st), 'pose')
    torch.cuda.synchronize()
    res[f'u_{din}'] = u.cpu().numpy()
print('saved', out, {k: v.shape for k, v in res.items()})
np.savez(out, **res)
