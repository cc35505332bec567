"""Plain-PyTorch fp32/fp64 references of the fused HIP kernels (test-only).

Same math as the reference TF graph (sequence_router.py:44-82 and
sequence_router_naive.py:129-193), written with torch autograd ops, plus a
numpy restatement of the counter-based dropout RNG of srf_amd/csrc/srf_rng.h so
GPU dropout masks can be reproduced bit-exactly on the host.
"""
import numpy as np
import torch
import torch.nn.functional as F

STREAMS = dict(conv0a=0, conv0b=1, conv1a=2, conv1b=3, encaps1=4, encaps2=5, input=6, mid0=7)
M32 = 0xFFFFFFFF


def _mix32(x):
    x = np.asarray(x, dtype=np.uint64) & np.uint64(M32)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7feb352d)) & np.uint64(M32)
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846ca68b)) & np.uint64(M32)
    x ^= x >> np.uint64(16)
    return x


def rng_uniform(seed, stream, n):
    """srf_uniform(seed, stream, idx) of srf_rng.h for idx in [0, n)."""
    seed = int(seed)
    k = int(_mix32((seed & M32) ^ int(_mix32(((seed >> 32) & M32) ^ ((stream * 0x9E3779B9 + 0x7F4A7C15) & M32)))))
    idx = np.arange(n, dtype=np.uint64)
    h = _mix32(_mix32((idx + np.uint64(k)) & np.uint64(M32)) ^ np.uint64(k))
    return (h >> np.uint64(8)).astype(np.float64) * (1.0 / 16777216.0)


def dropout_mult(seed, stream, shape, p):
    u = rng_uniform(seed, stream, int(np.prod(shape)))
    keep = (u.astype(np.float32) >= np.float32(p))
    return (keep.astype(np.float64) / (1.0 - p)).reshape(shape)


def dropout_mult_pair(seed, stream_a, shape, p):
    """srf_keep2 of srf_rng.h: both maxout branches from one hash keyed by stream_a
    (its high / low 16 bits)."""
    seed = int(seed)
    k = int(_mix32((seed & M32) ^ int(_mix32(((seed >> 32) & M32) ^ ((stream_a * 0x9E3779B9 + 0x7F4A7C15) & M32)))))
    idx = np.arange(int(np.prod(shape)), dtype=np.uint64)
    h = _mix32(_mix32((idx + np.uint64(k)) & np.uint64(M32)) ^ np.uint64(k))
    ua = (h >> np.uint64(16)).astype(np.float32) * np.float32(1.0 / 65536.0)
    ub = (h & np.uint64(0xFFFF)).astype(np.float32) * np.float32(1.0 / 65536.0)
    return tuple(((u >= np.float32(p)).astype(np.float64) / (1.0 - p)).reshape(shape) for u in (ua, ub))


def same_pad(n, k, s):
    out = -(-n // s)
    total = max((out - 1) * s + k - n, 0)
    return out, total // 2, total - total // 2


def conv2d_same(x, kern, bias, stride):
    _, H, W, _ = x.shape
    _, pt, pb = same_pad(H, kern.shape[0], stride)
    _, pl, pr = same_pad(W, kern.shape[1], stride)
    xn = F.pad(x.permute(0, 3, 1, 2), (pl, pr, pt, pb))
    return F.conv2d(xn, kern.permute(3, 2, 0, 1), bias, stride=stride).permute(0, 2, 3, 1)


def time_mask(inp_len, div, T, dtype):
    lens = (inp_len.to(torch.int64) + div - 1) // div
    return (torch.arange(T, device=inp_len.device)[None, :] < lens[:, None]).to(dtype)


def cnnfe(feats, inp_len, P, drop=None):
    """CapsulationLayer with BN in training mode; P: dict of tensors keyed
    conv0a_kernel ...; drop: dict of multiplier tensors or None."""
    x = feats.unsqueeze(-1)
    for k in range(2):
        x1 = conv2d_same(x, P[f'conv{k}a_kernel'], P[f'conv{k}a_bias'], 2)
        x2 = conv2d_same(x, P[f'conv{k}b_kernel'], P[f'conv{k}b_bias'], 2)
        if drop is not None:
            x1 = x1 * drop[f'conv{k}a']
            x2 = x2 * drop[f'conv{k}b']
        x = torch.maximum(x1, x2)
        m = time_mask(inp_len, 2 ** (k + 1), x.shape[1], x.dtype)[:, :, None, None]
        x = x * m
        mu = x.mean(dim=(0, 1, 2))
        var = x.var(dim=(0, 1, 2), unbiased=False)
        x = (x - mu) * torch.rsqrt(var + 1e-3) * P[f'bn{k}_gamma'] + P[f'bn{k}_beta']
        x = x * m
    return x


def squash(s, dim=-1):
    n2 = torch.sum(s * s, dim=dim, keepdim=True)
    return n2 / (1.0 + n2) * (s / torch.sqrt(n2 + 1e-7))


def layer_norm(x, gamma, beta):
    return F.layer_norm(x, x.shape[-1:], gamma, beta, 1e-3)


def primary_caps(X, inp_len, P, PH, PD, drop=None):
    """naive:129-142 on X [B,T,F2,C]; drop: dict with encaps1/encaps2/input multipliers."""
    B, T = X.shape[:2]
    e = X.reshape(B, T, -1) @ P['proj_kernel'] + P['proj_bias']
    e = e.unsqueeze(-1)
    e1 = conv2d_same(e, P['encaps1_kernel'], P['encaps1_bias'], 1)
    e2 = conv2d_same(e, P['encaps2_kernel'], P['encaps2_bias'], 1)
    if drop is not None:
        e1 = e1 * drop['encaps1']
        e2 = e2 * drop['encaps2']
    m = torch.maximum(e1, e2) * time_mask(inp_len, 4, T, e.dtype)[:, :, None, None]
    z = layer_norm(squash(m).reshape(B, T, PH * PD), P['ln_input_gamma'], P['ln_input_beta'])
    if drop is not None:
        z = z * drop['input']
    return z.reshape(B, T, PH, PD)


def capsnorm(v, gamma, beta, drop=None):
    B, T, J, D = v.shape
    y = layer_norm(v.reshape(B, T, J * D), gamma, beta)
    if drop is not None:
        y = y * drop
    return y.reshape(B, T, J, D)


def caps_head(v, gm, bm, go, bo, drop=None):
    y = capsnorm(v, gm, bm, drop)
    length = torch.sqrt(torch.sum(y * y, dim=-1) + 1e-7)
    return layer_norm(length, go, bo)
