"""torch.autograd wrappers around the C ABI (device memory from torch's caching
allocator, launches on torch's current HIP stream)."""
import torch

from . import _lib


def _ptr(t):
    return ctypes_void(t.data_ptr())


def ctypes_void(addr):
    import ctypes
    return ctypes.c_void_p(addr)


def _stream():
    return ctypes_void(torch.cuda.current_stream().cuda_stream)


def _check_dev(name, t, shape):
    if not t.is_cuda:
        raise ValueError(f'{name} must be a HIP device tensor (no CPU path exists)')
    if t.dtype != torch.float32:
        raise ValueError(f'{name} must be float32, got {t.dtype}')
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f'{name} has shape {tuple(t.shape)}, expected {tuple(shape)}')
    if not t.is_contiguous():
        raise ValueError(f'{name} must be contiguous')


class RouteGeom:
    """Static geometry of one DR layer (sequence_router_naive.py:146-147)."""

    def __init__(self, B, T, N, din, lpad, rpad, J, dout, iters, mask_first, n_chunks=0):
        self.B, self.T, self.N, self.din = B, T, N, din
        self.lpad, self.rpad, self.J, self.dout = lpad, rpad, J, dout
        self.iters, self.mask_first = iters, int(bool(mask_first))
        self.in_n = N * (lpad + rpad + 1)
        self.timing = None   # optional (starts, stops) hipEvent_t arrays for the profiling hook
        L = _lib.lib()
        if n_chunks <= 0:
            n_chunks = L.srf_route_dr_auto_chunks(B, T, N, din, lpad, rpad, J, dout)
        self.n_chunks = n_chunks

    def args(self):
        return (self.B, self.T, self.N, self.din, self.lpad, self.rpad, self.J, self.dout, self.iters,
                self.mask_first, self.n_chunks)

    def ws_args(self):
        return (self.B, self.T, self.N, self.din, self.lpad, self.rpad, self.J, self.dout, self.iters,
                self.n_chunks)


class DynamicRouting(torch.autograd.Function):
    """window -> pose (u = W x + b) -> ``iters`` DR iterations, one layer.

    emb [B,T,N,din] -> v [B,T,J,dout] (the last iteration's squashed capsules)."""

    @staticmethod
    def forward(ctx, emb, W, bias, geom):
        g = geom
        _check_dev('emb', emb, (g.B, g.T, g.N, g.din))
        _check_dev('W', W, (g.in_n, g.J, g.dout, g.din))
        _check_dev('bias', bias, (g.in_n, g.J, g.dout))
        L = _lib.lib()
        dev = emb.device
        v = torch.empty((g.B, g.T, g.J, g.dout), device=dev, dtype=torch.float32)
        saved = torch.empty(L.srf_route_dr_saved_floats(g.B, g.T, g.J, g.dout, g.iters), device=dev,
                            dtype=torch.float32)
        ws_bytes = L.srf_route_dr_fwd_workspace(*g.ws_args())
        ws = torch.empty(max(ws_bytes, 16), device=dev, dtype=torch.uint8)
        if g.timing is not None:
            starts, stops, n = g.timing.pop(0)
            _lib.check(L.srf_route_dr_set_timing_events(starts, stops, n), 'set_timing_events')
            if not g.timing:
                g.timing = None
        rc = L.srf_route_dr_fwd(_ptr(emb), _ptr(W), _ptr(bias), *g.args(), _ptr(v), _ptr(saved), _ptr(ws),
                                ws_bytes, _stream())
        _lib.check(rc, 'srf_route_dr_fwd')
        ctx.geom = g
        ctx.save_for_backward(emb, W, bias, saved)
        return v

    @staticmethod
    def backward(ctx, g_v):
        emb, W, bias, saved = ctx.saved_tensors
        g = ctx.geom
        g_v = g_v.contiguous()
        L = _lib.lib()
        g_emb = torch.empty_like(emb)
        g_W = torch.empty_like(W)
        g_b = torch.empty_like(bias)
        ws_bytes = L.srf_route_dr_bwd_workspace(*g.ws_args())
        ws = torch.empty(ws_bytes, device=emb.device, dtype=torch.uint8)
        rc = L.srf_route_dr_bwd(_ptr(emb), _ptr(W), _ptr(bias), *g.args(), _ptr(saved), _ptr(g_v), _ptr(g_emb),
                                _ptr(g_W), _ptr(g_b), _ptr(ws), ws_bytes, _stream())
        _lib.check(rc, 'srf_route_dr_bwd')
        return g_emb, g_W, g_b, None


def dynamic_routing(emb, W, bias, geom):
    return DynamicRouting.apply(emb, W, bias, geom)
