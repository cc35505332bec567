"""torch.autograd wrappers around the C ABI (device memory from torch's caching
allocator, launches on torch's current HIP stream)."""
import ctypes
import os

import torch

from . import _lib


def _ptr(t):
    return ctypes_void(t.data_ptr())


def ctypes_void(addr):
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


def _grad_target(p):
    """Where a backward kernel writes the gradient of parameter p: straight into
    the model's flat gradient buffer when p is one of its views (then autograd is
    handed None and adds nothing), else a fresh tensor returned to autograd."""
    if getattr(p, '_srf_flat', False) and p.grad is not None:
        return p.grad, True
    return torch.empty_like(p), False


def _returned(target_flags):
    return [None if inplace else t for t, inplace in target_flags]


class RouteGeom:
    """Static geometry of one DR layer (sequence_router_naive.py:146-147)."""

    def __init__(self, B, T, N, din, lpad, rpad, J, dout, iters, mask_first, n_chunks=0):
        self.B, self.T, self.N, self.din = B, T, N, din
        self.lpad, self.rpad, self.J, self.dout = lpad, rpad, J, dout
        self.iters, self.mask_first = iters, int(bool(mask_first))
        self.in_n = N * (lpad + rpad + 1)
        self.timing = None   # optional (starts, stops) hipEvent_t arrays for the profiling hook
        # a training forward keeps the couplings for the backward (srf_route_dr_fwd_ex's
        # coupling storage); False: it keeps nothing and the backward recomputes them
        self.store_couplings = True
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


# DR gW / gbias (srf_route_dr_bwd_weights_ex) on a side stream beside the layers below.
# Each layer's launch is deferred to the next DR backward (or the gradient buckets' next
# collective, or dr_side_join), so the backward's next kernel is captured first
# (STACK_CAPTURE_ORDER).  C4 8.31 -> 8.22 ms (r05ci).  OFF since round 6, as CNNFE_WGRAD_SIDE: with the side
# launches on, replays of a captured step gave W / b gradients off by 1e-3 .. 5e-2 of
# their max in up to ~10 % of replays on some boxes (scripts/dbg/graph_race.py: two
# processes x 150 replays of the C2-mini step), none on others; keeping the launch's
# tensors until the join or waiting for the issuing stream's tail did not remove it
# reliably; one stream: none in 598 replays.  Cause not found; bench --side-streams
# turns both on (A/B; C4 7.80 -> 7.57 ms, r06gd).
DR_GW_SIDE = False
_dr_side = {}        # device index -> side stream
_dr_pending = []     # (device, event, launch(stream_ptr), tensors the launch reads)
_dr_keep = []        # tensors of issued side launches, released once the side stream is joined
# diagnostics (A/B): SRF_SIDE_KEEP=0 releases them at issue (before round 6);
# SRF_SIDE_WAIT=tail waits for the issuing stream's tail instead of the launch's event
_SIDE_KEEP = os.environ.get('SRF_SIDE_KEEP', '1') != '0'
_SIDE_WAIT = os.environ.get('SRF_SIDE_WAIT', 'event')


def _dr_side_stream(dev):
    s = _dr_side.get(dev.index)
    if s is None:
        s = _dr_side[dev.index] = torch.cuda.Stream(device=dev)
    return s


def _dr_issue_pending():
    while _dr_pending:
        dev, ev, launch, keep = _dr_pending.pop(0)
        side = _dr_side_stream(dev)
        if _SIDE_WAIT == 'tail':
            side.wait_stream(torch.cuda.current_stream(dev))
        else:
            side.wait_event(ev)
        launch(ctypes_void(side.cuda_stream))
        for t in keep:
            if t is not None:
                t.record_stream(side)   # the allocator must not hand these out before the launch ran
        # ... and the tensors stay referenced until the side stream is joined: released
        # here, inside a capture, a block went back to the graph's pool, a later
        # allocation of the same capture took it, and in ~5 % of replays the side branch
        # read memory the main branch was rewriting -- W / b gradients off by 1e-4 .. 1e-1
        # of their max (scripts/dbg/graph_race.py, tests/test_graph_replay_gpu.py)
        if _SIDE_KEEP:
            _dr_keep.append(keep)


def dr_side_join():
    """Issue the deferred DR gW launches and make the current stream wait for them
    (the caller's backward is complete; gradients are read next).  The backward does
    this itself at its end (_dr_backward_done); calling it again is harmless."""
    _dr_issue_pending()
    for s in _dr_side.values():
        torch.cuda.current_stream(s.device).wait_stream(s)
    _dr_keep.clear()


_dr_state = {'queued': False, 'main': None}


def _dr_backward_done():
    """End-of-backward callback (queued by the first deferring DR backward): issue what
    is still deferred and make the backward's stream wait for the side stream, so every
    gradient is complete when backward() returns, whoever called it."""
    _dr_state['queued'] = False
    main, _dr_state['main'] = _dr_state['main'], None
    _dr_issue_pending()
    if main is not None:
        s = _dr_side.get(main.device.index)
        if s is not None:
            main.wait_stream(s)
            _dr_keep.clear()


def dr_reset():
    """Drop deferred DR gW launches and the end-of-backward flag after a backward that
    did not complete (a failed capture): the stale launches hold events recorded in
    the dead capture, and a flag left set would keep later backwards from installing
    their join.  GraphedTrainStep calls it when its capture raises."""
    _dr_pending.clear()
    _dr_keep.clear()
    _dr_state['queued'] = False
    _dr_state['main'] = None


def _defer_side(dev, ev, launch, keep):
    """Queue ``launch(side stream)`` behind ``ev``; issued by the next deferring op, the
    gradient buckets' next collective, or the end-of-backward callback queued here."""
    _dr_pending.append((dev, ev, launch, keep))
    _dr_state['main'] = torch.cuda.current_stream(dev)
    if not _dr_state['queued']:
        torch.autograd.Variable._execution_engine.queue_callback(_dr_backward_done)
        _dr_state['queued'] = True


class DynamicRouting(torch.autograd.Function):
    """window -> pose (u = W x + b) -> ``iters`` DR iterations, one layer.

    emb [B,T,N,din] -> v [B,T,J,dout] (the last iteration's squashed capsules)."""

    @staticmethod
    def forward(ctx, emb, W, bias, geom, need_bwd=True):
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
        # couplings of iterations r >= 1 for the backward (training only: a forward
        # under no_grad or on non-trainable inputs stores nothing; grad mode is off
        # inside Function.forward, so the caller decides, see dynamic_routing)
        nc = L.srf_route_dr_coupling_floats(g.B, g.T, g.N, g.din, g.lpad, g.rpad, g.J, g.dout, g.iters) \
            if need_bwd and g.store_couplings else 0
        cpl = torch.empty(nc, device=dev, dtype=torch.float32) if nc else None
        rc = L.srf_route_dr_fwd_ex(_ptr(emb), _ptr(W), _ptr(bias), *g.args(), _ptr(v), _ptr(saved),
                                   _ptr(cpl) if cpl is not None else None, _ptr(ws), ws_bytes, _stream())
        _lib.check(rc, 'srf_route_dr_fwd_ex')
        ctx.geom = g
        ctx.params = (W, bias)
        ctx.couplings = cpl
        ctx.save_for_backward(emb, W, bias, saved)
        return v

    @staticmethod
    def backward(ctx, g_v):
        emb, W, bias, saved = ctx.saved_tensors
        g = ctx.geom
        g_v = g_v.contiguous()
        L = _lib.lib()
        g_emb = torch.empty_like(emb)
        tW, tb = _grad_target(ctx.params[0]), _grad_target(ctx.params[1])
        g_W, g_b = tW[0], tb[0]
        ws_bytes = L.srf_route_dr_bwd_workspace(*g.ws_args())
        ws = torch.empty(ws_bytes, device=emb.device, dtype=torch.uint8)
        cpl = ctx.couplings
        ctx.couplings = None
        cp = _ptr(cpl) if cpl is not None else None
        _dr_issue_pending()   # the layer above's gW, behind the kernels enqueued since its gu pass
        # only where gW / gbias land in the model's flat gradient buffer (written in place,
        # autograd handed None): a returned gradient is consumed at once on this stream
        if DR_GW_SIDE and cpl is not None and tW[1] and tb[1]:
            rc = L.srf_route_dr_bwd_data_ex(_ptr(emb), _ptr(W), _ptr(bias), *g.args(), _ptr(saved), cp, _ptr(g_v),
                                            _ptr(g_emb), _ptr(ws), ws_bytes, _stream())
            _lib.check(rc, 'srf_route_dr_bwd_data_ex')
            ev = getattr(g, '_gw_event', None)   # kept with the geometry: a captured step's events outlive it
            if ev is None:
                ev = g._gw_event = torch.cuda.Event()
            ev.record()

            def launch(st, emb=emb, saved=saved, cpl=cpl, g_W=g_W, g_b=g_b, ws=ws):
                _lib.check(L.srf_route_dr_bwd_weights_ex(_ptr(emb), *g.args(), _ptr(saved), _ptr(cpl), _ptr(g_W),
                                                         _ptr(g_b), _ptr(ws), ws_bytes, st),
                           'srf_route_dr_bwd_weights_ex')
            _defer_side(emb.device, ev, launch, (emb, saved, cpl, ws))
        else:
            rc = L.srf_route_dr_bwd_ex(_ptr(emb), _ptr(W), _ptr(bias), *g.args(), _ptr(saved), cp, _ptr(g_v),
                                       _ptr(g_emb), _ptr(g_W), _ptr(g_b), _ptr(ws), ws_bytes, _stream())
            _lib.check(rc, 'srf_route_dr_bwd_ex')
        return (g_emb, *_returned([tW, tb]), None, None)


def dynamic_routing(emb, W, bias, geom):
    need_bwd = torch.is_grad_enabled() and (emb.requires_grad or W.requires_grad or bias.requires_grad)
    return DynamicRouting.apply(emb, W, bias, geom, need_bwd)


class SequentialRouting(torch.autograd.Function):
    """window -> pose -> SDR (frames routed in order, naive:162-170 with
    body_context / pad_body_context), one layer.  emb [B,T,N,din] -> v [B,T,J,dout]."""

    @staticmethod
    def forward(ctx, emb, W, bias, geom):
        g = geom
        _check_dev('emb', emb, (g.B, g.T, g.N, g.din))
        _check_dev('W', W, (g.in_n, g.J, g.dout, g.din))
        _check_dev('bias', bias, (g.in_n, g.J, g.dout))
        L = _lib.lib()
        dev = emb.device
        v = torch.empty((g.B, g.T, g.J, g.dout), device=dev, dtype=torch.float32)
        saved = torch.empty(L.srf_route_sdr_saved_floats(g.B, g.T, g.J, g.dout), device=dev, dtype=torch.float32)
        geo = (g.B, g.T, g.N, g.din, g.lpad, g.rpad, g.J, g.dout)
        ws_bytes = L.srf_route_sdr_fwd_workspace(*geo)
        ws = torch.empty(ws_bytes, device=dev, dtype=torch.uint8)
        rc = L.srf_route_sdr_fwd(_ptr(emb), _ptr(W), _ptr(bias), *geo, g.iters, g.mask_first, _ptr(v), _ptr(saved),
                                 _ptr(ws), ws_bytes, _stream())
        _lib.check(rc, 'srf_route_sdr_fwd')
        ctx.geom = g
        ctx.params = (W, bias)
        ctx.save_for_backward(emb, W, bias, saved)
        return v

    @staticmethod
    def backward(ctx, g_v):
        emb, W, bias, saved = ctx.saved_tensors
        g = ctx.geom
        g_v = g_v.contiguous()
        L = _lib.lib()
        g_emb = torch.empty_like(emb)
        tW, tb = _grad_target(ctx.params[0]), _grad_target(ctx.params[1])
        geo = (g.B, g.T, g.N, g.din, g.lpad, g.rpad, g.J, g.dout)
        ws_bytes = L.srf_route_sdr_bwd_workspace(*geo, g.iters)
        ws = torch.empty(ws_bytes, device=emb.device, dtype=torch.uint8)
        rc = L.srf_route_sdr_bwd(_ptr(emb), _ptr(W), _ptr(bias), *geo, g.iters, g.mask_first, _ptr(saved),
                                 _ptr(g_v), _ptr(g_emb), _ptr(tW[0]), _ptr(tb[0]), _ptr(ws), ws_bytes, _stream())
        _lib.check(rc, 'srf_route_sdr_bwd')
        return (g_emb, *_returned([tW, tb]), None)


def sequential_routing(emb, W, bias, geom):
    return SequentialRouting.apply(emb, W, bias, geom)


# ---------------------------------------------------------------------------
# CNN front end (CapsulationLayer)
CNNFE_PARAMS = ('conv0a_kernel', 'conv0a_bias', 'conv0b_kernel', 'conv0b_bias', 'bn0_gamma', 'bn0_beta',
                'conv1a_kernel', 'conv1a_bias', 'conv1b_kernel', 'conv1b_bias', 'bn1_gamma', 'bn1_beta')


# Stage-2 weight gradient (split-transpose, wgrad, reduce: ~240 us at C4) on the side
# stream beside the stage-2 data gradient and stage 1 (srf_cnnfe_bwd_parts; the parts share
# no workspace).  False: one srf_cnnfe_bwd call (bench --cnnfe-wgrad-inline, for A/B).
CNNFE_WGRAD_SIDE = False   # off since round 6: see DR_GW_SIDE
_cnnfe_events = {}   # device index -> the event after the prep part (one CNN-FE per step)


def cnnfe_out_dims(T, feat_dim):
    import ctypes
    t2, f2 = ctypes.c_int(), ctypes.c_int()
    _lib.check(_lib.lib().srf_cnnfe_out_dims(T, feat_dim, ctypes.byref(t2), ctypes.byref(f2)), 'srf_cnnfe_out_dims')
    return t2.value, f2.value


class CnnFe(torch.autograd.Function):
    """feats [B,T,F] -> mask2(BN2(maxout2(mask1(BN1(maxout1(feats)))))) [B,T2,F2,64]."""

    @staticmethod
    def forward(ctx, feats, inp_len_i32, moving, training, drop_p, seed, *params):
        B, T, Fd = feats.shape
        _check_dev('feats', feats, (B, T, Fd))
        L = _lib.lib()
        T2, F2 = cnnfe_out_dims(T, Fd)
        dev = feats.device
        out = torch.empty((B, T2, F2, 64), device=dev, dtype=torch.float32)
        sb = L.srf_cnnfe_saved_bytes(B, T, Fd, 64)
        saved = torch.empty(sb, device=dev, dtype=torch.uint8)
        wb = L.srf_cnnfe_fwd_workspace(B, T, Fd, 64)
        ws = torch.empty(wb, device=dev, dtype=torch.uint8)
        rc = L.srf_cnnfe_fwd(_ptr(feats), _ptr(inp_len_i32), B, T, Fd, 64, *[_ptr(p) for p in params],
                             *[_ptr(m) for m in moving], int(bool(training)), float(drop_p), int(seed), _ptr(out),
                             _ptr(saved), sb, _ptr(ws), wb, _stream())
        _lib.check(rc, 'srf_cnnfe_fwd')
        ctx.meta = (B, T, Fd, float(drop_p) if training else 0.0, int(seed))
        ctx.params = params
        ctx.save_for_backward(feats, inp_len_i32, saved, *params)
        return out

    @staticmethod
    def backward(ctx, g_out):
        feats, inp_len, saved, *params = ctx.saved_tensors
        B, T, Fd, drop_p, seed = ctx.meta
        P = dict(zip(CNNFE_PARAMS, params))
        targets = [_grad_target(p) for p in ctx.params]
        G = dict(zip(CNNFE_PARAMS, [t for t, _ in targets]))
        L = _lib.lib()
        wb = L.srf_cnnfe_bwd_workspace(B, T, Fd, 64)
        ws = torch.empty(wb, device=feats.device, dtype=torch.uint8)
        g_out = g_out.contiguous()
        args = (_ptr(feats), _ptr(inp_len), B, T, Fd, 64, _ptr(P['bn0_gamma']), _ptr(P['conv1a_kernel']),
                _ptr(P['conv1b_kernel']), _ptr(P['bn1_gamma']), drop_p, seed, _ptr(saved), _ptr(g_out),
                *[_ptr(G[k]) for k in CNNFE_PARAMS], _ptr(ws), wb)
        inplace = dict(zip(CNNFE_PARAMS, [t[1] for t in targets]))
        if CNNFE_WGRAD_SIDE and inplace['conv1a_kernel'] and inplace['conv1b_kernel']:
            _dr_issue_pending()
            _lib.check(L.srf_cnnfe_bwd_parts(1, *args, _stream()), 'srf_cnnfe_bwd_parts(prep)')
            dev = feats.device
            ev = _cnnfe_events.get(dev.index)
            if ev is None:
                ev = _cnnfe_events[dev.index] = torch.cuda.Event()
            ev.record()
            _lib.check(L.srf_cnnfe_bwd_parts(2, *args, _stream()), 'srf_cnnfe_bwd_parts(data)')

            def launch(st):
                _lib.check(L.srf_cnnfe_bwd_parts(4, *args, st), 'srf_cnnfe_bwd_parts(wgrad)')
            _defer_side(dev, ev, launch, (feats, inp_len, saved, g_out, ws))
        else:
            _lib.check(L.srf_cnnfe_bwd(*args, _stream()), 'srf_cnnfe_bwd')
        return (None, None, None, None, None, None, *_returned(targets))


def cnnfe(feats, inp_len_i32, params, moving, training, drop_p, seed):
    """params: the 12 tensors of CNNFE_PARAMS in order; moving: (mm0, mv0, mm1, mv1)."""
    return CnnFe.apply(feats, inp_len_i32, moving, training, drop_p, seed, *params)


# ---------------------------------------------------------------------------
# Primary capsules
CAPS_PARAMS = ('proj_kernel', 'proj_bias', 'encaps1_kernel', 'encaps1_bias', 'encaps2_kernel', 'encaps2_bias',
               'ln_input_gamma', 'ln_input_beta')


class PrimaryCaps(torch.autograd.Function):
    """X [B,T,F2,64] -> z [B,T,PH,PD] (naive:129-142)."""

    @staticmethod
    def forward(ctx, X, inp_len_i32, PH, PD, training, p_caps, p_in, seed, variant, *params):
        proj_scale, pos_enc = variant
        B, T = X.shape[:2]
        K = X.shape[2] * X.shape[3]
        _check_dev('X', X, tuple(X.shape))
        L = _lib.lib()
        z = torch.empty((B, T, PH, PD), device=X.device, dtype=torch.float32)
        sb = L.srf_primary_caps_saved_bytes(B, T, PH, PD)
        saved = torch.empty(sb, device=X.device, dtype=torch.uint8)
        tr = int(bool(training))
        rc = L.srf_primary_caps_fwd_ex(_ptr(X), _ptr(inp_len_i32), B, T, K, PH, PD, *[_ptr(p) for p in params], tr,
                                       float(p_caps), float(p_in), int(seed), float(proj_scale), int(bool(pos_enc)),
                                       _ptr(z), _ptr(saved), sb, _stream())
        _lib.check(rc, 'srf_primary_caps_fwd_ex')
        ctx.meta = (B, T, K, PH, PD, tr, float(p_caps), float(p_in), int(seed), float(proj_scale))
        ctx.params = params
        ctx.save_for_backward(X, inp_len_i32, saved, *params)
        return z

    @staticmethod
    def backward(ctx, g_z):
        X, inp_len, saved, *params = ctx.saved_tensors
        B, T, K, PH, PD, tr, p_caps, p_in, seed, proj_scale = ctx.meta
        P = dict(zip(CAPS_PARAMS, params))
        L = _lib.lib()
        g_X = torch.empty_like(X)
        targets = [_grad_target(p) for p in ctx.params]
        G = dict(zip(CAPS_PARAMS, [t for t, _ in targets]))
        wb = L.srf_primary_caps_bwd_workspace(B, T, K, PH, PD)
        ws = torch.empty(wb, device=X.device, dtype=torch.uint8)
        rc = L.srf_primary_caps_bwd_ex(_ptr(X), _ptr(inp_len), B, T, K, PH, PD, _ptr(P['proj_kernel']),
                                       _ptr(P['encaps1_kernel']), _ptr(P['encaps2_kernel']),
                                       _ptr(P['ln_input_gamma']), _ptr(P['ln_input_beta']), tr, p_caps, p_in, seed,
                                       proj_scale, _ptr(saved), _ptr(g_z.contiguous()), _ptr(g_X),
                                       *[_ptr(G[k]) for k in CAPS_PARAMS], _ptr(ws), wb, _stream())
        _lib.check(rc, 'srf_primary_caps_bwd_ex')
        return (g_X, None, None, None, None, None, None, None, None, *_returned(targets))


def primary_caps(X, inp_len_i32, PH, PD, training, p_caps, p_in, seed, params, proj_scale=1.0, pos_enc=False):
    """proj_scale / pos_enc: the einsum variant's sqrt(PH) scaling and positional
    encoding after proj_pe (sequence_router_einsum.py:129-131); 1 / off otherwise."""
    return PrimaryCaps.apply(X, inp_len_i32, PH, PD, training, p_caps, p_in, seed, (proj_scale, pos_enc), *params)


class CapsNorm(torch.autograd.Function):
    """y = drop(LN(v)) per frame over J*D (naive:187-191)."""

    @staticmethod
    def forward(ctx, v, gamma, beta, training, p, seed, layer):
        B, T, J, D = v.shape
        F, n = B * T, J * D
        L = _lib.lib()
        y = torch.empty_like(v)
        stat = torch.empty((F, 4), device=v.device, dtype=torch.float32)
        tr = int(bool(training))
        _lib.check(L.srf_capsnorm_fwd(_ptr(v), F, n, _ptr(gamma), _ptr(beta), tr, float(p), int(seed), int(layer),
                                      _ptr(y), _ptr(stat), _stream()), 'srf_capsnorm_fwd')
        ctx.meta = (F, n, tr, float(p), int(seed), int(layer))
        ctx.params = (gamma, beta)
        ctx.save_for_backward(v, gamma, beta, stat)
        return y

    @staticmethod
    def backward(ctx, g_y):
        v, gamma, beta, stat = ctx.saved_tensors
        F, n, tr, p, seed, layer = ctx.meta
        L = _lib.lib()
        g_v = torch.empty_like(v)
        targets = [_grad_target(p) for p in ctx.params]
        g_g, g_b = targets[0][0], targets[1][0]
        wb = L.srf_capsnorm_bwd_workspace(F, n, 0)
        ws = torch.empty(wb, device=v.device, dtype=torch.uint8)
        _lib.check(L.srf_capsnorm_bwd(_ptr(v), F, n, _ptr(gamma), _ptr(beta), tr, p, seed, layer, _ptr(stat),
                                      _ptr(g_y.contiguous()), _ptr(g_v), _ptr(g_g), _ptr(g_b), _ptr(ws), wb,
                                      _stream()), 'srf_capsnorm_bwd')
        return (g_v, *_returned(targets), None, None, None, None)


class CapsHead(torch.autograd.Function):
    """logits = LN_out(length_D(drop(LN_mid(v)))) (naive:187-193)."""

    @staticmethod
    def forward(ctx, v, gamma_mid, beta_mid, gamma_out, beta_out, training, p, seed, layer, length_eps=1e-7):
        B, T, J, D = v.shape
        F = B * T
        L = _lib.lib()
        logits = torch.empty((B, T, J), device=v.device, dtype=torch.float32)
        stat = torch.empty((F, 4), device=v.device, dtype=torch.float32)
        lens = torch.empty((F, J), device=v.device, dtype=torch.float32)
        tr = int(bool(training))
        _lib.check(L.srf_caps_head_fwd_ex(_ptr(v), F, J, D, _ptr(gamma_mid), _ptr(beta_mid), _ptr(gamma_out),
                                          _ptr(beta_out), tr, float(p), int(seed), int(layer), float(length_eps),
                                          _ptr(logits), _ptr(stat), _ptr(lens), _stream()), 'srf_caps_head_fwd_ex')
        ctx.meta = (F, J, D, tr, float(p), int(seed), int(layer))
        ctx.params = (gamma_mid, beta_mid, gamma_out, beta_out)
        ctx.save_for_backward(v, gamma_mid, beta_mid, gamma_out, beta_out, stat, lens)
        return logits

    @staticmethod
    def backward(ctx, g_logits):
        v, gm, bm, go, bo, stat, lens = ctx.saved_tensors
        F, J, D, tr, p, seed, layer = ctx.meta
        L = _lib.lib()
        g_v = torch.empty_like(v)
        targets = [_grad_target(p) for p in ctx.params]
        g_gm, g_bm, g_go, g_bo = (t for t, _ in targets)
        wb = L.srf_capsnorm_bwd_workspace(F, J * D, J)
        ws = torch.empty(wb, device=v.device, dtype=torch.uint8)
        _lib.check(L.srf_caps_head_bwd(_ptr(v), F, J, D, _ptr(gm), _ptr(bm), _ptr(go), tr, p, seed, layer,
                                       _ptr(stat), _ptr(lens), _ptr(g_logits.contiguous()), _ptr(g_v), _ptr(g_gm),
                                       _ptr(g_bm), _ptr(g_go), _ptr(g_bo), _ptr(ws), wb, _stream()),
                   'srf_caps_head_bwd')
        return (g_v, *_returned(targets), None, None, None, None, None)


class CtcLoss(torch.autograd.Function):
    """Per-utterance CTC NLL (blank = C-1 by the caller); the logit gradient is
    produced by the same kernel launch and scaled by the incoming per-utterance
    gradient in backward."""

    @staticmethod
    def forward(ctx, logits, labels_i32, label_len_i32, logit_len_i32, blank):
        B, T, C = logits.shape
        Lmax = labels_i32.shape[1]
        L = _lib.lib()
        nll = torch.empty(B, device=logits.device, dtype=torch.float32)
        need_grad = logits.requires_grad
        grad = torch.empty_like(logits) if need_grad else None
        wb = L.srf_ctc_workspace(B, T, C, Lmax)
        ws = torch.empty(wb, device=logits.device, dtype=torch.uint8)
        _lib.check(L.srf_ctc_loss(_ptr(logits.contiguous()), _ptr(labels_i32), _ptr(label_len_i32),
                                  _ptr(logit_len_i32), B, T, C, Lmax, int(blank), 1.0, _ptr(nll),
                                  _ptr(grad) if need_grad else None, _ptr(ws), wb, _stream()), 'srf_ctc_loss')
        if need_grad:
            ctx.save_for_backward(grad)
        return nll

    @staticmethod
    def backward(ctx, g_nll):
        (grad,) = ctx.saved_tensors
        return grad * g_nll[:, None, None], None, None, None, None


def _i32(t):
    return t if t.dtype == torch.int32 and t.is_contiguous() else t.to(torch.int32).contiguous()


def ctc_loss_and_grad(logits, labels, label_len, logit_len, blank, grad_scale):
    """(nll [B], grad_scale * d(sum nll)/d logits) without autograd."""
    B, T, C = logits.shape
    labels, label_len, logit_len = _i32(labels), _i32(label_len), _i32(logit_len)
    Lmax = labels.shape[1]
    L = _lib.lib()
    nll = torch.empty(B, device=logits.device, dtype=torch.float32)
    grad = torch.empty_like(logits)
    wb = L.srf_ctc_workspace(B, T, C, Lmax)
    ws = torch.empty(wb, device=logits.device, dtype=torch.uint8)
    _lib.check(L.srf_ctc_loss(_ptr(logits.detach()), _ptr(labels), _ptr(label_len), _ptr(logit_len), B, T, C, Lmax,
                              int(blank), float(grad_scale), _ptr(nll), _ptr(grad), _ptr(ws), wb, _stream()),
               'srf_ctc_loss')
    return nll, grad


def ctc_loss(logits, labels, label_len, logit_len, blank):
    return CtcLoss.apply(logits, _i32(labels), _i32(label_len), _i32(logit_len), blank)


# ---------------------------------------------------------------------------
# Fault word of the grouped SDR recurrences (srf_set_fault_flag): one per process
GROUP_RESERVE_CUS = 4   # CUs a grouped launch leaves free (srf_group.h kReserveCUs)
_FAULT = {}


def fault_flag(dev):
    """The process's device fault word on ``dev``, created and registered once
    (srf_set_fault_flag is process-wide; one process drives one GPU)."""
    dev = torch.device(dev)
    f = _FAULT.get(dev)
    if f is None:
        if _FAULT:
            raise RuntimeError(f'one process drives one GPU: the fault word already lives on {next(iter(_FAULT))}')
        f = torch.zeros(1, dtype=torch.int32, device=dev)
        _lib.check(_lib.lib().srf_set_fault_flag(f.data_ptr()), 'srf_set_fault_flag')
        _FAULT[dev] = f
    return f


def check_faults():
    """Raise if a grouped SDR recurrence gave up waiting for its members since the
    last check (its results, and every gradient computed from them, are wrong); the
    word is cleared.  Reads a device word: a synchronisation point."""
    for dev, f in _FAULT.items():
        if int(f.item()):
            f.zero_()
            raise RuntimeError('a grouped SDR recurrence timed out waiting for its workgroups (they were not '
                               'resident together): the step\'s results are wrong; run with fewer workgroups per '
                               'utterance (SdrStackPlan last_group) or less concurrent device work')


# ---------------------------------------------------------------------------
# SDR stack: every SDR layer and the LN + dropout between them, as a wavefront
class SdrStackPlan:
    """Static plan of an SDR stack (sequence_router_naive.py:145-191 with
    --model-caps-context, the per-layer LN / dropout of :187-191 between layers).

    The frames of each utterance are cut into K ranges.  Layer l's recurrence over
    range k (frames are routed in order, naive:162-170) needs only layer l-1's
    output up to frame t1 - 1 + rpad (the window, naive:150-151), so with the range
    bounds of layer l shifted down by l * rpad, range (l, k) depends on (l - 1, k)
    and (l, k - 1) only: the L layers run as a wavefront, one HIP stream per layer,
    L per-utterance recurrences in flight instead of one.  The backward walks the
    same ranges in reverse: (l, k) needs layer l+1's gx (the window adjoint) down to
    frame t0 - rpad, i.e. (l + 1, k), and the carry of (l, k + 1).
    layers: [(N, din, J, dout, mask_first)] per layer."""

    def __init__(self, B, T, layers, lpad, rpad, iters, n_chunks=0, pose_fp8=False, u_bf16=True,
                 store_couplings=True, store_u_bytes=None, last_group=None):
        """n_chunks: frame ranges per utterance (0: ~10 frames each); pose_fp8 / u_bf16: the
        opt-in e4m3 pose, and u kept in bf16 on its streamed layers; store_couplings:
        the forward keeps each frame's couplings for the backward (else recomputed where
        the layer's kernels can); store_u_bytes: budget for keeping every layer's u from
        the forward (None: 55 % of the device's memory; 0: recompute per range);
        last_group: workgroups per utterance for the last layer's recurrence
        (srf_sdr_range.group), one number for both directions or a (forward, backward)
        pair; None: the defaults of group()."""
        self.B, self.T, self.lpad, self.rpad, self.iters = B, T, lpad, rpad, iters
        self.pose_fp8 = bool(pose_fp8)
        self.store_couplings = bool(store_couplings)
        self.store_u_bytes = store_u_bytes
        self.layers = layers
        self.L = len(layers)
        self.win = lpad + rpad + 1
        if n_chunks <= 0:
            # ~10 frames per range (C3 step: 20-frame ranges 25.3 ms, 10-frame 23.95, 8-frame
            # 23.9, 5-frame 25.3: shorter ranges shorten the wavefront's fill and drain)
            n_chunks = max(1, min(32, -(-T // 10)))
        # ranges of S frames on one grid, layer l's shifted down by l * rpad; the grid
        # runs M >= K ranges so that no layer's shifted range is clipped into a long
        # one (C5: rpad = 20 frames per layer would otherwise leave the last layer one
        # 160-frame range at the end of the forward and the first layer one at the end
        # of the backward).  Ranges outside [0, T) are empty.  The backward uses the
        # same bounds: (l, k) needs (l + 1, k) for the window adjoint and (l, k + 1) for
        # the carry.
        S = -(-T // max(1, min(n_chunks, T)))
        K = -(-(T + rpad * (self.L - 1)) // S)
        self.K, self.S = K, S

        def bounds(shift):
            return [min(max(k * S + shift, 0), T) for k in range(K)] + [T]
        self.fwd = [bounds(-rpad * l) for l in range(self.L)]
        self.bwd = self.fwd
        self.nmax = max(max(b[k + 1] - b[k] for k in range(K)) for b in self.fwd)
        L_ = _lib.lib()
        self.rws = [L_.srf_route_sdr_recur_workspace(B, N * self.win, J, D, iters) for (N, din, J, D, mf) in layers]
        self.rzs = []   # (offset, bytes) of each workspace's part that starts zero (group counters)
        for (N, din, J, D, mf) in layers:
            off = ctypes.c_size_t(0)
            n = L_.srf_route_sdr_recur_zero_range(B, N * self.win, J, D, iters, ctypes.byref(off))
            self.rzs.append((off.value, n))
        # fp8 pose: layers on the streaming recurrence keep u in bf16 (half the bytes of
        # every read; 2^-9 against the e4m3 operands' 2^-4); u_bf16=False keeps fp32
        self.ubf = [self.pose_fp8 and bool(u_bf16)
                    and bool(L_.srf_route_sdr_couplings_required(N * self.win, J, D, iters))
                    for (N, din, J, D, mf) in layers]
        self.streamed = [bool(L_.srf_route_sdr_couplings_required(N * self.win, J, D, iters))
                         for (N, din, J, D, mf) in layers]
        # set by the caller when collectives overlap the backward (SequenceRouter with
        # grad buckets at world > 1): the last layer's backward is then not grouped
        self.collectives_overlap = False
        if last_group is None or isinstance(last_group, (tuple, list)):
            self.last_group = None if last_group is None else tuple(int(g) for g in last_group)
        else:
            self.last_group = (int(last_group), int(last_group))

    def group(self, l, dev, backward=False):
        """srf_sdr_range.group of layer l's recurrence launches.  Only the last layer's
        (stream B, one range per launch: the critical chain of the stack) are grouped:
        its B * G workgroups spin-wait on each other, so they must be resident next to
        stream A's batched inner-layer recurrence (B workgroups per inner layer, one CU
        each) -- the one grouped launch in flight at any time.  A streamed last layer
        (C5): as many as the CUs allow, both directions (955 -> 800 ms per step at
        G = 2).  Register kernels (C3; the grouped backward reads the stored couplings):
        the backward only, G = 2 -- its frame moves 2x the forward's bytes through one
        CU, so halving them pays for the three exchanges (r04n: 21.9 -> 21.2 ms), while
        the forward's exchanges cost more than they save (G = 2 / 4 slower)."""
        if l != self.L - 1 or not (self.streamed[l] or self.store_couplings):
            return 1
        if backward and self.collectives_overlap:
            # bucketed all-reduces run beside the backward: RCCL's kernels hold CUs the
            # group's members would have to share, so the backward is not grouped
            return 1
        if self.last_group is not None:
            return max(1, self.last_group[int(backward)])
        # the library keeps GROUP_RESERVE_CUS free (srf_group.h); the inner layers'
        # recurrences hold B CUs each on stream A
        cus = torch.cuda.get_device_properties(dev).multi_processor_count - GROUP_RESERVE_CUS
        if not self.streamed[l]:
            return 2 if backward and self.store_couplings and self.B * (self.L + 1) <= cus else 1
        return max(1, min(8, (cus - self.B * (self.L - 1)) // self.B))

    def recur_ws(self, l, dev):
        """Layer l's recurrence workspace with its group counters zeroed (srf_group.h;
        srf_route_sdr_recur_zero_range): one small fill, not a memset of the scratch."""
        ws = torch.empty(max(self.rws[l], 16), device=dev, dtype=torch.uint8)
        off, n = self.rzs[l]
        if n:
            ws[off:off + n].zero_()
        return ws

    def pose_mode(self, l):
        """srf_route_sdr_pose_n mode: 0 fp32, 1 fp8, 2 fp8 with bf16 u."""
        return 2 if self.ubf[l] else int(self.pose_fp8)

    def u_empty(self, l, frames, dev):
        """u buffer of `frames` frames per utterance (bf16 for ubf layers)."""
        return torch.empty(self.u_floats(l, frames), device=dev,
                           dtype=torch.bfloat16 if self.ubf[l] else torch.float32)

    def u_bytes(self, l, frames):
        return self.u_floats(l, frames) * (2 if self.ubf[l] else 4)

    def in_n(self, l):
        return self.layers[l][0] * self.win

    def events(self, which, n=None):
        """Events of the forward or backward wavefront ([L][K], or n of them), created
        once and kept with the plan: a captured step (hipGraph) must not see its
        events destroyed before the capture ends."""
        ev = getattr(self, '_ev_' + which, None)
        if ev is None:
            ev = ([[torch.cuda.Event() for _ in range(self.K)] for _ in range(self.L)] if n is None
                  else [torch.cuda.Event() for _ in range(n)])
            setattr(self, '_ev_' + which, ev)
        return ev

    def u_floats(self, l, frames):
        N, din, J, D, mf = self.layers[l]
        return self.B * frames * N * self.win * J * D


_stack_streams = {}


def _layer_streams(dev, n, role):
    """One stream per layer for the forward or the backward wavefront.  The two roles
    use disjoint streams: a captured step (hipGraph) that forks the same side streams
    in the forward (caller's thread) and again in the backward (torch's autograd device
    thread) crashes at capture end on this ROCm, while forking them twice from one
    thread, or disjoint streams per role, capture fine (scripts/dbg/capture_probe*.py)."""
    ss = _stack_streams.setdefault((dev, role), [])
    while len(ss) < n:
        ss.append(torch.cuda.Stream(device=dev))
    return ss[:n]


def _store_u(plan, dev):
    """Keep every layer's pose output u from the forward for the backward (instead of
    recomputing it per range) when it fits plan.store_u_bytes, by default 55 % of the
    device's memory: C5 keeps 135 GB of u on a 288 GB MI355X, C3 5.5 GB."""
    budget = plan.store_u_bytes
    if budget is None:
        budget = 0.55 * torch.cuda.get_device_properties(dev).total_memory
    return sum(plan.u_bytes(l, plan.T) for l in range(plan.L)) <= budget


def _sdr_r(**kw):
    r = _lib.SdrRange()
    for k, v in kw.items():
        setattr(r, k, v)
    return r


def _cn_call(fn, ranges, *args, what):
    """fn(ranges, n, *args) for up to CAPSNORM_MAX_ITEMS capsnorm ranges per launch."""
    for c in range(0, len(ranges), _lib.CAPSNORM_MAX_ITEMS):
        part = ranges[c:c + _lib.CAPSNORM_MAX_ITEMS]
        _lib.check(fn((_lib.CapsnormRange * len(part))(*part), len(part), *args), what)


# din-32 SDR layers: gx and gW in one launch that reads gu once (srf_route_sdr_gx_gw_n);
# False runs the two contractions' own launches (bench --sdr-separate-gxgw, for A/B)
SDR_FUSED_GXGW = True
# STACK_CAPTURE_ORDER: the stack's graph-captured launches keep each stream's next launch
# ahead (in issue order) of the other streams' launches that wait on it.  ROCm's graph
# executor splits the captured DAG into chains by depth-first search -- a node's first
# child in capture order continues its chain, every other child starts a new chain --
# and puts the chains on its few hardware queues in turn: a cross-stream child issued
# first made every last-layer range a new chain that shared a queue with the inner
# layers' every fourth range (C3 step 18.1 ms; eager 17.3).  scripts/dbg/graph_queues.py:
# the stack's stream patterns 1.14-1.23x their critical path in a graph, 1.00-1.01x in
# this order.
# the last layer's gx / gW of range k run on a third stream beside the recurrence of range
# k - 1 (the last layer's gu kept for every frame, so the streams are ordered one way
# only): off the backward's critical chain; False keeps them on the recurrence's stream
# (bench --sdr-last-gxw-inline, for A/B)
SDR_LAST_GXW_SIDE = True
# True (bench --sdr-gu-factors, opt-in): din = dout = 32 layers on the register recurrence
# with stored couplings (C3) have the recurrence backward write each frame's gu factors
# (gL^r, gs^r, Vc^r: 55 KB at the C3 last layer) instead of gu (320 KB), and the fused
# gx / gW pass form gu from them (srf_route_sdr_gx_gw_fact_n).  The recurrence gains
# (C3 16.0 -> 14.85 ms with gx / gW still reading gu, r06fa), but the factor pass reads
# gs^r / Vc^r once per input capsule from L2 and runs 482 us per inner diagonal against
# 131 (C3 25.5 ms, r06fc): off until a pass that reuses them exists
SDR_GU_FACTORS = False
# the inner layers' LN + dropout of one anti-diagonal in one launch (srf_capsnorm_*_range_n);
# False: one launch per layer (bench --sdr-capsnorm-per-layer, for A/B)
SDR_CAPSNORM_BATCHED = True


def _sdr_call(fn, ranges, *args, what):
    """fn(ranges, n, *args) for up to SDR_MAX_ITEMS ranges per launch."""
    for c in range(0, len(ranges), _lib.SDR_MAX_ITEMS):
        part = ranges[c:c + _lib.SDR_MAX_ITEMS]
        arr = (_lib.SdrRange * len(part))(*part)
        _lib.check(fn(arr, len(part), *args), what)


class SdrStack(torch.autograd.Function):
    """emb0 [B,T,N0,din0] -> v of the last layer [B,T,J,D]; in between, layer l's v
    goes through drop(LN_mid{l+1}(v)) (the CapsNorm of naive:187-191) into layer
    l+1.  params: W_l, b_l for every layer, then gamma_l, beta_l for l < L-1.

    Schedule (SdrStackPlan's wavefront): the ranges (l, k) of the inner layers
    l < L-1 on one anti-diagonal d = l + k are independent, so each diagonal is ONE
    batched launch per kernel (pose, recurrence, gx, gW over srf_sdr_range items, the
    layers in grid.y / grid.z) on one stream A, in diagonal order; the last layer
    (J = 32 for C3/C5, its own kernels and the critical chain of the backward) runs
    range by range on a second stream B, synchronised with A by one event per
    diagonal / range.  Two streams, so no range ever waits behind another stream's
    blocked packet in a shared in-order hardware queue."""

    @staticmethod
    def forward(ctx, emb0, plan, training, p_mid, seed, *params):
        L_ = _lib.lib()
        P, B, T, L = plan, plan.B, plan.T, plan.L
        dev = emb0.device
        if not torch.cuda.is_current_stream_capturing():
            fault_flag(dev)   # registered before the first grouped launch (never inside a capture)
        Ws, bs = params[0:2 * L:2], params[1:2 * L:2]
        gammas, betas = params[2 * L::2], params[2 * L + 1::2]
        _check_dev('emb0', emb0, (B, T, P.layers[0][0], P.layers[0][1]))
        need_bwd = P.need_bwd
        store = need_bwd and _store_u(P, dev)
        tr = int(bool(training))
        embs, vs, stats, us, rws, css = [emb0], [], [], [], [], []
        for l, (N, din, J, D, mf) in enumerate(P.layers):
            vs.append(torch.empty((B, T, J, D), device=dev, dtype=torch.float32))
            # each frame's couplings and s^r, for a backward without the recompute
            # (store_couplings=False: recompute them, where the shape's kernels can)
            ncs = L_.srf_route_sdr_coupling_floats(P.in_n(l), J, D, P.iters) \
                if need_bwd and (P.store_couplings
                                 or L_.srf_route_sdr_couplings_required(P.in_n(l), J, D, P.iters)) else 0
            css.append(torch.empty(B * T * ncs, device=dev, dtype=torch.float32) if ncs else None)
            if l < L - 1:
                embs.append(torch.empty((B, T, J, D), device=dev, dtype=torch.float32))
                stats.append(torch.empty((B * T, 4), device=dev, dtype=torch.float32))
            us.append(P.u_empty(l, T if store else P.nmax, dev))
            rws.append(P.recur_ws(l, dev))
        main = torch.cuda.current_stream(dev)
        sa, sb, sc = _layer_streams(dev, 3, 'fwd')
        ev_a, ev_p = P.events('fwd_a', P.K + L), P.events('fwd_p', P.K)
        for s_ in (sa, sb, sc):
            s_.wait_stream(main)
        pa, pb, pc = ctypes_void(sa.cuda_stream), ctypes_void(sb.cuda_stream), ctypes_void(sc.cuda_stream)
        # the last layer's pose runs ahead of its recurrence on stream C when u is kept
        # whole (a range buffer would be overwritten by the next pose)
        pose_ahead = store or not need_bwd and P.u_bytes(L - 1, T) <= 2 ** 30
        if pose_ahead and not store:
            us[L - 1] = P.u_empty(L - 1, T, dev)

        def item(l, k):
            t0, t1 = P.fwd[l][k], P.fwd[l][k + 1]
            v0, vn = (0, T) if (store or (pose_ahead and l == L - 1)) else (t0, P.nmax)
            return _sdr_r(t0=t0, t1=t1, emb=_ptr(embs[l]), W=_ptr(Ws[l]), bias=_ptr(bs[l]), u=_ptr(us[l]), v0=v0,
                          vn=vn, v=_ptr(vs[l]), couplings=_ptr(css[l]) if css[l] is not None else None,
                          workspace=_ptr(rws[l]), workspace_bytes=rws[l].numel(), u_bf16=int(P.ubf[l]),
                          group=P.group(l, dev))

        def pose(sp, ls, ks):
            N, din, J, D, mf = P.layers[ls[0]]
            rr = [item(l, k) for l, k in zip(ls, ks)]
            _sdr_call(L_.srf_route_sdr_pose_n, rr, B, T, N, din, P.lpad, P.rpad, J, D, P.pose_mode(ls[0]), sp,
                      what='sdr_pose_n')

        timing = getattr(P, 'timing', None)   # bench.py: [(start, end, frames)] of the last layer

        def run(sp, ls, ks, with_pose=True):
            """pose + recurrence (+ LN/dropout for inner layers) of ranges (ls[i], ks[i])
            of same-shaped layers, batched."""
            N, din, J, D, mf = P.layers[ls[0]]
            rr = [item(l, k) for l, k in zip(ls, ks)]
            if with_pose:
                pose(sp, ls, ks)
            tm = timing is not None and ls[0] == L - 1
            if tm:
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ev0.record(sb)
            _sdr_call(L_.srf_route_sdr_recur_fwd_n, rr, B, T, P.in_n(ls[0]), J, D, P.iters, mf, sp,
                      what='sdr_recur_fwd_n')
            if tm:
                ev1.record(sb)
                timing.append((ev0, ev1, B * sum(r.t1 - r.t0 for r in rr)))
            # LN + dropout of the inner layers' ranges, one launch
            cn = [_lib.CapsnormRange(t0=r.t0, t1=r.t1, layer=l, x=_ptr(vs[l]), gamma=_ptr(gammas[l]),
                                     beta=_ptr(betas[l]), y=_ptr(embs[l + 1]), stat=_ptr(stats[l]))
                  for l, r in zip(ls, rr) if l < L - 1]
            for c in ([cn] if SDR_CAPSNORM_BATCHED else [[x] for x in cn]):
                if c:
                    _cn_call(L_.srf_capsnorm_fwd_range_n, c, B, T, J * D, tr, float(p_mid), int(seed), sp,
                             what='capsnorm_fwd_range_n')

        def last(k):
            """the last layer's recurrence of range k on stream B (its pose too unless ahead)"""
            if pose_ahead:
                sb.wait_event(ev_p[k])
            elif L > 1:
                sb.wait_event(ev_a[k + L - 2])
            run(pb, [L - 1], [k], with_pose=not pose_ahead)

        # capture order (STACK_CAPTURE_ORDER): the recurrence of the last layer's range k
        # is issued one diagonal late, after the pose of range k + 1 (stream C) and inner
        # diagonal d + 1 (stream A) that follow the launches it waits on
        pending = None
        for d in range(P.K + L - 1):
            # inner layers: diagonal d on stream A, grouped by layer shape
            groups = {}
            for l in range(L - 1):
                k = d - l
                if 0 <= k < P.K and P.fwd[l][k] < P.fwd[l][k + 1]:
                    groups.setdefault(P.layers[l], []).append((l, k))
            for g in groups.values():
                run(pa, [l for l, _ in g], [k for _, k in g])
            ev_a[d].record(sa)
            # last layer: range k = d - (L-1) needs (L-2, k), done on diagonal d - 1
            k = d - (L - 1)
            live = 0 <= k < P.K and P.fwd[L - 1][k] < P.fwd[L - 1][k + 1]
            if live and pose_ahead:
                if L > 1:
                    sc.wait_event(ev_a[d - 1])
                pose(pc, [L - 1], [k])
                ev_p[k].record(sc)
            if pending is not None:
                last(pending)
            pending = k if live else None
        if pending is not None:
            last(pending)
        for s_ in (sa, sb, sc):
            main.wait_stream(s_)
        ctx.plan, ctx.meta = P, (tr, float(p_mid), int(seed), store)
        ctx.params = params
        ctx.css = css
        ctx.save_for_backward(*embs, *vs, *stats, *(us if store else []), *params)
        return vs[-1]

    @staticmethod
    def backward(ctx, g_v_last):
        L_ = _lib.lib()
        P = ctx.plan
        B, T, L = P.B, P.T, P.L
        tr, p_mid, seed, store = ctx.meta
        saved = list(ctx.saved_tensors)
        embs, saved = saved[:L], saved[L:]
        vs, saved = saved[:L], saved[L:]
        stats, saved = saved[:L - 1], saved[L - 1:]
        if store:
            us, saved = saved[:L], saved[L:]
        params = saved
        Ws, bs = params[0:2 * L:2], params[1:2 * L:2]
        gammas, betas = params[2 * L::2], params[2 * L + 1::2]
        dev = g_v_last.device
        g_v_last = g_v_last.contiguous()
        targets = [_grad_target(p) for p in ctx.params]
        gWs, gbs = [targets[2 * l][0] for l in range(L)], [targets[2 * l + 1][0] for l in range(L)]
        ggs = [targets[2 * L + 2 * l][0] for l in range(L - 1)]
        gbts = [targets[2 * L + 2 * l + 1][0] for l in range(L - 1)]
        g_embs = [torch.zeros_like(e) for e in embs]           # gx scatter targets
        g_vs, gparts, carries, WTs, gus, urs, rws, pws = [], [], [], [], [], [], [], []
        # per layer: floats of one frame's gu factors (0: the layer writes and reads gu)
        facts = [_gu_fact_floats(P, l, ctx.css[l] is not None) for l in range(L)]
        for l, (N, din, J, D, mf) in enumerate(P.layers):
            n = J * D
            g_vs.append(torch.empty((B, T, J, D), device=dev) if l < L - 1 else g_v_last)
            gparts.append(torch.empty((B * T, 2 * n), device=dev) if l < L - 1 else None)
            carries.append(torch.zeros((B, n), device=dev))
            WTs.append(torch.empty(Ws[l].numel(), device=dev))
            gus.append(torch.empty(B * P.nmax * facts[l] if facts[l] else P.u_floats(l, P.nmax), device=dev))
            urs.append(us[l] if store else P.u_empty(l, P.nmax, dev))
            rws.append(P.recur_ws(l, dev))
            pws.append(torch.empty(max(L_.srf_capsnorm_params_workspace(B * T, n), 16), device=dev,
                                   dtype=torch.uint8) if l < L - 1 else None)
        main = torch.cuda.current_stream(dev)
        side = SDR_LAST_GXW_SIDE
        sa, sb, sc = _layer_streams(dev, 3, 'bwd')
        ev_b = P.events('bwd_b', P.K)   # the last layer's range k has its gu and gx
        ev_r = P.events('bwd_r', P.K)   # the last layer's range k has its gu (side: gx / gW may start)
        # side: the last layer's gu covers every frame (C3: 1.8 GB), so the recurrence of
        # range k - 1 (stream B) never writes what gx / gW of range k (stream C) read: C
        # waits for B, never B for C (torch's capture crashed on streams ordered both ways)
        if side:
            gus[L - 1] = torch.empty(B * T * facts[L - 1] if facts[L - 1] else P.u_floats(L - 1, T), device=dev)
        for s_ in (sa, sb, sc):
            s_.wait_stream(main)
        pa, pb, pc = ctypes_void(sa.cuda_stream), ctypes_void(sb.cuda_stream), ctypes_void(sc.cuda_stream)
        for l, (N, din, J, D, mf) in enumerate(P.layers):
            _lib.check(L_.srf_route_sdr_transpose_w(_ptr(Ws[l]), P.in_n(l), J, D, din, _ptr(WTs[l]),
                                                    pb if l == L - 1 else pa), 'sdr_transpose_w')

        def item(l, k):
            t0, t1 = P.bwd[l][k], P.bwd[l][k + 1]
            v0, vn = (0, T) if store else (t0, P.nmax)
            cs = ctx.css[l]
            return _sdr_r(t0=t0, t1=t1, emb=_ptr(embs[l]), W=_ptr(Ws[l]), bias=_ptr(bs[l]), WT=_ptr(WTs[l]),
                          u=_ptr(urs[l]), v0=v0, vn=vn, v=_ptr(vs[l]),
                          couplings=_ptr(cs) if cs is not None else None, workspace=_ptr(rws[l]),
                          workspace_bytes=rws[l].numel(), g_v=_ptr(g_vs[l]), carry=_ptr(carries[l]),
                          gu=_ptr(gus[l]), g0=0 if side and l == L - 1 else t0,
                          gn=T if side and l == L - 1 else P.nmax, g_emb=_ptr(g_embs[l]), g_W=_ptr(gWs[l]),
                          g_bias=_ptr(gbs[l]), accumulate=int(k != P.K - 1), u_bf16=int(P.ubf[l]),
                          group=P.group(l, dev, backward=True), gu_factored=int(facts[l] > 0))

        def run(sp, ls, ks, ev=None, gw=True, part='all'):
            """backward of ranges (ls[i], ks[i]) of same-shaped layers, batched: LN
            backward of the range's rows (inner layers), pose (when u was not kept),
            recurrence, gx (window adjoint into the layer below), then (gw) gW / gbias;
            part 'rec' stops after the recurrence, 'grad' is the rest (another stream's
            launches); ev is recorded behind the part's last launch."""
            N, din, J, D, mf = P.layers[ls[0]]
            rr = [item(l, k) for l, k in zip(ls, ks)]
            live = [r for r in rr if r.t1 > r.t0]
            fused = gw and din == 32 and SDR_FUSED_GXGW   # gx + gW in one pass over gu
            if part != 'grad':
                cn = [_lib.CapsnormRange(t0=r.t0, t1=r.t1, layer=l, x=_ptr(vs[l]), gamma=_ptr(gammas[l]),
                                         beta=_ptr(betas[l]), stat=_ptr(stats[l]), g_y=_ptr(g_embs[l + 1]),
                                         g_x=_ptr(g_vs[l]), gpart=_ptr(gparts[l]))
                      for l, r in zip(ls, rr) if l < L - 1 and r.t1 > r.t0]
                for c in ([cn] if SDR_CAPSNORM_BATCHED else [[x] for x in cn]):
                    if c:   # LN + dropout backward of the inner layers' ranges, one launch
                        _cn_call(L_.srf_capsnorm_bwd_range_n, c, B, T, J * D, tr, float(p_mid), int(seed), sp,
                                 what='capsnorm_bwd_range_n')
                if live:
                    if not store:
                        _sdr_call(L_.srf_route_sdr_pose_n, live, B, T, N, din, P.lpad, P.rpad, J, D,
                                  P.pose_mode(ls[0]), sp, what='sdr_pose_n')
                    _sdr_call(L_.srf_route_sdr_recur_bwd_n, live, B, T, P.in_n(ls[0]), J, D, P.iters, mf, sp,
                              what='sdr_recur_bwd_n')
                if part == 'rec':
                    if ev is not None:
                        ev.record(streams[id(sp)])
                    return
            if live and not fused:
                _sdr_call(L_.srf_route_sdr_gx_n, live, B, T, N, din, P.lpad, P.rpad, J, D, sp, what='sdr_gx_n')
            if fused and facts[ls[0]]:
                _sdr_call(L_.srf_route_sdr_gx_gw_fact_n, rr, B, T, N, din, P.lpad, P.rpad, J, D, P.iters, sp,
                          what='sdr_gx_gw_fact_n')
            elif fused:
                _sdr_call(L_.srf_route_sdr_gx_gw_n, rr, B, T, N, din, P.lpad, P.rpad, J, D, sp, what='sdr_gx_gw_n')
            if ev is not None:
                ev.record(streams[id(sp)])
            if gw and not fused:
                gw_ranges(sp, ls, ks)
            for l, k in zip(ls, ks):
                if k == 0 and l < L - 1:
                    _lib.check(L_.srf_capsnorm_bwd_params(_ptr(gparts[l]), B * T, J * D, _ptr(ggs[l]),
                                                          _ptr(gbts[l]), _ptr(pws[l]), pws[l].numel(), sp),
                               'capsnorm_bwd_params')

        def gw_ranges(sp, ls, ks):
            """gW / gbias of the ranges (an empty first range still zeroes the layer's sums)."""
            N, din, J, D, mf = P.layers[ls[0]]
            rr = [item(l, k) for l, k in zip(ls, ks)]
            _sdr_call(L_.srf_route_sdr_gw_n, rr, B, T, N, din, P.lpad, P.rpad, J, D, sp, what='sdr_gw_n')

        streams = {id(pa): sa, id(pb): sb, id(pc): sc}   # ctypes pointers do not hash
        # diagonal e of the inner layers holds (l, k) with (K-1-k) + (L-2-l) = e: (l, k)
        # needs (l+1, k) (diagonal e-1, or the last layer's range k on stream B) and
        # (l, k+1) (diagonal e-1).  Capture order (STACK_CAPTURE_ORDER): iteration e issues
        # the last layer's recurrence of range K-1-e, its gx / gW of the range before
        # (stream C) and inner diagonal e - 2, so every launch's same-stream successor is
        # issued before the other streams' launches that wait on it
        for e in range(P.K + L + 1):
            k = P.K - 1 - e
            if k >= 0:   # last layer, range k, on stream B (gx / gW on stream C when side)
                if side:
                    run(pb, [L - 1], [k], ev=ev_r[k], part='rec')
                else:
                    run(pb, [L - 1], [k], ev=ev_b[k])
            kg = k + 1
            if side and 0 <= kg < P.K:
                sc.wait_event(ev_r[kg])
                run(pc, [L - 1], [kg], ev=ev_b[kg], part='grad')
            ed = e - 2
            groups = {}
            for l in range(L - 1):
                kk = P.K - 1 - (ed - (L - 2 - l))
                if ed >= 0 and 0 <= kk < P.K:
                    groups.setdefault(P.layers[l], []).append((l, kk))
            if not groups:
                continue
            kl = P.K - 1 - ed   # (L-2, kl) is in this diagonal: it needs the last layer's range kl
            if L > 1 and 0 <= kl < P.K:
                sa.wait_event(ev_b[kl])
            for g in groups.values():
                run(pa, [l for l, _ in g], [kk for _, kk in g])
        for s_ in (sa, sb, sc):
            main.wait_stream(s_)
        ctx.css = None
        return (g_embs[0], None, None, None, None, *_returned(targets))


def _gu_fact_floats(P, l, has_couplings):
    """Floats of one frame's gu factors for layer l's backward, or 0 where the layer
    writes gu: SDR_GU_FACTORS, the register recurrence with the forward's couplings, the
    fused gx / gW pass and its shape (din = dout = 32, J a multiple of 16, iters <= 3)."""
    N, din, J, D, mf = P.layers[l]
    if not (SDR_GU_FACTORS and SDR_FUSED_GXGW and has_couplings and not P.streamed[l]):
        return 0
    if din != 32 or D != 32 or J % 16 or P.iters > 3:
        return 0
    return int(_lib.lib().srf_route_sdr_fact_floats(P.in_n(l), J, D, P.iters))


def sdr_stack(emb0, plan, training, p_mid, seed, params):
    """SdrStack.apply; the forward keeps the pose outputs for the backward only when
    one will run (grad mode on and something requires a gradient)."""
    plan.need_bwd = torch.is_grad_enabled() and (emb0.requires_grad or any(p.requires_grad for p in params))
    return SdrStack.apply(emb0, plan, training, p_mid, seed, *params)
