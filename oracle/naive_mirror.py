"""torch-CPU op-for-op mirror of ``tfsr/model/sequence_router_naive.py`` -- TEST INFRASTRUCTURE ONLY.

Two uses, both as the checker / baseline, never as product code:
  * gradient oracle: run in float64 under autograd, cross-checked against the numpy
    ``srf_oracle`` forward and finite differences;
  * ``bench.py``'s ``cpu_baseline`` leg ("port"): the reference's TF graph restated
    op for op on torch CPU ops -- ``tf.tile``-materialised ``u_hat`` (naive:155-157),
    while-style routing loops (naive:162-185), ``ctc_loss`` (trainer_sr.py:64-66),
    Adam with ``CustomSchedule`` (train_helper.py:32-70).

Parity: unpinned against TensorFlow (see ``oracle/__init__.py``).
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from . import srf_oracle as so


def _same_pad_2d(x_nchw, k, stride):
    _, _, H, W = x_nchw.shape
    _, pt, pb = so.same_pad(H, k, stride)
    _, pl, pr = so.same_pad(W, k, stride)
    return F.pad(x_nchw, (pl, pr, pt, pb))


def conv2d_same(x, kern, bias, stride):
    """Keras Conv2D 'same' on NHWC with kernel [kh,kw,Cin,Cout] (sequence_router.py:48-53)."""
    xn = _same_pad_2d(x.permute(0, 3, 1, 2), kern.shape[0], stride)
    y = F.conv2d(xn, kern.permute(3, 2, 0, 1), bias, stride=stride)
    return y.permute(0, 2, 3, 1)


def feat_mask(x, inp_len, div):
    """model_helper.py:125-140."""
    lens = torch.ceil(inp_len.to(torch.int32).double() / div)
    T = x.shape[1]
    m = (torch.arange(T, dtype=torch.float64)[None, :] < lens[:, None]).to(x.dtype)
    return x * m.reshape(m.shape + (1,) * (x.dim() - 2))


def batch_norm_train(x, gamma, beta):
    mu = x.mean(dim=(0, 1, 2))
    var = x.var(dim=(0, 1, 2), unbiased=False)
    return (x - mu) * torch.rsqrt(var + so.BN_EPS) * gamma + beta, mu, var


def layer_norm(x, gamma, beta):
    mu = x.mean(-1, keepdim=True)
    var = x.var(-1, unbiased=False, keepdim=True)
    return (x - mu) * torch.rsqrt(var + so.LN_EPS) * gamma + beta


def squash(s, dim=-1):
    """naive:247-253."""
    n2 = torch.sum(torch.square(s), dim=dim, keepdim=True)
    return n2 / (1.0 + n2) * (s / torch.sqrt(n2 + so.SQUASH_EPS))


def length(s, dim=-1, eps=so.LENGTH_EPS):
    """naive:255-258 (einsum:238 uses eps 1e-9)."""
    return torch.sqrt(torch.sum(torch.square(s), dim=dim) + eps)


def pose_tiled(emb_win, W, bias):
    """naive:154-159 with the reference's materialising tiles."""
    B, T, I, E = emb_win.shape
    J = W.shape[1]
    caps1 = emb_win.unsqueeze(3).unsqueeze(-1)                  # [B,T,I,1,E,1]
    caps1_t = caps1.repeat(1, 1, 1, J, 1, 1)                    # tf.tile :155
    W_t = W.unsqueeze(0).unsqueeze(0).repeat(B, T, 1, 1, 1, 1)  # tf.tile :157
    u = torch.matmul(W_t, caps1_t)                              # [B,T,I,J,D,1]
    return u.squeeze(-1) + bias                                 # :158-159


def dynamic_routing(u, iters, mask_first):
    """naive:171-185, _loop_body :199-206 (while_loop restated as a python loop)."""
    B, T, I, J, D = u.shape
    b = torch.zeros(B, T, I, J, dtype=u.dtype)
    m = torch.zeros_like(b)
    if mask_first:
        m[..., 0] = so.MASK_LOGIT
    v = None
    for _ in range(iters):
        b = b + m
        c = torch.softmax(b, dim=3)
        s = torch.sum(c.unsqueeze(-1) * u, dim=2)
        v = squash(s, -1)
        b = b + torch.sum(u * v.unsqueeze(2), dim=-1)
    return v


def sequential_routing(u, iters, mask_first):
    """naive:162-170, body_context :231-245, pad_body_context :212-229."""
    B, T, I, J, D = u.shape
    v = torch.zeros(B, J, D, dtype=u.dtype)
    m = torch.zeros(B, I, J, dtype=u.dtype)
    if mask_first:
        m[..., 0] = so.MASK_LOGIT
    outs = []
    for t in range(T):
        ut = u[:, t]
        b = torch.zeros(B, I, J, dtype=u.dtype)
        for _ in range(iters):
            b = b + torch.sum(ut * v.unsqueeze(1), dim=-1)
            if mask_first:
                b = b + m
            c = torch.softmax(b, dim=2)
            s = torch.sum(c.unsqueeze(-1) * ut, dim=1)
            v = squash(s, -1)
        outs.append(v)
    return torch.stack(outs, 1)


def dr_layer_chunked(emb, W, bias, lpad, rpad, iters, mask_first, g_v, frames_per_chunk=128):
    """One DR layer -- window (naive:150-151), pose (:154-159), routing (:171-185,
    :199-206) -- and its backward for the upstream gradient g_v, in float64, over
    frame chunks so that a full-size layer (C4: 5,600 frames x 80 x 32 x 32 u) fits in
    memory.  DR is independent per frame, so chunking changes nothing but the
    summation order of g_W / g_bias.  emb [B,T,N,D] -> (v, g_emb, g_W, g_bias)."""
    emb = torch.as_tensor(emb, dtype=torch.float64)
    W = torch.as_tensor(W, dtype=torch.float64)
    bias = torch.as_tensor(bias, dtype=torch.float64)
    g_v = torch.as_tensor(g_v, dtype=torch.float64)
    B, T, N, D = emb.shape
    win = lpad + rpad + 1
    J, Dv = W.shape[1], W.shape[2]
    ep = F.pad(emb, (0, 0, 0, 0, lpad, rpad))
    xw_all = torch.cat([ep[:, w:w + T] for w in range(win)], dim=2).reshape(B * T, N * win, D)
    gv_all = g_v.reshape(B * T, J, Dv)
    v_all = torch.empty(B * T, J, Dv, dtype=torch.float64)
    gx_all = torch.empty_like(xw_all)
    gW = torch.zeros_like(W)
    gb = torch.zeros_like(bias)
    for f0 in range(0, B * T, frames_per_chunk):
        f1 = min(B * T, f0 + frames_per_chunk)
        xw = xw_all[f0:f1].clone().requires_grad_(True)
        Wc = W.clone().requires_grad_(True)
        bc = bias.clone().requires_grad_(True)
        u = torch.einsum('ijde,fie->fijd', Wc, xw) + bc
        v = dynamic_routing(u[None], iters, mask_first)[0]
        v.backward(gv_all[f0:f1])
        v_all[f0:f1] = v.detach()
        gx_all[f0:f1] = xw.grad
        gW += Wc.grad
        gb += bc.grad
    # window adjoint: capsule i = w*N + n of frame t reads emb[t - lpad + w, n]
    gx = gx_all.reshape(B, T, win, N, D)
    gep = torch.zeros_like(ep)
    for w in range(win):
        gep[:, w:w + T] += gx[:, :, w]
    return v_all.reshape(B, T, J, Dv), gep[:, lpad:lpad + T], gW, gb


def _pose_fp8_tbjid(xw, W, bias, bf16_u):
    """``srf_oracle.pose_fp8`` (same quantisation: per-vector 2^e scales, e4m3 operands,
    exact products summed in float64, scaled back, float32 bias, float32 or bf16 u) with
    the contraction on torch: xw [T,B,I,D] -> u [T,B,J,I,Dv] (float64)."""
    T, B, I, D = xw.shape
    J, Dv = W.shape[1], W.shape[2]
    x32 = xw.numpy().astype(np.float32).astype(np.float64)
    W32 = W.numpy().astype(np.float32).astype(np.float64)
    ex = so.e4m3_scale_exp(np.abs(x32).max(-1))                  # [T,B,I]
    ew = so.e4m3_scale_exp(np.abs(W32).max(-1))                  # [I,J,Dv]
    xq = torch.as_tensor(so.e4m3_round(x32 * np.exp2(ex)[..., None]))
    wq = torch.as_tensor(so.e4m3_round(W32 * np.exp2(ew)[..., None]))
    u = torch.bmm(wq.reshape(I, J * Dv, D), xq.permute(2, 3, 0, 1).reshape(I, D, T * B))
    u = u.reshape(I, J, Dv, T, B).permute(3, 4, 1, 0, 2)         # [T,B,J,I,Dv]
    u = u * torch.as_tensor(np.exp2(-ex.astype(np.float64))).permute(0, 1, 2)[:, :, None, :, None]
    u = u * torch.as_tensor(np.exp2(-ew.astype(np.float64))).permute(1, 0, 2)[None, None]
    u = (u + torch.as_tensor(bias.numpy().astype(np.float32).astype(np.float64)).permute(1, 0, 2)).numpy()
    return torch.as_tensor(so.bf16_round(u) if bf16_u else u.astype(np.float32).astype(np.float64))


def sdr_stack_frames(emb, Ws, bs, gammas, betas, lpad, rpad, iters, g_v, dtype=torch.float64, fp8_pose=None,
                     mask_last=True):
    """An SDR stack -- per layer window (naive:150-151), pose (:154-159), the frame
    recurrence (:162-170 with body_context :231-245, the last layer masked by
    pad_body_context :212-229) and, between layers, LN_mid (:187-191, dropout off) --
    and its backward for the upstream gradient g_v of the last layer's v, frame by
    frame, so that a bench-size stack (C3: 28 utterances x 200 frames x 80 x 32 x 32
    u per layer) runs under autograd without materialising u or its gradient: each
    frame's pose is formed from its own window, every intermediate is one frame.

    emb [B,T,N,D]; Ws[l] [in_n,J,Dv,D]; gammas / betas for the L-1 inner LNs.
    fp8_pose: None, or per-layer bf16-u flags -- the pose then takes the values of
    ``srf_oracle.pose_fp8`` (the build's opt-in e4m3 pose) with the exact pose's
    gradient, like ``NaiveMirror(fp8_pose=...)``.  mask_last: the last layer is the
    model's output layer (its capsule 0 masked); False for a stack cut out of a model.
    Returns (v_last [B,T,J,Dv], g_emb, [g_W], [g_bias], [g_gamma], [g_beta])."""
    def leaf(a):
        return torch.as_tensor(a).to(dtype).clone().requires_grad_(True)
    e0 = leaf(emb)
    Wl, bl = [leaf(w) for w in Ws], [leaf(b) for b in bs]
    gl, btl = [leaf(g) for g in gammas], [leaf(b) for b in betas]
    B, T = e0.shape[:2]
    L = len(Wl)
    x = [e0[:, t] for t in range(T)]            # layer input, one [B,N,D] per frame
    for l in range(L):
        W, bias = Wl[l], bl[l]
        I, J, Dv, D = W.shape
        N = x[0].shape[1]
        # the layer's pose for all frames in one product, held as [T, B, J, I, Dv] and
        # unbound into frames: its backward is one stack of the frames' gradients and
        # one product for g_W (no per-frame copies of W's gradient); per frame the
        # logits and s are batched matmuls that keep a reference to u_t, with no
        # u-sized temporaries per iteration
        zero = torch.zeros(B, N, D, dtype=dtype)
        xp = torch.stack([zero] * lpad + x + [zero] * rpad, 0)                       # [T+w-1, B, N, D]
        xw = torch.cat([xp[w:w + T] for w in range(lpad + rpad + 1)], 2)            # [T, B, I, D]
        u = torch.bmm(W.reshape(I, J * Dv, D), xw.permute(2, 3, 0, 1).reshape(I, D, T * B))
        u = u.reshape(I, J, Dv, T, B).permute(3, 4, 1, 0, 2).contiguous() + bias.permute(1, 0, 2)
        if fp8_pose is not None:
            u = u + (_pose_fp8_tbjid(xw.detach(), W.detach(), bias.detach(), bool(fp8_pose[l])).to(dtype)
                     - u).detach()
        m = torch.zeros(J, I, dtype=dtype)
        masked = mask_last and l == L - 1
        if masked:
            m[0] = so.MASK_LOGIT
        v = torch.zeros(B, J, Dv, dtype=dtype)
        outs = []
        for ut in u.unbind(0):
            b = torch.zeros(B, J, I, dtype=dtype)
            for _ in range(iters):
                b = b + torch.matmul(ut, v.unsqueeze(-1)).squeeze(-1)      # <u_ij, v_j>
                if masked:
                    b = b + m
                c = torch.softmax(b, dim=1)                                 # over j
                v = squash(torch.matmul(c.unsqueeze(2), ut).squeeze(2), -1)
            outs.append(v)
        del u
        if l < L - 1:
            x = [layer_norm(o.reshape(B, J * Dv), gl[l], btl[l]).reshape(B, J, Dv) for o in outs]
        else:
            vl = torch.stack(outs, 1)
    vl.backward(torch.as_tensor(g_v, dtype=dtype))
    return (vl.detach(), e0.grad, [w.grad for w in Wl], [b.grad for b in bl], [g.grad for g in gl],
            [b.grad for b in btl])


def sdr_layer_teacher_forced(emb, W, bias, v_run, lpad, rpad, iters, masked, fp8_bf16=None, frames_per_chunk=16):
    """One SDR layer's frames, each routed from the run's own previous output:
    frame t of the recurrence (naive:162-170, :231-245 / :212-229) in float64 with
    v_{t-1} taken from ``v_run`` (the implementation under test) instead of from this
    computation.  Every frame becomes an independent one-step check, so the bound
    does not have to cover the recurrence's amplification of rounding over time
    (at the reference init two fp32 runs of one C3 layer drift apart to ~0.3 by frame
    200).  fp8_bf16: None (exact fp32 pose) or the bf16-u flag of the opt-in fp8 pose
    (``_pose_fp8_tbjid``).  emb [B,T,N,D], v_run [B,T,J,Dv] -> v [B,T,J,Dv] float64."""
    emb = torch.as_tensor(emb, dtype=torch.float64)
    W = torch.as_tensor(W, dtype=torch.float64)
    bias = torch.as_tensor(bias, dtype=torch.float64)
    v_run = torch.as_tensor(v_run, dtype=torch.float64)
    B, T, N, D = emb.shape
    I, J, Dv, _ = W.shape
    ep = F.pad(emb, (0, 0, 0, 0, lpad, rpad)).transpose(0, 1)                  # [T+w-1, B, N, D]
    m = torch.zeros(J, I, dtype=torch.float64)
    if masked:
        m[0] = so.MASK_LOGIT
    out = torch.empty(B, T, J, Dv, dtype=torch.float64)
    for t0 in range(0, T, frames_per_chunk):
        t1 = min(T, t0 + frames_per_chunk)
        xw = torch.cat([ep[t0 + w:t1 + w] for w in range(lpad + rpad + 1)], 2)   # [n, B, I, D]
        n = t1 - t0
        if fp8_bf16 is None:
            u = torch.bmm(W.reshape(I, J * Dv, D), xw.permute(2, 3, 0, 1).reshape(I, D, n * B))
            u = u.reshape(I, J, Dv, n, B).permute(3, 4, 1, 0, 2) + bias.permute(1, 0, 2)
        else:
            u = _pose_fp8_tbjid(xw, W, bias, bool(fp8_bf16))                  # [n, B, J, I, Dv]
        v = torch.zeros(n, B, J, Dv, dtype=torch.float64)
        v[max(0, 1 - t0):] = v_run[:, max(t0 - 1, 0):t1 - 1].transpose(0, 1)
        b = torch.zeros(n, B, J, I, dtype=torch.float64)
        for _ in range(iters):
            b = b + torch.matmul(u, v.unsqueeze(-1)).squeeze(-1)
            if masked:
                b = b + m
            c = torch.softmax(b, dim=2)
            v = squash(torch.matmul(c.unsqueeze(3), u).squeeze(3), -1)
        out[:, t0:t1] = v.transpose(0, 1)
    return out


def sdr_layer_backward_teacher_forced(emb, W, bias, v_run, g_bar, lpad, rpad, iters, masked, frames_per_chunk=8):
    """The adjoint of each frame of one SDR layer, teacher-forced like
    ``sdr_layer_teacher_forced``: frame t's routing (naive:162-170 with :231-245 /
    :212-229) as a float64 function of its own pose u_t and of v_{t-1} taken from
    ``v_run``, differentiated (TF's tape.gradient of the frame, trainer_sr.py:70) for
    the cotangent ``g_bar[:, t]`` = dL/dv_t as the implementation under test holds it
    (the loss gradient of frame t plus the carry from frame t + 1).  Every frame is an
    independent check, so the bound need not cover the recurrence's amplification of
    rounding along the frames.  Returns (g_u [B,T,I,J,Dv], g_vprev [B,T,J,Dv]) float64:
    the gradient of the frame's pose and the carry into frame t - 1."""
    emb = torch.as_tensor(emb, dtype=torch.float64)
    W = torch.as_tensor(W, dtype=torch.float64)
    bias = torch.as_tensor(bias, dtype=torch.float64)
    v_run = torch.as_tensor(v_run, dtype=torch.float64)
    g_bar = torch.as_tensor(g_bar, dtype=torch.float64)
    B, T, N, D = emb.shape
    I, J, Dv, _ = W.shape
    ep = F.pad(emb, (0, 0, 0, 0, lpad, rpad)).transpose(0, 1)                  # [T+w-1, B, N, D]
    m = torch.zeros(J, I, dtype=torch.float64)
    if masked:
        m[0] = so.MASK_LOGIT
    g_u = torch.empty(B, T, I, J, Dv, dtype=torch.float64)
    g_vp = torch.empty(B, T, J, Dv, dtype=torch.float64)
    for t0 in range(0, T, frames_per_chunk):
        t1 = min(T, t0 + frames_per_chunk)
        n = t1 - t0
        xw = torch.cat([ep[t0 + w:t1 + w] for w in range(lpad + rpad + 1)], 2)   # [n, B, I, D]
        u = torch.bmm(W.reshape(I, J * Dv, D), xw.permute(2, 3, 0, 1).reshape(I, D, n * B))
        u = (u.reshape(I, J, Dv, n, B).permute(3, 4, 1, 0, 2) + bias.permute(1, 0, 2)).requires_grad_(True)
        vp = torch.zeros(n, B, J, Dv, dtype=torch.float64)
        vp[max(0, 1 - t0):] = v_run[:, max(t0 - 1, 0):t1 - 1].transpose(0, 1)
        vp.requires_grad_(True)
        v = vp
        b = torch.zeros(n, B, J, I, dtype=torch.float64)
        for _ in range(iters):
            b = b + torch.matmul(u, v.unsqueeze(-1)).squeeze(-1)
            if masked:
                b = b + m
            c = torch.softmax(b, dim=2)
            v = squash(torch.matmul(c.unsqueeze(3), u).squeeze(3), -1)
        gu, gv = torch.autograd.grad(v, (u, vp), g_bar[:, t0:t1].transpose(0, 1))
        g_u[:, t0:t1] = gu.permute(1, 0, 3, 2, 4)                              # [n,B,J,I,Dv] -> [B,n,I,J,Dv]
        g_vp[:, t0:t1] = gv.transpose(0, 1)
    return g_u, g_vp


class NaiveMirror(torch.nn.Module):
    """Parameters are held in a dict of tensors keyed like ``srf_oracle.init_params``."""

    def __init__(self, shape, params, dtype=torch.float64, tile=True, fp8_pose=None):
        """tile=False contracts the pose with an einsum instead of the reference's
        tf.tile-materialised W (same products, float64; for full-size fixtures,
        whose tiled W would not fit in memory).  fp8_pose: per-layer bf16-u flags;
        the pose then takes the values of ``srf_oracle.pose_fp8`` (the build's opt-in
        e4m3 pose, not reference arithmetic) with the exact pose's gradient
        (straight-through), as the build's backward treats the pose as exact."""
        super().__init__()
        self.shape = shape
        self.tile = tile
        self.fp8_pose = fp8_pose
        self.p = torch.nn.ParameterDict()
        self.buffers_ = {}
        for k, v in params.items():
            t = torch.as_tensor(v, dtype=dtype)
            if k.endswith('moving_mean') or k.endswith('moving_var'):
                self.buffers_[k] = t.clone()
            else:
                self.p[k.replace('.', '__')] = torch.nn.Parameter(t.clone())

    def P(self, name):
        return self.p[name.replace('.', '__')]

    def forward(self, feats, inp_len, drop=None):
        sh = self.shape
        x = feats.unsqueeze(-1)
        for k in range(sh.cnn_n):
            x1 = conv2d_same(x, self.P(f'conv{k}a.kernel'), self.P(f'conv{k}a.bias'), 2)
            x2 = conv2d_same(x, self.P(f'conv{k}b.kernel'), self.P(f'conv{k}b.bias'), 2)
            if drop is not None:
                x1 = x1 * drop[f'conv{k}a']
                x2 = x2 * drop[f'conv{k}b']
            x = torch.maximum(x1, x2)
            x = feat_mask(x, inp_len, 2 ** (k + 1))
            x, _, _ = batch_norm_train(x, self.P(f'bn{k}.gamma'), self.P(f'bn{k}.beta'))
            x = feat_mask(x, inp_len, 2 ** (k + 1))
        B, T2, F2, C = x.shape
        emb = x.reshape(B, T2, F2 * C) @ self.P('proj.kernel') + self.P('proj.bias')
        if sh.caps_type == 'einsum':   # sequence_router_einsum.py:130-131
            pe = torch.as_tensor(so.pos_enc(T2, sh.ph), dtype=emb.dtype)
            emb = emb * so.einsum_scale(sh.ph) + pe
        emb = emb.unsqueeze(-1)
        e1 = conv2d_same(emb, self.P('encaps1.kernel'), self.P('encaps1.bias'), 1)
        e2 = conv2d_same(emb, self.P('encaps2.kernel'), self.P('encaps2.bias'), 1)
        if drop is not None:
            e1 = e1 * drop['encaps1']
            e2 = e2 * drop['encaps2']
        emb = feat_mask(torch.maximum(e1, e2), inp_len, 4)
        emb = squash(emb, -1)
        flat = layer_norm(emb.reshape(B, T2, -1), self.P('ln_input.gamma'), self.P('ln_input.beta'))
        if drop is not None and 'input' in drop:
            flat = flat * drop['input']
        emb = flat.reshape(B, T2, sh.ph, sh.pd)
        L = sh.enc_num
        for l in range(L):
            Tn = emb.shape[1]
            ep = F.pad(emb, (0, 0, 0, 0, sh.lpad, sh.rpad))
            xw = torch.cat([ep[:, w:w + Tn] for w in range(sh.window)], dim=2)
            if sh.caps_type == 'lowmemory' and not sh.context:
                J = self.P(f'W{l}').shape[1]
                u = xw.unsqueeze(3).repeat(1, 1, 1, J, 1)              # lowmemory:162, no W / bias
            elif self.tile:
                u = pose_tiled(xw, self.P(f'W{l}'), self.P(f'b{l}'))
            else:
                u = torch.einsum('ijde,btie->btijd', self.P(f'W{l}'), xw) + self.P(f'b{l}')
            if self.fp8_pose is not None:
                uq = so.pose_fp8(xw.detach().numpy(), self.P(f'W{l}').detach().numpy(),
                                 self.P(f'b{l}').detach().numpy(), bool(self.fp8_pose[l]))
                u = u + (torch.as_tensor(uq, dtype=u.dtype) - u).detach()
            if sh.context:
                v = sequential_routing(u, sh.route_iters, l == L - 1)
            else:
                v = dynamic_routing(u, sh.route_iters, l == L - 1)
            J, Dv = v.shape[2], v.shape[3]
            flat = layer_norm(v.reshape(B, Tn, J * Dv), self.P(f'ln_mid{l + 1}.gamma'),
                              self.P(f'ln_mid{l + 1}.beta'))
            if drop is not None and f'mid{l}' in drop:
                flat = flat * drop[f'mid{l}']
            emb = flat.reshape(B, Tn, J, Dv)
        return layer_norm(length(emb, -1, sh.length_eps), self.P('ln_output.gamma'), self.P('ln_output.beta'))


def ctc_per_utt(logits, labels, inp_len, tar_len, class_n, div=4):
    """trainer_sr.py:64-66 restated with torch's CTC (blank = C-1)."""
    lp = torch.log_softmax(logits, -1).transpose(0, 1)          # [T,B,C]
    lens = torch.ceil(inp_len.double() / div).long()
    return F.ctc_loss(lp, labels.long(), lens, tar_len.long(), blank=class_n - 1,
                      reduction='none', zero_infinity=False)


class TfAdam:
    """Keras Adam + CustomSchedule (train_helper.py:32-70): lr evaluated at the
    0-based iteration count, bias correction at iterations+1."""

    def __init__(self, params, k, d_model=1, warmup=25000, max_lr=1e3, b1=0.9, b2=0.98, eps=1e-9):
        self.params = list(params)
        self.k, self.d_model, self.warmup, self.max_lr = k, d_model, warmup, max_lr
        self.b1, self.b2, self.eps = b1, b2, eps
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.iterations = 0

    def lr(self, step):
        step = float(step)
        a1 = math.inf if step == 0 else 1.0 / math.sqrt(step)
        a2 = step * self.warmup ** -1.5
        return min(self.k / math.sqrt(self.d_model) * min(a1, a2), self.max_lr)

    @torch.no_grad()
    def step(self):
        lr = self.lr(self.iterations)
        t = self.iterations + 1
        alpha = lr * math.sqrt(1 - self.b2 ** t) / (1 - self.b1 ** t)
        for p, m, v in zip(self.params, self.m, self.v):
            g = p.grad
            m.mul_(self.b1).add_(g, alpha=1 - self.b1)
            v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            p.sub_(alpha * m / (v.sqrt() + self.eps))
        self.iterations += 1


def train_step(model, opt, feats, labels, inp_len, tar_len, n_gpus=1):
    """process_train_step (trainer_sr.py:41-75) on torch CPU ops."""
    T = int(inp_len.max())
    feats = feats[:, :T]
    for p in model.parameters():
        p.grad = None
    logits = model(feats, inp_len)
    pe = ctc_per_utt(logits, labels, inp_len, tar_len, model.shape.class_n)
    loss = pe.sum() / (feats.shape[0] * n_gpus)
    loss.backward()
    opt.step()
    return loss.detach(), pe.detach()
