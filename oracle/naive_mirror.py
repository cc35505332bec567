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
