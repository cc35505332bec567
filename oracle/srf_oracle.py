"""numpy float64 restatement of the reference SRF forward path -- TEST INFRASTRUCTURE ONLY.

Parity: unpinned against TensorFlow (see ``oracle/__init__.py``).  Every function
cites the reference file:line it restates (paths relative to the reference
checkout, ``tfsr/...``).  Keras/TF op semantics that the reference relies on but
does not spell out are restated explicitly and marked "[TF semantics]".

Layouts follow the reference: activations NHWC (H = time, W = frequency /
capsule index), conv kernels ``[kh, kw, Cin, Cout]``, routing weight
``W[in_n, out_n, out_d, in_d]`` and bias ``[in_n, out_n, out_d]`` (the reference
variables carry extra singleton axes, ``sequence_router_naive.py:88-103``).

``SrfShape.caps_type`` selects the reference variant (``trainer_sr.py:188-199``):
naive (the default), einsum (``sequence_router_einsum.py:129-131,238``) or lowmemory
(``sequence_router_lowmemory.py:107-109,162-164,190``).
"""
import math

import numpy as np

SQUASH_EPS = 1e-7      # sequence_router_naive.py:248, sequence_router.py:29
LENGTH_EPS = 1e-7      # sequence_router_naive.py:256
LN_EPS = 1e-3          # Keras LayerNormalization default (naive:104-107)
BN_EPS = 1e-3          # Keras BatchNormalization default (sequence_router.py:64)
BN_MOMENTUM = 0.99     # Keras BatchNormalization default
MASK_LOGIT = -1e9      # sequence_router_naive.py:176,219


# ----------------------------------------------------------------------------
# TF / Keras primitive semantics
# ----------------------------------------------------------------------------
def same_pad(n, k, s):
    """[TF semantics] 'SAME' padding: out = ceil(n/s); pad_before = total//2."""
    out = -(-n // s)
    total = max((out - 1) * s + k - n, 0)
    return out, total // 2, total - total // 2


def conv2d_same(x, kern, bias, stride):
    """Keras Conv2D(padding='same') on NHWC; kern [kh, kw, Cin, Cout].

    Restates the Conv2D layers of ``sequence_router.py:48-53`` (stride 2) and
    ``sequence_router_naive.py:77-81`` (stride 1).
    """
    B, H, W, Cin = x.shape
    kh, kw, _, Cout = kern.shape
    Ho, pt, pb = same_pad(H, kh, stride)
    Wo, pl, pr = same_pad(W, kw, stride)
    xp = np.pad(x, ((0, 0), (pt, pb), (pl, pr), (0, 0)))
    out = np.zeros((B, Ho, Wo, Cout), dtype=x.dtype)
    for a in range(kh):
        for c in range(kw):
            patch = xp[:, a:a + stride * (Ho - 1) + 1:stride, c:c + stride * (Wo - 1) + 1:stride, :]
            out += patch @ kern[a, c]
    return out + bias


def mask_lengths(inp_len, div):
    """``model_helper.py:136``: ceil(int32(len) / div) (TF true division -> ceil)."""
    return np.ceil(np.asarray(inp_len).astype(np.int32) / div).astype(np.int64)


def feat_mask(x, inp_len, div):
    """``model_helper.py:125-140``: zero time steps t >= ceil(len/div)."""
    lens = mask_lengths(inp_len, div)
    T = x.shape[1]
    m = (np.arange(T)[None, :] < lens[:, None]).astype(x.dtype)
    assert m.shape[1] == T
    return x * m.reshape(m.shape + (1,) * (x.ndim - 2))


def batch_norm(x, gamma, beta, mean=None, var=None, training=True):
    """[TF semantics] Keras BatchNormalization(axis=-1), eps 1e-3.

    Training: batch statistics over every axis but the last, biased variance,
    zero-masked padded positions included.  Returns
    (y, batch_mean, batch_var_unbiased) -- the unbiased variance is what the fused
    NHWC kernel feeds the moving average [inference: TF FusedBatchNorm].
    """
    axes = tuple(range(x.ndim - 1))
    if training:
        mu = x.mean(axis=axes)
        var_b = x.var(axis=axes)
        n = x.size // x.shape[-1]
        var_u = var_b * n / max(n - 1, 1)
    else:
        mu, var_b, var_u = mean, var, var
    y = (x - mu) / np.sqrt(var_b + BN_EPS) * gamma + beta
    return y, mu, var_u


def layer_norm(x, gamma, beta):
    """Keras LayerNormalization over the last axis, eps 1e-3 (naive:104-107)."""
    mu = x.mean(-1, keepdims=True)
    var = x.var(-1, keepdims=True)
    return (x - mu) / np.sqrt(var + LN_EPS) * gamma + beta


def squash(s, axis=-1, eps=SQUASH_EPS):
    """``sequence_router_naive.py:247-253``."""
    n2 = np.sum(np.square(s), axis=axis, keepdims=True)
    return n2 / (1.0 + n2) * (s / np.sqrt(n2 + eps))


def length(s, axis=-1, eps=LENGTH_EPS):
    """``sequence_router_naive.py:255-258``."""
    return np.sqrt(np.sum(np.square(s), axis=axis) + eps)


def softmax(b, axis):
    m = np.max(b, axis=axis, keepdims=True)
    e = np.exp(b - m)
    return e / e.sum(axis=axis, keepdims=True)


# ----------------------------------------------------------------------------
# Capsule layer pieces
# ----------------------------------------------------------------------------
def window(emb, lpad, rpad):
    """``sequence_router_naive.py:150-151``: ZeroPadding2D on time, then concat of
    the lpad+1+rpad shifted views on the capsule axis (capsule i = w*N + n)."""
    B, T, N, D = emb.shape
    ep = np.pad(emb, ((0, 0), (lpad, rpad), (0, 0), (0, 0)))
    return np.concatenate([ep[:, w:w + T] for w in range(lpad + rpad + 1)], axis=2)


def pose(x, W, bias):
    """``sequence_router_naive.py:154-159``: u[b,t,i,j,:] = W[i,j] @ x[b,t,i] + bias[i,j]."""
    return np.einsum('ijde,btie->btijd', W, x) + bias


def e4m3_round(a):
    """OCP e4m3 (fn) round-to-nearest-even of |a| <= 448 (subnormals down to 2^-9).
    Not reference arithmetic: the numerics of the build's opt-in fp8 pose
    (``include/srf.h`` srf_route_sdr_pose_n mode 1/2), restated to check it."""
    a = np.asarray(a, dtype=np.float64)
    mag = np.abs(a)
    e = np.floor(np.log2(np.where(mag > 0, mag, 1.0)))
    q = np.exp2(np.maximum(e, -6.0) - 3.0)      # 3 mantissa bits; exponent floor -6
    return np.sign(a) * np.round(mag / q) * q   # np.round: half to even


def e4m3_scale_exp(amax):
    """Per-vector power-of-two scale 2^e with amax * 2^e in (224, 448]: e = e0 - 1
    where 448/amax = m 2^e0, m in [0.5, 1), the quotient rounded to float32 as the
    kernel computes it; 0 for an all-zero vector; clamped to [-100, 100]."""
    amax = np.asarray(amax, dtype=np.float32)
    with np.errstate(divide='ignore'):
        q = np.float32(448.0) / np.where(amax > 0, amax, np.float32(1.0))
    _, e0 = np.frexp(q)
    e = np.clip(e0.astype(np.int64) - 1, -100, 100)
    return np.where(amax > 0, e, 0)


def bf16_round(a):
    """float32 -> bf16 round to nearest even, back to float64."""
    x = np.asarray(a, dtype=np.float32).view(np.uint32).astype(np.uint64)
    x = (x + 0x7FFF + ((x >> 16) & 1)) >> 16 << 16
    return x.astype(np.uint32).view(np.float32).astype(np.float64)


def pose_fp8(x, W, bias, bf16_u=False):
    """The fp8 pose transform as the build declares it (not reference arithmetic):
    every frame's input capsule x[b,t,i,:] and every row W[i,j,d,:] rounded to
    float32, scaled by its own 2^e (``e4m3_scale_exp``) and rounded to e4m3; exact
    products summed, scaled back, float32 bias added; u optionally stored as bf16.
    x [B,T,I,E], W [I,J,D,E] -> u [B,T,I,J,D]."""
    x32 = np.asarray(x, np.float32).astype(np.float64)
    W32 = np.asarray(W, np.float32).astype(np.float64)
    ex = e4m3_scale_exp(np.abs(x32).max(-1))
    ew = e4m3_scale_exp(np.abs(W32).max(-1))
    xq = e4m3_round(x32 * np.exp2(ex)[..., None])
    wq = e4m3_round(W32 * np.exp2(ew)[..., None])
    u = np.einsum('ijde,btie->btijd', wq, xq)
    u = u * np.exp2(-ex)[..., None, None] * np.exp2(-ew)[None, None] + np.asarray(bias, np.float32)
    return bf16_round(u) if bf16_u else np.asarray(u, np.float32).astype(np.float64)


def dynamic_routing(u, iters, mask_first):
    """DR, ``sequence_router_naive.py:171-185`` + ``_loop_body`` ``:199-206``.

    u [B,T,I,J,D].  The mask (-1e9 on output capsule 0, last layer only) is added
    to the logits every iteration (``:201``)."""
    B, T, I, J, D = u.shape
    b = np.zeros((B, T, I, J), dtype=u.dtype)
    m = np.zeros_like(b)
    if mask_first:
        m[..., 0] = MASK_LOGIT
    v = None
    for _ in range(iters):
        b = b + m
        c = softmax(b, axis=3)
        s = np.einsum('btij,btijd->btjd', c, u)
        v = squash(s, -1)
        b = b + np.einsum('btijd,btjd->btij', u, v)
    return v


def sequential_routing(u, iters, mask_first):
    """SDR, ``sequence_router_naive.py:162-170`` + ``body_context`` ``:231-245`` /
    ``pad_body_context`` ``:212-229``: frames routed in order, the previous frame's
    final v seeds the agreement of the next frame (v_0 = 0)."""
    B, T, I, J, D = u.shape
    v = np.zeros((B, J, D), dtype=u.dtype)
    m = np.zeros((B, I, J), dtype=u.dtype)
    if mask_first:
        m[..., 0] = MASK_LOGIT
    out = np.zeros((B, T, J, D), dtype=u.dtype)
    for t in range(T):
        ut = u[:, t]
        b = np.zeros((B, I, J), dtype=u.dtype)
        for _ in range(iters):
            b = b + np.einsum('bijd,bjd->bij', ut, v)
            if mask_first:
                b = b + m
            c = softmax(b, axis=2)
            s = np.einsum('bij,bijd->bjd', c, ut)
            v = squash(s, -1)
        out[:, t] = v
    return out


# ----------------------------------------------------------------------------
# Model configuration / parameters
# ----------------------------------------------------------------------------
class SrfShape:
    """Static shape of a SequenceRouter (``sequence_router_naive.py:42-103``)."""

    def __init__(self, feat_dim=123, nfilt=64, cnn_n=2, enc_num=3, iters=3, lpad=4, rpad=4,
                 ph=8, pd=8, ch=8, cd=8, vd=8, class_n=63, context=False, caps_type='naive'):
        self.feat_dim, self.nfilt, self.cnn_n = feat_dim, nfilt, cnn_n
        self.caps_type = caps_type   # trainer_sr.py:188-199: lowmemory | einsum | naive
        self.enc_num, self.iters, self.lpad, self.rpad = enc_num, iters, lpad, rpad
        self.ph, self.pd, self.ch, self.cd, self.vd = ph, pd, ch, cd, vd
        self.class_n, self.context = class_n, context
        self.window = lpad + rpad + 1
        # lowmemory routes once whatever --model-caps-iter says (lowmemory:107-109,190)
        self.route_iters = 1 if caps_type == 'lowmemory' else iters
        self.length_eps = 1e-9 if caps_type == 'einsum' else LENGTH_EPS   # einsum:238 / naive:256
        self.feat_out = math.ceil(feat_dim / (2 * cnn_n))   # naive:50 (quirk: only right for cnn_n=2)

    def layer_shapes(self):
        """(in_n, out_n, out_d, in_d) per routing layer, ``naive:88-95``."""
        w = self.window
        if self.enc_num == 1:
            return [(self.ph * w, self.class_n, self.vd, self.pd)]
        s = [(self.ph * w, self.ch, self.cd, self.pd)]
        for _ in range(1, self.enc_num - 1):
            s.append((self.ch * w, self.ch, self.cd, self.cd))
        s.append((self.ch * w, self.class_n, self.vd, self.cd))
        return s


def init_params(shape, seed=0, randomize_norms=True, dtype=np.float64):
    """Random parameters with the reference's initialisers (fan_avg uniform for
    conv/dense kernels, ``model_helper.py:156-160``; N(0, 0.1) for W and bias,
    ``naive:97-103``).  ``randomize_norms`` perturbs LN/BN gamma/beta away from
    1/0 so tests see the padded-frame beta leakage."""
    rng = np.random.default_rng(seed)
    P = {}

    def fan_avg(kshape):
        rf = int(np.prod(kshape[:-2])) if len(kshape) > 2 else 1
        fan_in, fan_out = kshape[-2] * rf, kshape[-1] * rf
        lim = math.sqrt(3.0 / max(1.0, (fan_in + fan_out) / 2.0))
        return rng.uniform(-lim, lim, size=kshape)

    def norm(n, tag):
        if randomize_norms:
            P[tag + '.gamma'] = 1.0 + 0.1 * rng.standard_normal(n)
            P[tag + '.beta'] = 0.1 * rng.standard_normal(n)
        else:
            P[tag + '.gamma'] = np.ones(n)
            P[tag + '.beta'] = np.zeros(n)

    cin = 1
    for k in range(shape.cnn_n):
        for ab in 'ab':
            P[f'conv{k}{ab}.kernel'] = fan_avg((3, 3, cin, shape.nfilt))
            P[f'conv{k}{ab}.bias'] = (0.05 * rng.standard_normal(shape.nfilt)) if randomize_norms \
                else np.zeros(shape.nfilt)
        norm(shape.nfilt, f'bn{k}')
        P[f'bn{k}.moving_mean'] = np.zeros(shape.nfilt)
        P[f'bn{k}.moving_var'] = np.ones(shape.nfilt)
        cin = shape.nfilt
    P['proj.kernel'] = fan_avg((shape.feat_out * shape.nfilt, shape.ph))
    P['proj.bias'] = 0.05 * rng.standard_normal(shape.ph) if randomize_norms else np.zeros(shape.ph)
    for e in (1, 2):
        P[f'encaps{e}.kernel'] = fan_avg((3, 3, 1, shape.pd))
        P[f'encaps{e}.bias'] = 0.05 * rng.standard_normal(shape.pd) if randomize_norms else np.zeros(shape.pd)
    norm(shape.ph * shape.pd, 'ln_input')
    for l, (in_n, out_n, out_d, in_d) in enumerate(shape.layer_shapes()):
        P[f'W{l}'] = 0.1 * rng.standard_normal((in_n, out_n, out_d, in_d))
        P[f'b{l}'] = 0.1 * rng.standard_normal((in_n, out_n, out_d))
        norm(out_n * out_d, f'ln_mid{l + 1}')
    norm(shape.class_n, 'ln_output')
    return {k: np.asarray(v, dtype=dtype) for k, v in P.items()}


# ----------------------------------------------------------------------------
# Forward
# ----------------------------------------------------------------------------
def cnn_fe(P, shape, feats, inp_len, bn_training=True, drop=None):
    """``CapsulationLayer.call`` (``sequence_router.py:69-82``).  ``drop`` maps
    names ``conv{k}{a|b}`` to inverted-dropout multipliers (keep/(1-p)) or is None
    (dropout off).  Returns (x, bn_stats)."""
    x = feats[..., None]
    stats = []
    for k in range(shape.cnn_n):
        # Masking layer (:73) is numerically the identity.
        x1 = conv2d_same(x, P[f'conv{k}a.kernel'], P[f'conv{k}a.bias'], 2)
        x2 = conv2d_same(x, P[f'conv{k}b.kernel'], P[f'conv{k}b.bias'], 2)
        if drop is not None:
            x1 = x1 * drop[f'conv{k}a']
            x2 = x2 * drop[f'conv{k}b']
        x = np.maximum(x1, x2)                                   # :76
        x = feat_mask(x, inp_len, 2 ** (k + 1))                  # :77
        x, mu, var = batch_norm(x, P[f'bn{k}.gamma'], P[f'bn{k}.beta'],
                                P[f'bn{k}.moving_mean'], P[f'bn{k}.moving_var'], bn_training)
        stats.append((mu, var))
        x = feat_mask(x, inp_len, 2 ** (k + 1))                  # :79
    return x, stats


def pos_enc(length, hidden):
    """``get_pos_enc`` (model_helper.py:30-58), computed in float32 as the reference
    does: [sin(t * inv_k) | cos(t * inv_k)], inv_k = exp(-k * log(1e4) / (hidden/2 - 1))."""
    f32 = np.float32
    nts = hidden // 2
    inc = f32(math.log(1e4 / 1.0)) / (f32(nts) - f32(1))
    inv = np.exp(np.arange(nts, dtype=f32) * -inc).astype(f32)
    st = np.arange(length, dtype=f32)[:, None] * inv[None, :]
    return np.concatenate([np.sin(st), np.cos(st)], axis=1).astype(f32)


def einsum_scale(ph):
    """tf.math.sqrt(tf.cast(ph, tf.float32)) (einsum:130), the float32 value."""
    return float(np.sqrt(np.float32(ph)))


def primary_caps(P, shape, conv_out, inp_len, drop=None):
    """``sequence_router_naive.py:129-142``; einsum variant adds the sqrt(PH) scale
    and positional encoding after proj_pe (``sequence_router_einsum.py:129-131``)."""
    B, T2, F2, C = conv_out.shape
    emb = conv_out.reshape(B, T2, F2 * C) @ P['proj.kernel'] + P['proj.bias']   # :131-132
    if shape.caps_type == 'einsum':
        emb = emb * einsum_scale(shape.ph) + pos_enc(T2, shape.ph)
    emb = emb[..., None]                                                        # [B,T',PH,1]
    e1 = conv2d_same(emb, P['encaps1.kernel'], P['encaps1.bias'], 1)
    e2 = conv2d_same(emb, P['encaps2.kernel'], P['encaps2.bias'], 1)
    if drop is not None:
        e1 = e1 * drop['encaps1']
        e2 = e2 * drop['encaps2']
    emb = np.maximum(e1, e2)                                                    # :133
    emb = feat_mask(emb, inp_len, 4)                                            # :134 (Masking :135 = id)
    emb = squash(emb, -1)                                                       # :137
    flat = emb.reshape(B, T2, shape.ph * shape.pd)
    flat = layer_norm(flat, P['ln_input.gamma'], P['ln_input.beta'])            # :139-141
    if drop is not None and 'input' in drop:
        flat = flat * drop['input']
    return flat.reshape(B, T2, shape.ph, shape.pd)


def routing_layers(P, shape, emb, drop=None, return_all=False):
    """Per-layer window -> pose -> DR/SDR -> LN (+dropout); ``naive:145-193``.
    lowmemory: one iteration, and DR without W / bias, u_ij = x_i (lowmemory:162-164)."""
    outs = []
    L = shape.enc_num
    for l in range(L):
        B, T, N, D = emb.shape
        x = window(emb, shape.lpad, shape.rpad)
        last = l == L - 1
        if shape.caps_type == 'lowmemory' and not shape.context:
            J = P[f'W{l}'].shape[1]
            u = np.broadcast_to(x[:, :, :, None, :], x.shape[:3] + (J, x.shape[3]))   # tf.tile :162
        else:
            u = pose(x, P[f'W{l}'], P[f'b{l}'])
        if shape.context:
            v = sequential_routing(u, shape.route_iters, last)
        else:
            v = dynamic_routing(u, shape.route_iters, last)
        J, Dv = v.shape[2], v.shape[3]
        outs.append(v)
        # every layer, the last included, is LN'd (ln_mid%d, :187-191) before length/ln_o
        flat = layer_norm(v.reshape(B, T, J * Dv), P[f'ln_mid{l + 1}.gamma'], P[f'ln_mid{l + 1}.beta'])
        if drop is not None and f'mid{l}' in drop:
            flat = flat * drop[f'mid{l}']
        emb = flat.reshape(B, T, J, Dv)
    logits = layer_norm(length(emb, -1, shape.length_eps), P['ln_output.gamma'], P['ln_output.beta'])  # :193
    return (logits, outs) if return_all else logits


def srf_forward(P, shape, feats, inp_len, bn_training=True, drop=None):
    """``SequenceRouter.call`` (naive:120-193): feats [B,T,F] (already cropped to
    max(inp_len), ``trainer_sr.py:59-60``) -> logits [B, ceil(T/4), class_n]."""
    conv_out, _ = cnn_fe(P, shape, feats, inp_len, bn_training, drop)
    emb = primary_caps(P, shape, conv_out, inp_len, drop)
    return routing_layers(P, shape, emb, drop)


# ----------------------------------------------------------------------------
# CTC + decoding
# ----------------------------------------------------------------------------
def log_softmax(x, axis=-1):
    m = x.max(axis=axis, keepdims=True)
    return x - m - np.log(np.exp(x - m).sum(axis=axis, keepdims=True))


def ctc_nll(logits, labels, blank):
    """CTC negative log likelihood of one utterance (log-space alpha recursion).

    Restates ``tf.nn.ctc_loss`` as called at ``trainer_sr.py:64-66`` (dense labels,
    batch-major logits, ``blank_index = C-1``): standard CTC NLL with log-softmax
    applied to the logits.  logits [T, C], labels [L]."""
    lp = log_softmax(np.asarray(logits, dtype=np.float64), -1)
    T = lp.shape[0]
    L = len(labels)
    S = 2 * L + 1
    ext = np.full(S, blank, dtype=np.int64)
    ext[1::2] = labels
    neg = -np.inf
    alpha = np.full(S, neg)
    if T == 0:
        return np.inf
    alpha[0] = lp[0, blank]
    if S > 1:
        alpha[1] = lp[0, ext[1]]
    for t in range(1, T):
        new = np.full(S, neg)
        for s in range(S):
            a = alpha[s]
            if s >= 1:
                a = np.logaddexp(a, alpha[s - 1])
            if s >= 2 and ext[s] != blank and ext[s] != ext[s - 2]:
                a = np.logaddexp(a, alpha[s - 2])
            new[s] = a + lp[t, ext[s]]
        alpha = new
    ll = alpha[S - 1] if S == 1 else np.logaddexp(alpha[S - 1], alpha[S - 2])
    return -ll


def ctc_batch(logits, labels, inp_len, tar_len, class_n, div=4):
    """Per-utterance NLL as ``trainer_sr.py:64-66``: logit_length = ceil(len/4)."""
    lens = np.ceil(np.asarray(inp_len) / div).astype(np.int64)
    return np.array([ctc_nll(logits[b, :lens[b]], labels[b, :tar_len[b]], class_n - 1)
                     for b in range(logits.shape[0])])


def greedy_decode(logits, lengths, blank):
    """Best-path decode: per-frame argmax, merge repeats, drop blank."""
    out = []
    for b in range(logits.shape[0]):
        best = np.argmax(logits[b, :lengths[b]], axis=-1)
        seq, prev = [], -1
        for k in best:
            if k != prev and k != blank:
                seq.append(int(k))
            prev = k
        out.append(seq)
    return out
