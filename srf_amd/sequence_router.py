"""``SequenceRouter`` -- drop-in for tfsr/model/sequence_router_naive.py:33-258.

Same constructor ``SequenceRouter(config, logger, class_n)`` and call
``model(feats, input_lengths=..., training=...)`` returning logits
[B, ceil(T/4), class_n].  ``feats`` must already be cropped to max(inp_len)
(trainer_sr.py:59-60), as in the reference.

Compute placement: every stage runs in the HIP library through ``srf_amd.ops``
(CNN front end, primary capsules, the routing layers, the per-layer norms and
the output head); there is no CPU or torch-op fallback.  All parameters are
views into one flat fp32 buffer (``flat_params``) with a matching flat gradient
buffer, so the data-parallel all-reduce and the Adam update are one launch each.
Dropout masks come from a counter-based RNG keyed by a per-call seed, so the
backward kernels regenerate them instead of storing them.
"""
import math

import numpy as np
import torch

from . import ops

SQUASH_EPS = 1e-7   # naive:248
LENGTH_EPS = 1e-7   # naive:256
LENGTH_EPS_EINSUM = 1e-9   # sequence_router_einsum.py:238
CAPS_TYPES = ('lowmemory', 'einsum', 'naive')   # trainer_sr.py:188-199, common_helper.py:228-231
LN_EPS = 1e-3       # Keras LayerNormalization default
BN_EPS = 1e-3       # Keras BatchNormalization default
BN_MOMENTUM = 0.99
CNN_DROPOUT = 0.2   # hard-coded, sequence_router.py:62 and naive:82


def _replica_id():
    import torch.distributed as dist
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


class SequenceRouter(torch.nn.Module):
    """SRF acoustic model.  ``config.model_caps_type`` picks the reference variant
    (trainer_sr.py:188-199); all three run on the same HIP kernels:

    * ``naive`` (sequence_router_naive.py): the semantics everything else is built to;
    * ``einsum`` (sequence_router_einsum.py): proj_pe output scaled by sqrt(PH) plus the
      sinusoidal positional encoding (:129-131), output length eps 1e-9 (:238);
    * ``lowmemory`` (sequence_router_lowmemory.py): one routing iteration whatever
      --model-caps-iter says (:107-109,190); its DR layers route the windowed input
      capsules themselves, u_ij = x_i, without W or bias (:162-164), so W%d / b%d of a
      DR layer get no gradient (TF's apply_gradients skips them).  The DR kernels run
      with an identity W and zero bias for that; the SDR layers keep W and bias
      (lowmemory:226-250).
    """

    iter = -1  # class-level like the reference (naive:40,56): shared by every instance

    def __init__(self, config, logger, class_n, device=None, seed=None, replica_id=None):
        super().__init__()
        dev = torch.device(device) if device is not None else torch.device('cuda', torch.cuda.current_device())
        self.stride = 2
        self.cnn_n = config.model_conv_layer_num
        if self.cnn_n != 2:
            # the reference's transposed conv-list indexing only works for 2 layers
            # (sequence_router.py:76-77)
            raise ValueError('model-conv-layer-num must be 2 (as in the reference CapsulationLayer)')
        self.feat_dim_in = config.feat_dim
        self.feat_dim = math.ceil(config.feat_dim / (self.stride * self.cnn_n))   # naive:50
        self.nfilt = config.model_conv_filter_num
        self.class_n = class_n
        self.enc_num = config.model_encoder_num
        self.iter = SequenceRouter.iter = config.model_caps_iter
        self.lpad = config.model_caps_window_lpad
        self.rpad = config.model_caps_window_rpad
        self.window = self.lpad + self.rpad + 1
        self.is_context = bool(config.model_caps_context)
        self.caps_inp_n = config.model_caps_primary_num
        self.caps_inp_d = config.model_caps_primary_dim
        self.caps_cov_n = config.model_caps_convolution_num
        self.caps_cov_d = config.model_caps_convolution_dim
        self.caps_cls_d = config.model_caps_class_dim
        self.inp_dropout = float(config.train_inp_dropout)
        self.inn_dropout = float(config.train_inn_dropout)
        self.init = config.model_initializer
        self.caps_type = getattr(config, 'model_caps_type', 'naive')
        if self.caps_type not in CAPS_TYPES:
            raise ValueError('model-caps-type must be lowmemory, einsum or naive but %s' % self.caps_type)
        self.route_iters = 1 if self.caps_type == 'lowmemory' else self.iter
        self.proj_scale = math.sqrt(self.caps_inp_n) if self.caps_type == 'einsum' else 1.0
        self.length_eps = LENGTH_EPS_EINSUM if self.caps_type == 'einsum' else LENGTH_EPS
        # Opt-in fp8 (e4m3) pose transform for SDR stacks (BASELINE C5 "fp8 pose-transform
        # MFMA"; not a reference flag: the reference is fp32 throughout).  Its bound is
        # stated in include/srf.h (srf_route_sdr_pose_fp8); gradients stay fp32.
        self.pose_fp8 = bool(getattr(config, 'model_pose_fp8', False))
        self.dropout_enabled = True     # test hook: parity runs use BN batch stats without dropout
        self.n_chunks_override = {}     # DR layer -> input-capsule chunks of its routing passes (plan argument)
        # SDR: every layer as one layer-pipelined wavefront (ops.SdrStack; False: layer by
        # layer), with ops.SdrStackPlan options (n_chunks, store_couplings, store_u_bytes, u_bf16)
        self.sdr_stack = True
        self.sdr_options = {}
        # Dropout seed base.  Parameters are initialised from `seed` identically on every
        # replica (MirroredStrategy mirrors one set of variables), but each replica draws
        # its own dropout masks, so the replica id is mixed in (rank 0 keeps the plain
        # seed's stream).
        self._seed_base = int(np.random.default_rng(seed).integers(1, 2 ** 62))
        self.replica_id = _replica_id() if replica_id is None else int(replica_id)
        if self.replica_id:
            self._seed_base = int(np.random.default_rng([self._seed_base, self.replica_id]).integers(1, 2 ** 62))
        self._calls = 0
        # grad_hook(names): called from the backward once the gradient kernels of those
        # parameters are enqueued (trainer_sr.GradBuckets); None: no hooks
        self.grad_hook = None
        self.grad_buckets = None

        w = self.window
        if self.enc_num > 1:   # (in_n, out_n, out_d, in_d), naive:88-95
            shapes = [(self.caps_inp_n * w, self.caps_cov_n, self.caps_cov_d, self.caps_inp_d)]
            shapes += [(self.caps_cov_n * w, self.caps_cov_n, self.caps_cov_d, self.caps_cov_d)] * (self.enc_num - 2)
            shapes.append((self.caps_cov_n * w, class_n, self.caps_cls_d, self.caps_cov_d))
        else:
            shapes = [(self.caps_inp_n * w, class_n, self.caps_cls_d, self.caps_inp_d)]
        self.layer_shapes = shapes

        spec = []   # (name, shape, init)
        cin = 1
        for k in range(self.cnn_n):
            for ab in 'ab':
                spec.append((f'conv{k}{ab}_kernel', (3, 3, cin, self.nfilt), 'kernel'))
                spec.append((f'conv{k}{ab}_bias', (self.nfilt,), 'zeros'))
            spec.append((f'bn{k}_gamma', (self.nfilt,), 'ones'))
            spec.append((f'bn{k}_beta', (self.nfilt,), 'zeros'))
            cin = self.nfilt
        spec.append(('proj_kernel', (self.feat_dim * self.nfilt, self.caps_inp_n), 'kernel'))
        spec.append(('proj_bias', (self.caps_inp_n,), 'zeros'))
        for e in (1, 2):
            spec.append((f'encaps{e}_kernel', (3, 3, 1, self.caps_inp_d), 'kernel'))
            spec.append((f'encaps{e}_bias', (self.caps_inp_d,), 'zeros'))
        spec.append(('ln_input_gamma', (self.caps_inp_n * self.caps_inp_d,), 'ones'))
        spec.append(('ln_input_beta', (self.caps_inp_n * self.caps_inp_d,), 'zeros'))
        for l, (in_n, out_n, out_d, in_d) in enumerate(shapes):
            spec.append((f'W{l}', (in_n, out_n, out_d, in_d), 'normal0.1'))
            spec.append((f'b{l}', (in_n, out_n, out_d), 'normal0.1'))
            spec.append((f'ln_mid{l + 1}_gamma', (out_n * out_d,), 'ones'))
            spec.append((f'ln_mid{l + 1}_beta', (out_n * out_d,), 'zeros'))
        spec.append(('ln_output_gamma', (class_n,), 'ones'))
        spec.append(('ln_output_beta', (class_n,), 'zeros'))
        self._spec = spec

        offsets, off = {}, 0
        for name, shape, _ in spec:
            offsets[name] = off
            off += (int(np.prod(shape)) + 63) // 64 * 64   # 256-B aligned slices (float4 kernel loads)
        self.n_flat = off
        self.flat_params = torch.zeros(off, device=dev, dtype=torch.float32)
        self.flat_grad = torch.zeros(off, device=dev, dtype=torch.float32)
        self.params = torch.nn.ParameterDict()
        rng = np.random.default_rng(seed)
        for name, shape, init in spec:
            n = int(np.prod(shape))
            view = self.flat_params[offsets[name]:offsets[name] + n].view(shape)
            with torch.no_grad():
                view.copy_(torch.from_numpy(self._init_value(rng, shape, init)))
            p = torch.nn.Parameter(view)
            p.grad = self.flat_grad[offsets[name]:offsets[name] + n].view(shape)
            p._srf_flat = True    # backward kernels write this gradient in place (overwrite)
            self.params[name] = p
        self.offsets = offsets
        for k in range(self.cnn_n):
            self.register_buffer(f'bn{k}_moving_mean', torch.zeros(self.nfilt, device=dev))
            self.register_buffer(f'bn{k}_moving_var', torch.ones(self.nfilt, device=dev))
        self._geoms = {}
        self._identity = {}
        if self.caps_type == 'lowmemory' and not self.is_context:
            for l, (in_n, out_n, out_d, in_d) in enumerate(shapes):
                if out_d != in_d:
                    # u_hat = tile(x) has in_d components; the reshape to out_n*out_d
                    # (lowmemory:196-197) only works when they agree
                    raise ValueError(f'lowmemory DR needs equal capsule dims, layer {l}: {in_d} -> {out_d}')
                eye = torch.eye(in_d, device=dev, dtype=torch.float32).expand(in_n, out_n, in_d, in_d)
                self._identity[l] = (eye.contiguous(), torch.zeros((in_n, out_n, out_d), device=dev))
        if logger is not None:
            logger.info('Layer x %d, Iter x %d, Init %s, Win %d (l:%d, r:%d), ' % (
                self.enc_num, SequenceRouter.iter, 'SDR' if self.is_context else 'DR', self.window, self.lpad,
                self.rpad))

    def _init_value(self, rng, shape, init):
        """Keras initialisers used by the reference (model_helper.py:156-164,
        naive:97-103); conv/dense biases, LN/BN as Keras defaults."""
        if init == 'zeros':
            return np.zeros(shape, np.float32)
        if init == 'ones':
            return np.ones(shape, np.float32)
        if init == 'normal0.1':
            return (0.1 * rng.standard_normal(shape)).astype(np.float32)
        # kernel: fan_avg uniform (== glorot_uniform), or uniform(-0.05, 0.05)
        if self.init == 'uniform':
            return rng.uniform(-0.05, 0.05, size=shape).astype(np.float32)
        rf = int(np.prod(shape[:-2])) if len(shape) > 2 else 1
        fan_in, fan_out = shape[-2] * rf, shape[-1] * rf
        lim = math.sqrt(6.0 / (fan_in + fan_out))
        return rng.uniform(-lim, lim, size=shape).astype(np.float32)

    # ------------------------------------------------------------------ utils
    def P(self, name):
        return self.params[name]

    def zero_grad(self, set_to_none=False):
        self.flat_grad.zero_()

    def load_params(self, named):
        """Copy parameters from a dict keyed like ``conv0a.kernel`` / ``W0``."""
        with torch.no_grad():
            for k, v in named.items():
                key = k.replace('.', '_')
                if key.endswith('moving_mean') or key.endswith('moving_var'):
                    getattr(self, key).copy_(torch.as_tensor(v, dtype=torch.float32))
                else:
                    self.params[key].copy_(torch.as_tensor(v, dtype=torch.float32))

    def export_params(self):
        """Parameters + BN moving statistics as numpy, keyed like ``conv0a.kernel``."""
        out = {}
        for k, v in self.params.items():
            head, _, tail = k.rpartition('_')
            key = f'{head}.{tail}' if tail in ('kernel', 'bias', 'gamma', 'beta') else k
            out[key] = v.detach().cpu().numpy()
        for k in range(self.cnn_n):
            out[f'bn{k}.moving_mean'] = getattr(self, f'bn{k}_moving_mean').cpu().numpy()
            out[f'bn{k}.moving_var'] = getattr(self, f'bn{k}_moving_var').cpu().numpy()
        return out

    def _geom(self, l, B, T):
        key = (l, B, T)
        g = self._geoms.get(key)
        if g is None:
            in_n, out_n, out_d, in_d = self.layer_shapes[l]
            N = in_n // self.window
            g = ops.RouteGeom(B, T, N, in_d, self.lpad, self.rpad, out_n, out_d, self.route_iters,
                              l == self.enc_num - 1, self.n_chunks_override.get(l, 0))
            self._geoms[key] = g
        return g

    def _stack_plan(self, B, T):
        key = ('sdr_stack', B, T)
        p = self._geoms.get(key)
        if p is None:
            layers = []
            for l, (in_n, out_n, out_d, in_d) in enumerate(self.layer_shapes):
                layers.append((in_n // self.window, in_d, out_n, out_d, int(l == self.enc_num - 1)))
            p = ops.SdrStackPlan(B, T, layers, self.lpad, self.rpad, self.route_iters, pose_fp8=self.pose_fp8,
                                 **self.sdr_options)
            self._geoms[key] = p
        return p

    def _on_grad(self, t, names):
        """Tell grad_hook that ``names``' gradients are enqueued once the backward has
        produced the gradient of ``t`` (the input of the op that writes them)."""
        hook = self.grad_hook
        if hook is not None and t.requires_grad and torch.is_grad_enabled():
            def fire(g, names=tuple(names)):
                hook(names)
            t.register_hook(fire)

    def _next_seed(self):
        self._calls += 1
        return (self._seed_base * 0x9E3779B1 + self._calls) % (1 << 63)

    # ---------------------------------------------------------------- forward
    def forward(self, feats, input_lengths=None, training=False, **kwargs):
        """naive:120-193.  Extra kwargs (mask=, att_mask=) are ignored like the
        reference's Keras call."""
        inp_len = input_lengths
        if not torch.is_tensor(inp_len):
            inp_len = torch.as_tensor(inp_len)
        il32 = inp_len.to(device=feats.device, dtype=torch.int32).contiguous()
        drop = bool(training) and self.dropout_enabled
        seed = self._next_seed() if drop else 0
        moving = [getattr(self, n) for n in ('bn0_moving_mean', 'bn0_moving_var', 'bn1_moving_mean',
                                             'bn1_moving_var')]
        x = ops.cnnfe(feats.contiguous(), il32, [self.P(k) for k in ops.CNNFE_PARAMS], moving, training,
                      CNN_DROPOUT if drop else 0.0, seed)
        self._on_grad(x, ops.CAPS_PARAMS)
        emb = ops.primary_caps(x, il32, self.caps_inp_n, self.caps_inp_d, training, CNN_DROPOUT if drop else 0.0,
                               self.inp_dropout if drop else 0.0, seed, [self.P(k) for k in ops.CAPS_PARAMS],
                               self.proj_scale, self.caps_type == 'einsum')
        B, T2 = emb.shape[:2]
        p_mid = self.inn_dropout if drop else 0.0
        if self.is_context and self.enc_num > 1 and self.sdr_stack:
            # every SDR layer (and the LN + dropout between them) as one layer-pipelined
            # wavefront (ops.SdrStack); the head as below
            last = self.enc_num - 1
            params = [self.P(f'{w}{l}') for l in range(self.enc_num) for w in ('W', 'b')]
            params += [self.P(f'ln_mid{l + 1}_{t}') for l in range(last) for t in ('gamma', 'beta')]
            self._on_grad(emb, [f'{w}{l}' for l in range(self.enc_num) for w in ('W', 'b')]
                          + [f'ln_mid{l + 1}_{t}' for l in range(last) for t in ('gamma', 'beta')])
            plan = self._stack_plan(B, T2)
            # bucketed all-reduces overlapping the backward take CUs a grouped recurrence needs
            plan.collectives_overlap = self.grad_buckets is not None and self.grad_buckets.active()
            v = ops.sdr_stack(emb, plan, training, p_mid, seed, params)
            self._on_grad(v, [f'ln_mid{last + 1}_gamma', f'ln_mid{last + 1}_beta', 'ln_output_gamma',
                              'ln_output_beta'])
            return ops.CapsHead.apply(v, self.P(f'ln_mid{last + 1}_gamma'), self.P(f'ln_mid{last + 1}_beta'),
                                      self.P('ln_output_gamma'), self.P('ln_output_beta'), training, p_mid, seed,
                                      last, self.length_eps)
        for l in range(self.enc_num):
            route = ops.sequential_routing if self.is_context else ops.dynamic_routing
            W, bias = self._identity.get(l, (self.P(f'W{l}'), self.P(f'b{l}')))
            if l in self._identity and torch.is_grad_enabled():
                # lowmemory DR reads no W / bias: their gradients are zero, written here
                # so that "backward writes every gradient" holds for this variant too
                self.P(f'W{l}').grad.zero_()
                self.P(f'b{l}').grad.zero_()
            self._on_grad(emb, [f'W{l}', f'b{l}'])
            v = route(emb, W, bias, self._geom(l, B, T2))
            norms = [f'ln_mid{l + 1}_gamma', f'ln_mid{l + 1}_beta']
            self._on_grad(v, norms if l < self.enc_num - 1 else norms + ['ln_output_gamma', 'ln_output_beta'])
            if l < self.enc_num - 1:
                emb = ops.CapsNorm.apply(v, self.P(f'ln_mid{l + 1}_gamma'), self.P(f'ln_mid{l + 1}_beta'), training,
                                         p_mid, seed, l)
            else:
                return ops.CapsHead.apply(v, self.P(f'ln_mid{l + 1}_gamma'), self.P(f'ln_mid{l + 1}_beta'),
                                          self.P('ln_output_gamma'), self.P('ln_output_beta'), training, p_mid,
                                          seed, l, self.length_eps)
