"""Step functions and driver of tfsr/trainer_sr.py, one process per GPU.

``process_train_step`` / ``process_valid_step`` / ``process_test_step`` keep the
reference's argument lists (trainer_sr.py:41-117).  Data parallelism replaces
tf.distribute.MirroredStrategy (trainer_sr.py:139) with one process per GPU
(torchrun); the implicit NCCL all-reduce inside ``apply_gradients`` becomes one
explicit RCCL all-reduce (SUM) of the model's flat gradient buffer -- with the
loss scaled by 1/(B_local * n_gpus) as in trainer_sr.py:58,67-68 the sum is the
global-batch mean.
"""
import torch
import torch.distributed as dist

from . import ctc


class Mean:
    """tf.keras.metrics.Mean (trainer_sr.py:161-163).  Device tensors are summed on
    their device (no host synchronisation per step); result() reads the total."""

    def __init__(self, name=''):
        self.name = name
        self.reset_states()

    def reset_states(self):
        self.total = 0.0
        self.count = 0

    def update_state(self, values):
        if torch.is_tensor(values):
            v = values.detach()
            self.total = self.total + v.sum(dtype=torch.float64)
            self.count += v.numel()
        else:
            v = torch.as_tensor(values, dtype=torch.float64).reshape(-1)
            self.total = self.total + float(v.sum())
            self.count += v.numel()

    def _total(self):
        return float(self.total) if torch.is_tensor(self.total) else self.total

    def result(self):
        return self._total() / self.count if self.count else 0.0


class Sum(Mean):
    """tf.keras.metrics.Sum (trainer_sr.py:164)."""

    def result(self):
        return self._total()


def _crop(feats, inp_len):
    """trainer_sr.py:59-60: crop the padded batch to the longest utterance.  With
    host-resident lengths (what the data pipeline yields) this needs no device sync."""
    T = int(inp_len.max())
    return feats if T == feats.shape[1] else feats[:, :T, :].contiguous()


def ceil_div(inp_len, div):
    return torch.div(inp_len + (div - 1), div, rounding_mode='floor').to(torch.int32)


def _world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def allreduce_grads(model):
    if _world() > 1:
        dist.all_reduce(model.flat_grad, op=dist.ReduceOp.SUM)


def replica_mean_moving_statistics(model):
    """BatchNorm moving statistics as a MirroredStrategy checkpoint holds them.

    Batch statistics stay per replica (Keras BN is not SyncBN), so each rank's
    moving mean / variance drift apart.  Under MirroredStrategy they are SyncOnRead
    variables with MEAN aggregation: a replica reads its own value (validation runs
    inside strategy.run, trainer_sr.py:224-228), while a cross-replica read -- the
    checkpoint save (trainer_sr.py:281-288) -- sees the mean over replicas.  Every
    rank calls this (one all-reduce of 4*64 floats); it returns {buffer name: mean}
    for CheckpointManager.save(overrides=...) and leaves the local buffers alone."""
    names = [f'bn{k}_moving_{s}' for k in range(model.cnn_n) for s in ('mean', 'var')]
    bufs = [getattr(model, n) for n in names]
    flat = torch.cat([b.detach().reshape(-1) for b in bufs])
    if _world() > 1:
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
        flat /= _world()
    out, off = {}, 0
    for n, b in zip(names, bufs):
        out[n] = flat[off:off + b.numel()].view_as(b)
        off += b.numel()
    return out


def process_train_step(in_len_div, inputs, model, optimizer, loss_state, frame_state, n_gpus, blank_idx, samples):
    """trainer_sr.py:41-75."""
    feats, labels, inp_len, tar_len = inputs
    batch = feats.shape[0]
    feats = _crop(feats, inp_len)
    host_len = inp_len
    inp_len = inp_len.to(feats.device, non_blocking=True)
    y_pred = model(feats, input_lengths=inp_len, training=True)
    # loss = sum(nll) / (B * n_gpus): its logit gradient comes out of the CTC launch
    # already scaled, and seeds the backward directly (no scalar autograd ops)
    pe_loss, g_logits = ctc.ctc_loss_and_grad(labels, y_pred, tar_len, ceil_div(inp_len, in_len_div), blank_idx,
                                              1.0 / float(batch * n_gpus))
    y_pred.backward(g_logits)
    allreduce_grads(model)
    optimizer.apply_gradients(model)
    if loss_state is not None:
        loss_state.update_state(pe_loss)
    if frame_state is not None:
        frame_state.update_state(host_len.sum())
    if samples is not None:
        samples.update_state(batch)
    return pe_loss


class GraphedTrainStep:
    """process_train_step with its forward, CTC loss head and backward captured
    into one hipGraph (torch.cuda.CUDAGraph) for a fixed batch shape; the gradient
    all-reduce, the Adam update and the metrics run eagerly after each replay.

    The ~110 kernel launches of a step then cost one graph launch on the host, so
    the step is bound by the GPU, not by Python/ctypes launch overhead (which
    grows when several ranks share a host).  Dropout stays random per step: the
    captured step first advances a device-resident step counter that every dropout
    kernel mixes into its seed (srf_set_seed_source).

    The graph reads the static tensors ``self.feats`` (cropped to max(inp_len),
    which may be a private copy of the caller's feats), ``self.labels``,
    ``self.inp_len`` (device copy) and ``self.tar_len``, not the caller's
    ``inputs``.  Feed a new batch of the same shape and lengths with
    ``refill(...)``, which copies into those tensors and refuses any other shape
    or lengths.
    """

    def __init__(self, in_len_div, inputs, model, optimizer, n_gpus, blank_idx, warmup=2):
        from . import _lib
        self.model, self.optimizer = model, optimizer
        self.in_len_div, self.n_gpus, self.blank_idx = in_len_div, n_gpus, blank_idx
        feats, labels, inp_len, tar_len = inputs
        dev = feats.device
        self.batch = feats.shape[0]
        self.host_len = inp_len
        self.feats = _crop(feats, inp_len)
        self.labels, self.tar_len = labels, tar_len
        self.inp_len = inp_len.to(dev)
        self.logit_len = ceil_div(self.inp_len, in_len_div)
        self.counter = torch.zeros(1, dtype=torch.int64, device=dev)
        rc = _lib.lib().srf_set_seed_source(self.counter.data_ptr())
        _lib.check(rc, 'srf_set_seed_source')
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._fwd_bwd()
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.nll = self._fwd_bwd()

    def refill(self, feats, labels, inp_len, tar_len):
        """Copy a new batch into the tensors the captured graph reads."""
        if not torch.equal(torch.as_tensor(inp_len).cpu().to(torch.int64),
                           torch.as_tensor(self.host_len).cpu().to(torch.int64)):
            raise ValueError('GraphedTrainStep.refill: input lengths differ from the captured batch')
        feats = feats[:, :self.feats.shape[1], :]
        for dst, src, what in ((self.feats, feats, 'feats'), (self.labels, labels, 'labels'),
                               (self.tar_len, tar_len, 'tar_len')):
            if tuple(src.shape) != tuple(dst.shape):
                raise ValueError(f'GraphedTrainStep.refill: {what} shape {tuple(src.shape)} != {tuple(dst.shape)}')
            dst.copy_(src, non_blocking=True)

    def _fwd_bwd(self):
        self.counter.add_(1)
        y_pred = self.model(self.feats, input_lengths=self.inp_len, training=True)
        pe_loss, g_logits = ctc.ctc_loss_and_grad(self.labels, y_pred, self.tar_len, self.logit_len, self.blank_idx,
                                                  1.0 / float(self.batch * self.n_gpus))
        y_pred.backward(g_logits)
        return pe_loss

    def close(self):
        """Detach the dropout kernels from this step's counter (before it is freed)."""
        from . import _lib
        if getattr(self, 'counter', None) is not None:
            _lib.lib().srf_set_seed_source(None)
            self.counter = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __call__(self, loss_state=None, frame_state=None, samples=None):
        self.graph.replay()
        allreduce_grads(self.model)
        self.optimizer.apply_gradients(self.model)
        if loss_state is not None:
            loss_state.update_state(self.nll)
        if frame_state is not None:
            frame_state.update_state(self.host_len.sum())
        if samples is not None:
            samples.update_state(self.batch)
        return self.nll


@torch.no_grad()
def process_valid_step(in_len_div, inputs, model, loss_state, blank_idx):
    """trainer_sr.py:77-94."""
    feats, labels, inp_len, tar_len = inputs
    feats = _crop(feats, inp_len)
    y_pred = model(feats, input_lengths=inp_len, training=False)
    pe_loss = ctc.ctc_loss(labels, y_pred, tar_len, ceil_div(inp_len, in_len_div), blank_index=blank_idx)
    if loss_state is not None:
        loss_state.update_state(pe_loss)
    return pe_loss


@torch.no_grad()
def process_test_step(in_len_div, inputs, model, beam_width=None):
    """trainer_sr.py:96-117: forward, then tf.nn.ctc_beam_search_decoder(beam_width,
    top_paths=1) on the host (srf_amd.ctc.beam_search_decode); best-path decoding
    when no beam width is configured.  Decode lengths use floor division, as the
    reference does (:110)."""
    feats, _, inp_len, _, utt_id = inputs
    feats = _crop(feats, inp_len)
    y_pred = model(feats, input_lengths=inp_len, training=False)
    lens = inp_len.to(torch.int64) // in_len_div
    if beam_width:
        hyps, _ = ctc.beam_search_decode(y_pred, lens, y_pred.shape[-1] - 1, beam_width)
    else:
        hyps = ctc.greedy_decode(y_pred, lens, y_pred.shape[-1] - 1)
    for u, h in zip(utt_id, hyps):
        print('UTTID:', u)
        print(h)
    return hyps
