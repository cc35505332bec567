"""Step functions and driver of tfsr/trainer_sr.py, one process per GPU.

``process_train_step`` / ``process_valid_step`` / ``process_test_step`` keep the
reference's argument lists (trainer_sr.py:41-117).  Data parallelism replaces
tf.distribute.MirroredStrategy (trainer_sr.py:139) with one process per GPU
(torchrun); the implicit NCCL all-reduce inside ``apply_gradients`` becomes one
explicit RCCL all-reduce (SUM) of the model's flat gradient buffer -- with the
loss scaled by 1/(B_local * n_gpus) as in trainer_sr.py:58,67-68 the sum is the
global-batch mean.
"""
from collections import OrderedDict

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


_SEED_COUNTERS = {}


def seed_counter(dev):
    """The process's device-resident dropout step counter on ``dev`` (one per
    process, created once and never released: srf_set_seed_source is process-wide).
    Every captured training step advances it, so graph replays draw fresh masks;
    eager steps leave it alone and differ through their per-call seeds."""
    dev = torch.device(dev)
    c = _SEED_COUNTERS.get(dev)
    if c is None:
        from . import _lib
        if _SEED_COUNTERS:
            raise RuntimeError('one process drives one GPU: the dropout step counter already lives on '
                               f'{next(iter(_SEED_COUNTERS))}')
        c = torch.zeros(1, dtype=torch.int64, device=dev)
        _lib.check(_lib.lib().srf_set_seed_source(c.data_ptr()), 'srf_set_seed_source')
        _SEED_COUNTERS[dev] = c
    return c


def _label_capacity(L):
    return max(8, -(-int(L) // 8) * 8)


class GraphedTrainStep:
    """process_train_step with its forward, CTC loss head and backward captured
    into one hipGraph (torch.cuda.CUDAGraph) for one batch shape (B utterances
    cropped to T frames); the gradient all-reduce, the Adam update and the
    metrics run eagerly after each replay.

    The ~110 kernel launches of a step then cost one graph launch on the host, so
    the step is bound by the GPU, not by Python/ctypes launch overhead (which
    grows when several ranks share a host).  Dropout stays random per step: the
    captured step first advances the process's device step counter
    (seed_counter), which every dropout kernel mixes into its seed.

    Every per-batch quantity the kernels read is device-resident: ``self.feats``
    [B, T, F], ``self.labels`` [B, label_capacity] (zero-padded past tar_len),
    ``self.inp_len`` / ``self.tar_len`` [B] int32; the logit lengths
    ceil(inp_len / 4) are computed inside the graph.  ``refill(...)`` copies any
    batch of the same B and T (max(inp_len) == T, trainer_sr.py:59-60) with at most
    label_capacity labels into them; utterance lengths and label lengths may differ
    from the captured batch.
    """

    def __init__(self, in_len_div, inputs, model, optimizer, n_gpus, blank_idx, warmup=2, label_capacity=None):
        self.model, self.optimizer = model, optimizer
        self.in_len_div, self.n_gpus, self.blank_idx = in_len_div, n_gpus, blank_idx
        feats, labels, inp_len, tar_len = inputs
        dev = feats.device
        self.batch = feats.shape[0]
        host_len = torch.as_tensor(inp_len)
        self.T = int(host_len.max())
        self.host_len = host_len.cpu()
        self.label_capacity = _label_capacity(labels.shape[1] if label_capacity is None else label_capacity)
        self.feats = torch.zeros((self.batch, self.T, feats.shape[2]), dtype=torch.float32, device=dev)
        self.labels = torch.zeros((self.batch, self.label_capacity), dtype=torch.int32, device=dev)
        self.inp_len = torch.zeros(self.batch, dtype=torch.int32, device=dev)
        self.tar_len = torch.zeros(self.batch, dtype=torch.int32, device=dev)
        self.refill(feats, labels, inp_len, tar_len)
        self.counter = seed_counter(dev)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._fwd_bwd()
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.nll = self._fwd_bwd()

    def accepts(self, feats, labels, inp_len):
        return (feats.shape[0] == self.batch and int(torch.as_tensor(inp_len).max()) == self.T
                and labels.shape[1] <= self.label_capacity)

    def refill(self, feats, labels, inp_len, tar_len):
        """Copy a new batch into the tensors the captured graph reads."""
        host_len = torch.as_tensor(inp_len)
        if feats.shape[0] != self.batch or int(host_len.max()) != self.T:
            raise ValueError(f'GraphedTrainStep.refill: batch of {feats.shape[0]} utterances cropped to '
                             f'{int(host_len.max())} frames, the graph runs {self.batch} x {self.T}')
        if labels.shape[1] > self.label_capacity:
            raise ValueError(f'GraphedTrainStep.refill: {labels.shape[1]} labels exceed the capacity '
                             f'{self.label_capacity}')
        self.host_len = host_len.cpu()
        self.feats.copy_(torch.as_tensor(feats)[:, :self.T, :], non_blocking=True)
        self.labels[:, labels.shape[1]:].zero_()
        self.labels[:, :labels.shape[1]].copy_(torch.as_tensor(labels), non_blocking=True)
        self.inp_len.copy_(host_len, non_blocking=True)
        self.tar_len.copy_(torch.as_tensor(tar_len), non_blocking=True)

    def _fwd_bwd(self):
        self.counter.add_(1)
        y_pred = self.model(self.feats, input_lengths=self.inp_len, training=True)
        logit_len = ceil_div(self.inp_len, self.in_len_div)
        pe_loss, g_logits = ctc.ctc_loss_and_grad(self.labels, y_pred, self.tar_len, logit_len, self.blank_idx,
                                                  1.0 / float(self.batch * self.n_gpus))
        y_pred.backward(g_logits)
        return pe_loss

    @property
    def logit_len(self):
        return ceil_div(self.inp_len, self.in_len_div)

    def close(self):
        """Release the graph (its private memory pool goes with it).  The process's
        step counter stays attached: other graphs and models keep using it."""
        self.graph = None

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


class GraphCache:
    """One GraphedTrainStep per batch shape (B, T), least recently used evicted
    past ``max_graphs``.  Bucketed batches (load_speech_data.create_ds_bucket) come
    in a bounded set of shapes; a new label length beyond a cached graph's capacity
    re-captures that shape with a larger one."""

    def __init__(self, in_len_div, model, optimizer, n_gpus, blank_idx, max_graphs=32, warmup=1):
        self.args = (in_len_div, model, optimizer, n_gpus, blank_idx)
        self.max_graphs, self.warmup = max_graphs, warmup
        self.graphs = OrderedDict()
        self.captures = 0

    def step(self, inputs, loss_state=None, frame_state=None, samples=None):
        feats, labels, inp_len, tar_len = inputs
        key = (feats.shape[0], int(torch.as_tensor(inp_len).max()))
        g = self.graphs.get(key)
        if g is not None and not g.accepts(feats, labels, inp_len):
            g.close()
            del self.graphs[key]
            g = None
        if g is None:
            in_len_div, model, optimizer, n_gpus, blank_idx = self.args
            g = GraphedTrainStep(in_len_div, inputs, model, optimizer, n_gpus, blank_idx, warmup=self.warmup)
            self.captures += 1
            self.graphs[key] = g
            while len(self.graphs) > self.max_graphs:
                _, old = self.graphs.popitem(last=False)
                old.close()
        else:
            g.refill(feats, labels, inp_len, tar_len)
            self.graphs.move_to_end(key)
        return g(loss_state, frame_state, samples)


def batch_to_device(batch, dev):
    """A dataset batch (numpy: feats [B,T,F] f32, labels [B,L], inp_len [B],
    tar_len [B]) as process_train_step takes it: feats / labels / tar_len on the
    device, inp_len host-resident (the crop needs no device sync)."""
    feats, labels, inp_len, tar_len = batch[:4]
    pin = torch.device(dev).type == 'cuda'

    def dev_t(a, dtype):
        t = torch.as_tensor(a).to(dtype)
        return (t.pin_memory() if pin else t).to(dev, non_blocking=True)
    return (dev_t(feats, torch.float32), dev_t(labels, torch.int32), torch.as_tensor(inp_len).to(torch.int32),
            dev_t(tar_len, torch.int32))


def distributed_train_step(dataset, in_len_div, model, optimizer, loss_state, frame_state, n_gpus, blank_idx,
                           samples, train_num=None, graphs=None, log=print):
    """trainer_sr.py:205-222 (the hot loop): every batch of this replica's
    dataset (data_helper.create_ds_for_training(..., rank, world)) through one
    training step, with the reference's progress line every 50 steps.  ``graphs``
    (a GraphCache) replays a captured step per batch shape; None runs
    process_train_step eagerly."""
    dev = model.flat_params.device
    index = 0
    if log is not None:
        log('Step, Progress%, Average Loss, lr')
    for example in dataset:
        inputs = batch_to_device(example, dev)
        if graphs is None:
            process_train_step(in_len_div, inputs, model, optimizer, loss_state, frame_state, n_gpus, blank_idx,
                               samples)
        else:
            graphs.step(inputs, loss_state, frame_state, samples)
        if index % 50 == 0 and index > 0 and log is not None:
            prog = samples.result() / train_num * 100 if train_num else float('nan')
            log('STEP', optimizer.iterations, prog, loss_state.result(), optimizer.current_lr())
        index += 1
    return index


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
