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

from . import ctc, ops


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


def reduce_metrics(*metrics):
    """Cross-replica read of Mean / Sum metrics: the reference's metrics are
    sync-on-read variables that every replica updates, and its log line
    (trainer_sr.py:218-221) and epoch-end early-stop check (:263-279) read them
    across replicas.  One SUM all-reduce of (total, count) per metric; every rank
    calls it and gets the same values.  The metrics themselves are left alone."""
    if _world() <= 1:
        return [m.result() for m in metrics]
    dev = torch.device('cuda', torch.cuda.current_device()) if dist.get_backend() == 'nccl' else 'cpu'
    t = torch.tensor([[m._total(), float(m.count)] for m in metrics], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    t = t.cpu()
    return [float(tot) if isinstance(m, Sum) else (float(tot) / float(cnt) if cnt else 0.0)
            for m, (tot, cnt) in zip(metrics, t.tolist())]


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
    """The flat form: one SUM all-reduce of the whole gradient after the backward."""
    if _world() > 1:
        dist.all_reduce(model.flat_grad, op=dist.ReduceOp.SUM)
        agree_faults(model)


def agree_faults(model):
    """MAX all-reduce of the process's fault word (ops.fault_flag) after the gradient
    collectives, on the stream the optimizer runs on.  A grouped SDR recurrence that
    timed out on one rank made every rank's summed gradient wrong: with the word
    agreed, every rank's Adam launch skips the update (adam.hip reads the word) and
    every rank's ops.check_faults raises at the same step, so no rank is left waiting
    in a collective its peers never join.  Only models with SDR layers have the word
    (the SdrStack forward registers it on every rank before the first step)."""
    if _world() <= 1 or not model.flat_grad.is_cuda or not getattr(model, 'is_context', False):
        return
    dist.all_reduce(ops.fault_flag(model.flat_grad.device), op=dist.ReduceOp.MAX)


class GradBuckets:
    """Bucketed gradient all-reduce overlapped with the backward: the
    reference's implicit all-reduce inside apply_gradients (trainer_sr.py:71,213)
    issued in pieces as the top-down backward completes them.

    The model's parameters are views into one flat buffer in constructor order
    (CNN front end, primary capsules, routing layers 0..L-1, output head), and the
    backward writes them in the reverse order, so a bucket is a contiguous range of
    flat_grad cut at parameter boundaries from the end, >= ``bucket_mb`` each.  The
    model calls ``ready(names)`` from tensor hooks once the backward kernels of those
    parameters are enqueued (SequenceRouter.grad_hook); a bucket whose parameters are
    all ready is all-reduced asynchronously (RCCL orders it after the kernels already
    on the stream, then runs it beside the rest of the backward).  Buckets launch in
    index order on every rank, so the collectives match.  ``finish()`` launches what
    is left (the CNN front end's parameters, whose backward is last) and makes the
    current stream wait for every bucket.

    ``force`` runs the collectives at world size 1 too (the RCCL path test).

    On the GPU a ready bucket records an event on the backward's stream and its
    collective is issued at the next hook (from a side stream that waits on the
    event), i.e. after more of the backward has been enqueued: in a captured step the
    backward's next kernel then precedes the collective in capture order, which keeps
    the backward one chain of ROCm's graph executor instead of a new chain per bucket
    that may share a hardware queue with the collectives (ops.STACK_CAPTURE_ORDER)."""

    def __init__(self, model, bucket_mb=25.0, force=False):
        self.model, self.force = model, force
        names = [name for name, _, _ in model._spec]
        limit = max(1, int(bucket_mb * 2 ** 20 / 4))
        self.buckets = []      # (lo, hi, parameter names), in backward order
        hi, cur = model.n_flat, []
        for i in reversed(range(len(names))):
            cur.append(names[i])
            lo = model.offsets[names[i]]
            if hi - lo >= limit or i == 0:
                self.buckets.append((lo, hi, cur))
                hi, cur = lo, []
        self.of = {n: k for k, (_, _, ns) in enumerate(self.buckets) for n in ns}
        dev = model.flat_grad.device
        self.gpu = dev.type == 'cuda'
        # created once: a captured step must not see its events destroyed before capture ends
        self.events = [torch.cuda.Event() for _ in self.buckets] if self.gpu else None
        self.side = torch.cuda.Stream(device=dev) if self.gpu else None
        self.begin()
        if self.active() and dist.is_initialized() and dist.get_backend() == 'nccl':
            # every rank constructs the buckets at the same point: one collective now sets
            # up the communicator, so that no rank's first collective is a captured one
            dist.all_reduce(torch.zeros(1, device=model.flat_grad.device), op=dist.ReduceOp.SUM)

    def active(self):
        return self.force or _world() > 1

    def begin(self):
        self.pending = [set(ns) for _, _, ns in self.buckets]
        self.launched = 0
        self.works = []
        self.deferred = []   # ready buckets whose collective is not issued yet

    def ready(self, names):
        self._issue()
        for n in names:
            self.pending[self.of[n]].discard(n)
        while self.launched < len(self.buckets) and not self.pending[self.launched]:
            self._launch()

    def _launch(self):
        k = self.launched
        self.launched += 1
        if not self.active():
            return
        if self.gpu:
            self.events[k].record()   # the bucket's gradients are enqueued on the current stream
        self.deferred.append(k)
        if not self.gpu:
            self._issue()

    def _issue(self):
        if self.gpu and self.deferred:
            # DR gW / gbias deferred onto their side stream (ops.DR_GW_SIDE) write gradients
            # of these buckets: issue them, and order the collectives after them
            ops._dr_issue_pending()
            dr = ops._dr_side.get(self.model.flat_grad.device.index)
            if dr is not None:
                self.side.wait_stream(dr)
        for k in self.deferred:
            lo, hi, _ = self.buckets[k]
            if self.gpu:
                self.side.wait_event(self.events[k])
                with torch.cuda.stream(self.side):
                    self.works.append(dist.all_reduce(self.model.flat_grad[lo:hi], op=dist.ReduceOp.SUM,
                                                      async_op=True))
            else:
                self.works.append(dist.all_reduce(self.model.flat_grad[lo:hi], op=dist.ReduceOp.SUM, async_op=True))
        self.deferred = []

    def finish(self):
        while self.launched < len(self.buckets):
            self._launch()
        self._issue()
        for w in self.works:
            w.wait()
        if self.gpu and self.works:
            torch.cuda.current_stream().wait_stream(self.side)
        if self.works:
            agree_faults(self.model)
        self.begin()


def _reduce(model):
    b = getattr(model, 'grad_buckets', None)
    if b is not None:
        b.finish()
    else:
        allreduce_grads(model)


def use_grad_buckets(model, bucket_mb=25.0, force=False):
    """Switch ``model`` to the bucketed, backward-overlapped all-reduce (GradBuckets);
    returns the buckets.  ``None`` as bucket_mb restores the flat form."""
    if bucket_mb is None:
        model.grad_buckets = None
        model.grad_hook = None
        return None
    b = GradBuckets(model, bucket_mb, force)
    model.grad_buckets = b
    model.grad_hook = b.ready
    return b


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
    b = getattr(model, 'grad_buckets', None)
    if b is not None:
        b.begin()
    y_pred = model(feats, input_lengths=inp_len, training=True)
    # loss = sum(nll) / (B * n_gpus): its logit gradient comes out of the CTC launch
    # already scaled, and seeds the backward directly (no scalar autograd ops)
    pe_loss, g_logits = ctc.ctc_loss_and_grad(labels, y_pred, tar_len, ceil_div(inp_len, in_len_div), blank_idx,
                                              1.0 / float(batch * n_gpus))
    y_pred.backward(g_logits)
    ops.dr_side_join()   # DR gW launches deferred onto a side stream (ops.DR_GW_SIDE)
    _reduce(model)
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

    def __init__(self, in_len_div, inputs, model, optimizer, n_gpus, blank_idx, warmup=2, label_capacity=None,
                 pool=None):
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
        # bucketed all-reduce inside the graph (RCCL collectives captured with the
        # backward they overlap) when the model asks for buckets on an nccl group;
        # otherwise one flat all-reduce after each replay
        b = getattr(model, 'grad_buckets', None)
        self.buckets = b if (b is not None and b.active() and dist.is_initialized()
                             and dist.get_backend() == 'nccl') else None
        hook = getattr(model, 'grad_hook', None)
        # the warm-up steps run the training forward, which updates the BatchNorm moving
        # statistics: restore them, so that building a graph changes no model state.
        # They issue no collectives: only this rank may be building a graph at this step
        # (GraphCache agrees on capture steps, but a direct caller need not), and the
        # captured collectives do not execute until the replay, which every rank joins
        buffers = [b_.clone() for b_ in model.buffers()]
        try:
            model.grad_hook = None
            side = torch.cuda.Stream(device=dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(warmup):
                    self._fwd_bwd(collectives=False)
            torch.cuda.current_stream(dev).wait_stream(side)
            if self.buckets is not None:
                model.grad_hook = hook
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, pool=pool):
                self.nll = self._fwd_bwd()
        except BaseException:
            ops.dr_reset()   # deferred side-stream launches of the failed backward are void
            if self.buckets is not None:
                self.buckets.begin()
            raise
        finally:
            model.grad_hook = hook
        with torch.no_grad():
            for b_, saved in zip(model.buffers(), buffers):
                b_.copy_(saved)

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

    def _fwd_bwd(self, collectives=True):
        self.counter.add_(1)
        buckets = self.buckets if collectives else None
        if buckets is not None:
            buckets.begin()
        y_pred = self.model(self.feats, input_lengths=self.inp_len, training=True)
        logit_len = ceil_div(self.inp_len, self.in_len_div)
        pe_loss, g_logits = ctc.ctc_loss_and_grad(self.labels, y_pred, self.tar_len, logit_len, self.blank_idx,
                                                  1.0 / float(self.batch * self.n_gpus))
        y_pred.backward(g_logits)
        ops.dr_side_join()
        if buckets is not None:
            buckets.finish()
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
        # the per-utterance NLL lives in the graph's memory pool, which graphs of a
        # GraphCache share: hand out a copy a later replay cannot overwrite
        nll = self.nll.clone()
        if self.buckets is None:
            allreduce_grads(self.model)
        self.optimizer.apply_gradients(self.model)
        if loss_state is not None:
            loss_state.update_state(nll)
        if frame_state is not None:
            frame_state.update_state(self.host_len.sum())
        if samples is not None:
            samples.update_state(self.batch)
        return nll


def capture_agreed(capture, fallback, group=None):
    """``capture()`` on every rank, falling back to ``fallback()`` on EVERY rank when
    any rank's capture raised RuntimeError (one int MIN all-reduce over ``group``, a
    CPU gloo group, after the attempt).  A rank-local fallback would leave one rank
    replaying captured bucket collectives while another issues a flat all-reduce:
    the collective sequences would differ and the job hang.  Returns (result, error)
    with error the local exception, or a note that a peer failed, when the fallback
    ran; a capture that succeeded here but not on a peer is closed."""
    err = None
    try:
        g = capture()
    except RuntimeError as e:
        g, err = None, e
    ok = err is None
    if group is not None:
        t = torch.tensor([int(ok)], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
        ok = bool(t.item())
    if ok:
        return g, None
    if g is not None:
        close = getattr(g, 'close', None)
        if close is not None:
            close()
        err = RuntimeError('the capture failed on another rank')
    return fallback(), err


class GraphCache:
    """Captured training steps per batch shape (B, T), least recently used evicted
    past ``max_graphs``.

    The key is the exact shape: process_train_step crops each batch to its longest
    utterance (trainer_sr.py:59-60), and padding a batch further would change its
    results -- the BatchNorm batch statistics count the masked padded positions
    (sequence_router.py:78-80) and the routing window reads padded frames into valid
    ones (naive:150-151).  Bucketed data (load_speech_data.create_ds_bucket) gives a
    bounded number of batch sizes but many crop lengths, so a shape is captured only
    once it has been seen ``min_hits`` times; until then its steps run eagerly
    (process_train_step), which costs no more than an uncaptured step.  All graphs
    share one memory pool (they never run concurrently), so the cache holds one
    step's worth of activations, not one per shape.  A new label length beyond a
    cached graph's capacity re-captures that shape with a larger one.

    Under data parallelism each rank crops its own batch, so the ranks see different
    shapes.  Whether a step replays or captures a graph, or runs eagerly, is agreed
    over the process group (one int MIN all-reduce per step on a CPU gloo group): a
    step takes the graph path only when every rank can, so every rank issues the same
    gradient collectives in the same order (from its replay or its eager backward) and
    captures only when all do."""

    def __init__(self, in_len_div, model, optimizer, n_gpus, blank_idx, max_graphs=32, warmup=1, min_hits=2):
        self.args = (in_len_div, model, optimizer, n_gpus, blank_idx)
        self.max_graphs, self.warmup, self.min_hits = max_graphs, warmup, max(1, int(min_hits))
        self.graphs = OrderedDict()
        self.seen = OrderedDict()    # shape -> times seen, bounded like the graphs
        self.captures = 0
        self.eager_steps = 0
        self.pool = None
        self.flag_group = None
        if _world() > 1:   # every rank constructs the cache at the same point
            self.flag_group = dist.group.WORLD if dist.get_backend() == 'gloo' else dist.new_group(backend='gloo')

    def agree(self, want):
        """True when every rank of the group wants the graph path this step."""
        if self.flag_group is None:
            return want
        t = torch.tensor([int(bool(want))], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.flag_group)
        return bool(t.item())

    def step(self, inputs, loss_state=None, frame_state=None, samples=None):
        feats, labels, inp_len, tar_len = inputs
        key = (feats.shape[0], int(torch.as_tensor(inp_len).max()))
        in_len_div, model, optimizer, n_gpus, blank_idx = self.args
        g = self.graphs.get(key)
        if g is not None and not g.accepts(feats, labels, inp_len):
            g.close()
            del self.graphs[key]
            g = None
        want = True
        if g is None:
            hits = self.seen.pop(key, 0) + 1
            self.seen[key] = hits
            while len(self.seen) > 4 * self.max_graphs:
                self.seen.popitem(last=False)
            want = hits >= self.min_hits
        if not self.agree(want):
            self.eager_steps += 1
            return process_train_step(in_len_div, inputs, model, optimizer, loss_state, frame_state, n_gpus,
                                      blank_idx, samples)
        if g is None:
            if self.pool is None:
                self.pool = torch.cuda.graph_pool_handle()
            g = GraphedTrainStep(in_len_div, inputs, model, optimizer, n_gpus, blank_idx, warmup=self.warmup,
                                 pool=self.pool)
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
        if index % 50 == 0 and index > 0 and samples is not None and loss_state is not None:
            # every rank joins the cross-replica read, logging or not (:218-221)
            n_samples, loss = reduce_metrics(samples, loss_state)
            _check_faults(dev)
            if log is not None:
                prog = n_samples / train_num * 100 if train_num else float('nan')
                log('STEP', optimizer.iterations, prog, loss, optimizer.current_lr())
        index += 1
    _check_faults(dev)
    return index


def _check_faults(dev):
    """Fail the run if a grouped SDR recurrence timed out since the last check
    (ops.check_faults; a device read, so only at points that synchronise anyway)."""
    if torch.device(dev).type == 'cuda':
        from . import ops
        ops.check_faults()


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
