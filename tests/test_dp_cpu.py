"""Data-parallel path on CPU (gloo, world_size 2): the per-rank loss scaling of
process_train_step (sum / (B_local * n_gpus), trainer_sr.py:58,67-68) followed by
allreduce_grads (SUM over the flat gradient buffer) must give every rank the
gradient of the global-batch mean, and identical parameters after the update."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from srf_amd import trainer_sr


class FlatModel:
    """Stand-in with the model's flat-buffer contract (flat_params/flat_grad)."""

    def __init__(self, n):
        g = torch.Generator().manual_seed(0)
        self.flat_params = torch.randn(n, generator=g)
        self.flat_grad = torch.zeros(n)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.manual_seed(100 + rank)
    B = 3 + rank                               # ragged local batches, as bucketing yields
    X = torch.randn(B, 5)
    model = FlatModel(5)
    w = model.flat_params.clone().requires_grad_()
    per_utt = (X @ w) ** 2
    loss = per_utt.sum() / float(B * world)    # compute_average_loss with global size B*world... per rank
    loss.backward()
    model.flat_grad.copy_(w.grad)
    trainer_sr.allreduce_grads(model)
    # plain numpy copies: a queued tensor travels as a shared-memory fd that the
    # parent must fetch from this process, which may already have exited
    q.put((rank, model.flat_grad.numpy().copy(), X.numpy().copy(), B))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_allreduce_gives_global_gradient():
    world = 2
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g0, g1 = torch.from_numpy(res[0][1]), torch.from_numpy(res[1][1])
    assert torch.allclose(g0, g1)
    # reference: each rank scales by its own B (the reference's semantics), summed
    w = FlatModel(5).flat_params.clone().requires_grad_()
    total = sum(((torch.from_numpy(X) @ w) ** 2).sum() / float(B * world) for _, _, X, B in res)
    total.backward()
    assert torch.allclose(g0, w.grad, atol=1e-6)


def _bn_worker(rank, world, port, ckdir, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from srf_amd import checkpoint as ck
    from tests.test_checkpoint_cpu import _model
    model = _model(0)
    with torch.no_grad():     # per-replica batch statistics drift apart
        model.bn0_moving_mean.fill_(1.0 + rank)
        model.bn1_moving_var.fill_(2.0 * (rank + 1))
    means = trainer_sr.replica_mean_moving_statistics(model)
    if rank == 0:
        ck.CheckpointManager(model, None, ckdir, max_to_keep=None).save(overrides=means)
    dist.barrier()
    q.put((rank, float(model.bn0_moving_mean[0]), float(means['bn0_moving_mean'][0]),
           float(means['bn1_moving_var'][0])))
    dist.destroy_process_group()


def test_gloo_checkpoint_holds_replica_mean_bn_statistics(tmp_path):
    """MirroredStrategy saves SyncOnRead(MEAN) BN moving statistics: the checkpoint
    holds the mean over ranks, each rank keeps its own local values."""
    from srf_amd import checkpoint as ck
    world = 2
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_bn_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [1.0, 2.0]                 # local values untouched
    assert all(r[2] == 1.5 and r[3] == 3.0 for r in res)     # mean over replicas
    st = ck.read_checkpoint(os.path.join(str(tmp_path), 'ckpt-1'))
    assert float(st['model/conv/bn_layers/0/moving_mean/' + ck.VALUE][0]) == 1.5
    assert float(st['model/conv/bn_layers/1/moving_variance/' + ck.VALUE][0]) == 3.0


class SpecModel:
    """Flat-buffer stand-in with the SequenceRouter layout fields GradBuckets reads."""

    def __init__(self, sizes, seed):
        self._spec = [(f'p{i}', (n,), None) for i, n in enumerate(sizes)]
        self.offsets, off = {}, 0
        for i, n in enumerate(sizes):
            self.offsets[f'p{i}'] = off
            off += (n + 63) // 64 * 64
        self.n_flat = off
        self.flat_grad = torch.randn(off, generator=torch.Generator().manual_seed(seed))


_SIZES = [700, 64, 5000, 33, 12000, 900, 4100, 10]


def _bucket_worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    m = SpecModel(_SIZES, seed=10 + rank)
    mine = m.flat_grad.clone()
    b = trainer_sr.GradBuckets(m, bucket_mb=3000 * 4 / 2 ** 20)
    # the backward's order: the last parameters first, in uneven groups
    names = [n for n, _, _ in m._spec][::-1]
    for grp in (names[:1], names[1:4], names[4:5], names[5:7]):
        b.ready(grp)
    b.finish()                      # the rest (the first parameter) and the waits
    q.put((rank, mine.numpy().copy(), m.flat_grad.numpy().copy(),
           [(lo, hi) for lo, hi, _ in b.buckets]))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_bucketed_allreduce_equals_flat():
    """GradBuckets over gloo (world 2): buckets tile the flat buffer from the end at
    parameter boundaries, and the bucketed result equals the flat SUM all-reduce."""
    import numpy as np
    world = 2
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total = res[0][1] + res[1][1]
    for _, _, got, buckets in res:
        np.testing.assert_allclose(got, total, rtol=1e-6, atol=1e-6)
        assert len(buckets) >= 3
        assert buckets[0][1] == len(total) and buckets[-1][0] == 0
        assert all(buckets[k + 1][1] == buckets[k][0] for k in range(len(buckets) - 1))


class _FakeGraphStep:
    """GraphedTrainStep stand-in: capture issues no collective (the real warm-up issues
    none since round 5), each replay one (the flat all-reduce or the captured buckets)."""
    log = None

    def __init__(self, in_len_div, inputs, model, optimizer, n_gpus, blank_idx, warmup=1, pool=None):
        self.model = model
        self.shape = (inputs[0].shape[0], int(inputs[2].max()))
        _FakeGraphStep.log.append('capture')

    def accepts(self, feats, labels, inp_len):
        return (feats.shape[0], int(inp_len.max())) == self.shape

    def refill(self, *a):
        pass

    def close(self):
        pass

    def __call__(self, *a):
        _FakeGraphStep.log.append('replay')
        dist.all_reduce(self.model.flat_grad)


def _cache_worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    log = []
    _FakeGraphStep.log = log

    def eager(in_len_div, inputs, model, *a):
        log.append('eager')
        dist.all_reduce(model.flat_grad)
    trainer_sr.GraphedTrainStep = _FakeGraphStep
    trainer_sr.process_train_step = eager
    model = FlatModel(4)
    cache = trainer_sr.GraphCache(4, model, None, world, 0, min_hits=2)
    # each rank crops its own batches: different crop lengths, seen at different steps
    lens = [[100, 100, 100, 120, 120, 100, 120], [90, 95, 90, 90, 95, 95, 90]][rank]
    for T in lens:
        cache.step((torch.zeros(3, T, 1), torch.zeros(3, 2), torch.tensor([T, T - 5, T - 9]), torch.zeros(3)))
    q.put((rank, log, cache.captures, cache.eager_steps))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_graph_cache_agrees_on_capture_steps():
    """GraphCache under data parallelism (world 2, gloo): ranks crop to different
    lengths, so a rank that has seen its shape twice would capture or replay while
    another still runs eagerly.  The cache agrees over the group: a step takes the
    graph path only when every rank can, so every rank issues one gradient collective
    per step in the same order (the run would hang otherwise) and captures only when
    all do."""
    world = 2
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_cache_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    paths = [[x for x in log if x != 'capture'] for _, log, _, _ in res]
    graph = [[x == 'replay' for x in p] for p in paths]
    assert len(paths[0]) == len(paths[1]) == 7 and graph[0] == graph[1]
    # step 1: rank 0's 100 is ready, rank 1's 95 is not -> both eager; step 2: both
    # ready (100, 90) -> both capture; step 3: rank 0 sees 120 first -> both eager,
    # though rank 1 holds a graph for 90; steps 4-6: graph on both
    assert graph[0] == [False, False, True, False, True, True, True]
    assert res[0][2] == res[1][2] == 2 and res[0][3] == res[1][3] == 3


class _Capture:
    def __init__(self, form, log):
        self.form, self.log = form, log
        self.closed = False
        log.append('capture ' + form)

    def close(self):
        self.closed = True
        self.log.append('close ' + self.form)


def _fallback_worker(rank, world, port, fail_rank, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    log = []

    def bucketed():
        if rank == fail_rank:
            raise RuntimeError('capture failed (forced)')
        return _Capture('bucketed', log)

    def flat():
        return _Capture('flat', log)
    g, err = trainer_sr.capture_agreed(bucketed, flat, dist.group.WORLD)
    # the form every rank replays must issue the same collective: one all-reduce per step
    # whose size tells the form (bucketed: 2 elements, flat: 1); a mismatch would hang
    t = torch.ones(2 if g.form == 'bucketed' else 1)
    work = dist.all_reduce(t, async_op=True)
    work.wait(timeout=__import__('datetime').timedelta(seconds=30))
    q.put((rank, g.form, err is not None, log, float(t.sum())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('fail_rank', [1, -1])
def test_gloo_capture_fallback_is_collective(fail_rank):
    """bench.py's capture of the bucketed step (world 2, gloo): when one rank's capture
    fails, EVERY rank falls back to the flat all-reduce (a rank whose capture succeeded
    closes it), so both replay the same collective form; when none fails, both keep the
    captured buckets."""
    world = 2
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_fallback_worker, args=(r, world, port, fail_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    forms = [r[1] for r in res]
    if fail_rank < 0:
        assert forms == ['bucketed', 'bucketed'] and not any(r[2] for r in res)
        assert all(r[4] == 4.0 for r in res)
    else:
        assert forms == ['flat', 'flat'] and all(r[2] for r in res)
        assert res[1 - fail_rank][3] == ['capture bucketed', 'close bucketed', 'capture flat']
        assert res[fail_rank][3] == ['capture flat']
        assert all(r[4] == 2.0 for r in res)
