"""Training-loop pieces on the GPU: the fused Adam against the oracle's Keras Adam,
and the captured step serving real bucketed TFRecord batches.

* Adam (train_helper.py:32-70, the Keras apply at trainer_sr.py:71): five
  apply_gradients of srf_adam_step against oracle/naive_mirror.TfAdam from the
  same gradients, through lr(0) = 0, the warm-up ramp and the train_lr_max cap;
  parameters, m and v within fp32 rounding (|err| <= 4e-6 * (1 + |ref|): 1 - beta_2
  alone rounds to fp32 with a 1e-6 relative error, as in Keras' fp32 Adam).
* Graphed steps over data (trainer_sr.py:205-222): a small TFRecord corpus
  bucketed by length into three batch sizes (two batches share one (B, T) shape
  with different lengths, so the cached graph is refilled), each batch's gradient
  from GraphCache equal to the eager process_train_step's
  (|err| <= 1e-4 * max|g|), and distributed_train_step over the same dataset; the
  BatchNorm moving statistics equal the eager model's after both (graph building
  must not update them).
"""
import numpy as np
import pytest
import torch

from tests.helpers import config_from_shape, load_model_fixture

pytestmark = pytest.mark.gpu


class _Flat:
    def __init__(self, p, dev):
        self.flat_params = torch.tensor(p, dtype=torch.float32, device=dev)
        self.flat_grad = torch.zeros_like(self.flat_params)
        self.n_flat = self.flat_params.numel()


@pytest.mark.parametrize('k,warmup,max_lr', [(0.5, 1200, 1e3),     # warm-up ramp (TIMIT script values)
                                             (100.0, 2, 1e-2),     # capped at train_lr_max from step 1
                                             (2.0, 3, 0.5)])       # ramp, then the s^-1/2 decay
def test_adam_matches_oracle(cuda, k, warmup, max_lr):
    from oracle import naive_mirror as nm
    from srf_amd import train_helper
    n = 4096 + 64
    rng = np.random.default_rng(5)
    p0 = rng.standard_normal(n)
    cfg = config_from_shape({'feat_dim': 123, 'enc_num': 1, 'iters': 1, 'lpad': 0, 'rpad': 0, 'ph': 4, 'pd': 8,
                             'ch': 4, 'cd': 8, 'vd': 8, 'context': False},
                            train_lr_param_k=k, train_warmup_n=warmup, train_lr_max=max_lr)
    opt = train_helper.get_optimizer(cfg)
    model = _Flat(p0, cuda)
    ref_p = torch.nn.Parameter(torch.tensor(p0.astype(np.float32), dtype=torch.float64))
    ref = nm.TfAdam([ref_p], k=k, d_model=1, warmup=warmup, max_lr=max_lr, b1=0.9, b2=0.98, eps=1e-9)
    for step in range(5):
        g = rng.standard_normal(n).astype(np.float32) * (10.0 ** (step - 2))
        model.flat_grad.copy_(torch.from_numpy(g))
        opt.apply_gradients(model)
        ref_p.grad = torch.tensor(g, dtype=torch.float64)
        ref.step()
        torch.cuda.synchronize()
        assert abs(opt.current_lr() - ref.lr(ref.iterations)) <= 1e-12 * max(1.0, ref.lr(ref.iterations))
        for got, want, what in ((model.flat_params, ref_p.detach(), 'params'), (opt._m, ref.m[0], 'm'),
                                (opt._v, ref.v[0], 'v')):
            got = got.double().cpu()
            err = ((got - want).abs() / (1 + want.abs())).max().item()
            assert err <= 4e-6, (step, what, err)
    if k == 0.5:      # lr(0) == 0: the first update is a no-op, later ones move the parameters
        assert not np.allclose(model.flat_params.cpu().numpy(), p0.astype(np.float32))


def test_adam_skips_update_while_fault_word_set(cuda):
    """A grouped SDR recurrence that timed out sets the process's fault word
    (srf_set_fault_flag): until the host has read and cleared it, the fused Adam must
    not apply a gradient computed from the wrong results (adam.hip reads the word)."""
    from srf_amd import ops, train_helper
    n = 1024 + 3
    cfg = config_from_shape({'feat_dim': 123, 'enc_num': 1, 'iters': 1, 'lpad': 0, 'rpad': 0, 'ph': 4, 'pd': 8,
                             'ch': 4, 'cd': 8, 'vd': 8, 'context': False},
                            train_lr_param_k=100.0, train_warmup_n=2, train_lr_max=1e-2)
    opt = train_helper.get_optimizer(cfg)
    model = _Flat(np.linspace(-1, 1, n), cuda)
    model.flat_grad.fill_(1.0)
    p0 = model.flat_params.clone()
    f = ops.fault_flag(cuda)
    f.fill_(1)
    opt.apply_gradients(model)
    torch.cuda.synchronize()
    assert torch.equal(model.flat_params, p0) and not opt._m.abs().max().item()
    with pytest.raises(RuntimeError, match='timed out'):
        ops.check_faults()          # reads and clears the word
    assert int(f.item()) == 0
    opt.apply_gradients(model)
    torch.cuda.synchronize()
    assert (model.flat_params - p0).abs().min().item() > 0


# ---------------------------------------------------------------------------
# bucketed TFRecord batches through the captured step
_BUCKETS = ([30, 45], [4, 3, 2])
_LENGTHS = [28, 25, 22, 28, 44, 40, 33, 28, 20, 24, 21, 60, 52, 44, 31, 38, 57, 49]


def _corpus(tmp_path, class_n):
    from srf_amd import load_speech_data as lsd
    rng = np.random.default_rng(9)
    d = tmp_path / 'tfr'
    d.mkdir()
    with lsd.TFRecordWriter(str(d / 'train-00001-of-00001')) as w:
        for i, T in enumerate(_LENGTHS):
            L = int(rng.integers(1, (-(-T // 4)) // 2 + 1))
            w.write_example(rng.standard_normal((T, 123)).astype(np.float32), rng.integers(1, class_n - 1, L),
                            utt_id=f'u{i}')
    ds = lsd.create_ds_bucket(str(d / '*'), False, 1, _BUCKETS[0], _BUCKETS[1], -1, -1)
    return ds.map(lsd.map_data_for_transformer_fn, 123)


def _build(cfg, sh, P, dev):
    from srf_amd.sequence_router import SequenceRouter
    m = SequenceRouter(cfg, None, sh.class_n, device=dev)
    m.load_params(P)
    m.dropout_enabled = False
    return m


def test_graph_cache_serves_bucketed_batches(cuda, tmp_path):
    from srf_amd import train_helper, trainer_sr
    kw, sh, P, _ = load_model_fixture('c2_mini')
    cfg = config_from_shape(kw, train_opti_type='adam', train_lr_param_k=0.0)   # lr 0: parameters stay put
    ds = _corpus(tmp_path, sh.class_n)
    eager, graphed = _build(cfg, sh, P, cuda), _build(cfg, sh, P, cuda)
    cache = trainer_sr.GraphCache(4, graphed, train_helper.get_optimizer(cfg), 1, sh.class_n - 1, warmup=1)
    opt_e = train_helper.get_optimizer(cfg)
    shapes = []
    for batch in ds:
        inputs = trainer_sr.batch_to_device(batch, cuda)
        shapes.append((inputs[0].shape[0], int(inputs[2].max())))
        nll_e = trainer_sr.process_train_step(4, inputs, eager, opt_e, None, None, 1, sh.class_n - 1, None)
        nll_g = cache.step(inputs)
        torch.cuda.synchronize()
        assert torch.allclose(nll_g, nll_e, rtol=1e-5, atol=1e-5), (shapes[-1], nll_g, nll_e)
        err = (graphed.flat_grad - eager.flat_grad).abs().max().item()
        assert err <= 1e-4 * eager.flat_grad.abs().max().item(), (shapes[-1], err)
    assert shapes == [(4, 28), (3, 44), (4, 28), (2, 60), (3, 44), (2, 57)], shapes
    # a shape is captured on its second sighting, its first step runs eagerly
    assert cache.captures == 2 and cache.eager_steps == 4
    assert torch.equal(graphed.flat_params, eager.flat_params)
    _same_bn(graphed, eager)            # building a graph does not update BN a second time

    # the hot loop itself, on the cached graphs; the eager model through the same loop
    loss, frames, samples = trainer_sr.Mean(), trainer_sr.Mean(), trainer_sr.Sum()
    n = trainer_sr.distributed_train_step(ds, 4, graphed, cache.args[2], loss, frames, 1, sh.class_n - 1,
                                          samples, train_num=len(_LENGTHS), graphs=cache, log=None)
    assert n == 6 and samples.result() == 18 and np.isfinite(loss.result())
    assert cache.captures == 4          # (2, 60) and (2, 57) on their second sighting; the rest replayed
    trainer_sr.distributed_train_step(ds, 4, eager, opt_e, trainer_sr.Mean(), trainer_sr.Mean(), 1, sh.class_n - 1,
                                      trainer_sr.Sum(), log=None)
    torch.cuda.synchronize()
    _same_bn(graphed, eager)
    for g in cache.graphs.values():
        g.close()


def _same_bn(a, b):
    for name in ('bn0_moving_mean', 'bn0_moving_var', 'bn1_moving_mean', 'bn1_moving_var'):
        x, y = getattr(a, name), getattr(b, name)
        assert torch.allclose(x, y, rtol=1e-5, atol=1e-6), (name, (x - y).abs().max().item())
