"""End-to-end GPU parity of SequenceRouter + CTC against the golden fixtures
(numpy float64 oracle of sequence_router_naive.py; gradients from the float64
torch mirror).  Batch-norm runs in training mode (batch statistics, as in
process_train_step); dropout is disabled so the two sides see identical graphs.

Tolerances (fp32 GPU vs fp64 oracle, stated per north_star): logits
|err| <= 1e-4 * (1 + |ref|); CTC NLL |err| <= 1e-4 * max(1, |ref|);
greedy label sequences bit-exact; gradients |err| <= 2e-3 * max|ref| + 1e-5.
"""
import numpy as np
import pytest
import torch

from tests.helpers import config_from_shape, gradient_mismatches, load_model_fixture

pytestmark = pytest.mark.gpu

DR_FIXTURES = ['c1_mini', 'c2_mini', 'c3_mini_sdr',   # c3: SDR routing
               'c4_mini',                                # DR at DIM 32 (C3/C4 capsule width)
               # the einsum / lowmemory variants (trainer_sr.py:188-199)
               'c2_mini_einsum', 'c2_mini_lowmemory', 'c3_mini_sdr_lowmemory',
               # BASELINE's real configurations (oracle/gen_golden.py BIG_CASES): C2 as the
               # bench runs it (B=17, T=320, ragged), C4 / C3 at L=6 PH=CH=16 DIM=32,
               # C5 at L=8 DIM=64 LPAD=RPAD=20 with 5 SDR iterations
               'c2_full', 'c4_real', 'c3_real', 'c5_real']


def _build(name, dev):
    from srf_amd.sequence_router import SequenceRouter
    kw, sh, P, z = load_model_fixture(name)
    cfg = config_from_shape(kw)
    model = SequenceRouter(cfg, None, sh.class_n, device=dev)
    model.load_params(P)
    model.dropout_enabled = False
    return model, sh, z


@pytest.mark.parametrize('name', DR_FIXTURES)
def test_forward_logits_ctc_greedy(cuda, name):
    from srf_amd import ctc
    model, sh, z = _build(name, cuda)
    feats = torch.tensor(z['feats'], dtype=torch.float32, device=cuda)
    inp_len = torch.tensor(z['inp_len'], device=cuda)
    logits = model(feats, input_lengths=inp_len, training=True)
    got = logits.detach().cpu().double().numpy()
    ref = z['logits']
    assert got.shape == ref.shape
    assert np.all(np.abs(got - ref) <= 1e-4 * (1 + np.abs(ref))), np.abs(got - ref).max()
    nll = ctc.ctc_loss(torch.tensor(z['labels'], device=cuda), logits, torch.tensor(z['tar_len'], device=cuda),
                       (inp_len + 3) // 4, blank_index=sh.class_n - 1)
    nll = nll.detach().cpu().double().numpy()
    assert np.all(np.abs(nll - z['nll']) <= 1e-4 * np.maximum(1, np.abs(z['nll']))), (nll, z['nll'])
    hyp = ctc.greedy_decode(logits, (inp_len + 3) // 4, sh.class_n - 1)
    assert hyp == z['greedy']


@pytest.mark.parametrize('name', DR_FIXTURES)
def test_gradients(cuda, name):
    from srf_amd import ctc
    model, sh, z = _build(name, cuda)
    feats = torch.tensor(z['feats'], dtype=torch.float32, device=cuda)
    inp_len = torch.tensor(z['inp_len'], device=cuda)
    model.zero_grad()
    logits = model(feats, input_lengths=inp_len, training=True)
    nll = ctc.ctc_loss(torch.tensor(z['labels'], device=cuda), logits, torch.tensor(z['tar_len'], device=cuda),
                       (inp_len + 3) // 4, blank_index=sh.class_n - 1)
    (nll.sum() / feats.shape[0]).backward()
    bad = gradient_mismatches(z, lambda p: model.P(p).grad.detach().cpu().double().numpy())
    assert not bad, bad


@pytest.mark.parametrize('name', ['c4_mini', 'c4_real'])
def test_dr_gw_side_stream_matches(cuda, name):
    """ops.DR_GW_SIDE (each DR layer's gW / gbias deferred onto a side stream, joined by
    ops.dr_side_join) and ops.CNNFE_WGRAD_SIDE (the CNN front end's stage-2 weight gradient
    there too) compute the gradients of the one-stream backward: the same kernels
    on the same inputs, only on another stream (up to the order of the gx pass's float
    atomics into g_emb, which differs run to run either way)."""
    from srf_amd import ctc, ops
    model, sh, z = _build(name, cuda)
    feats = torch.tensor(z['feats'], dtype=torch.float32, device=cuda)
    inp_len = torch.tensor(z['inp_len'], device=cuda)
    grads = []
    defaults = (ops.DR_GW_SIDE, ops.CNNFE_WGRAD_SIDE)
    for side in (False, True):
        ops.DR_GW_SIDE = ops.CNNFE_WGRAD_SIDE = side
        try:
            model.zero_grad()
            logits = model(feats, input_lengths=inp_len, training=True)
            nll = ctc.ctc_loss(torch.tensor(z['labels'], device=cuda), logits, torch.tensor(z['tar_len'], device=cuda),
                               (inp_len + 3) // 4, blank_index=sh.class_n - 1)
            (nll.sum() / feats.shape[0]).backward()
            ops.dr_side_join()
            torch.cuda.synchronize()
            grads.append(model.flat_grad.detach().clone())
        finally:
            ops.DR_GW_SIDE, ops.CNNFE_WGRAD_SIDE = defaults
    err, mag = (grads[0] - grads[1]).abs().max().item(), grads[0].abs().max().item()
    assert err <= 1e-5 * mag, (err, mag)


def test_train_step_runs_and_updates(cuda):
    """process_train_step: loss finite, params move after step 2 (lr(0) == 0)."""
    from srf_amd import train_helper, trainer_sr
    model, sh, z = _build('c2_mini', cuda)
    model.dropout_enabled = True
    cfg = config_from_shape({'feat_dim': 123, 'enc_num': 3, 'iters': 3, 'lpad': 4, 'rpad': 4, 'ph': 8,
                             'pd': 16, 'ch': 8, 'cd': 16, 'vd': 16, 'context': False})
    opt = train_helper.get_optimizer(cfg)
    inputs = (torch.tensor(z['feats'], dtype=torch.float32, device=cuda),
              torch.tensor(z['labels'], device=cuda), torch.tensor(z['inp_len'], device=cuda),
              torch.tensor(z['tar_len'], device=cuda))
    p0 = model.flat_params.clone()
    loss_state, frames, samples = trainer_sr.Mean(), trainer_sr.Mean(), trainer_sr.Sum()
    trainer_sr.process_train_step(4, inputs, model, opt, loss_state, frames, 1, sh.class_n - 1, samples)
    assert torch.equal(model.flat_params, p0)          # lr(0) = 0: first update is a no-op
    trainer_sr.process_train_step(4, inputs, model, opt, loss_state, frames, 1, sh.class_n - 1, samples)
    assert not torch.equal(model.flat_params, p0)
    assert np.isfinite(loss_state.result())
    assert samples.result() == 4


@pytest.mark.parametrize('name', ['c2_mini', 'c2_mini_lowmemory', 'c3_mini_sdr_lowmemory', 'c4_mini'])
def test_backward_overwrites_every_gradient(cuda, name):
    """The train step never zeroes grads: every parameter's gradient must be
    written (not accumulated) by the backward kernels.  Poison the flat gradient
    buffer, run one backward, and require every slice finite and equal to a
    backward from zeroed grads."""
    from srf_amd import ctc, trainer_sr
    model, sh, z = _build(name, cuda)
    feats = torch.tensor(z['feats'], dtype=torch.float32, device=cuda)
    inp_len = torch.tensor(z['inp_len'], dtype=torch.int32, device=cuda)
    labels = torch.tensor(z['labels'], device=cuda)
    tar_len = torch.tensor(z['tar_len'], device=cuda)

    def grads(poison):
        model.flat_grad.fill_(float('nan') if poison else 0.0)
        logits = model(feats, input_lengths=inp_len, training=True)
        _, g = ctc.ctc_loss_and_grad(labels, logits, tar_len, trainer_sr.ceil_div(inp_len, 4), sh.class_n - 1,
                                     1.0 / feats.shape[0])
        logits.backward(g)
        return {k: p.grad.detach().clone() for k, p in model.params.items()}

    clean = grads(False)
    poisoned = grads(True)
    for k in clean:
        assert torch.isfinite(poisoned[k]).all(), k
        # equal up to float-atomic reassociation in the routing backward (an
        # accumulation into stale values would be off by O(1) relative)
        err = (poisoned[k] - clean[k]).abs().max().item()
        assert err <= 1e-4 * clean[k].abs().max().item() + 1e-7, (k, err)


def test_fused_loss_head_matches_autograd(cuda):
    """ctc_loss_and_grad + logits.backward(g) == autograd of sum(nll)/B."""
    from srf_amd import ctc, trainer_sr
    model, sh, z = _build('c2_mini', cuda)
    feats = torch.tensor(z['feats'], dtype=torch.float32, device=cuda)
    inp_len = torch.tensor(z['inp_len'], dtype=torch.int32, device=cuda)
    labels = torch.tensor(z['labels'], device=cuda)
    tar_len = torch.tensor(z['tar_len'], device=cuda)
    lens4 = trainer_sr.ceil_div(inp_len, 4)
    model.zero_grad()
    logits = model(feats, input_lengths=inp_len, training=True)
    nll = ctc.ctc_loss(labels, logits, tar_len, lens4, blank_index=sh.class_n - 1)
    (nll.sum() / feats.shape[0]).backward()
    ref = model.flat_grad.clone()
    model.zero_grad()
    logits = model(feats, input_lengths=inp_len, training=True)
    nll2, g = ctc.ctc_loss_and_grad(labels, logits, tar_len, lens4, sh.class_n - 1, 1.0 / feats.shape[0])
    logits.backward(g)
    assert torch.allclose(nll2, nll.detach())
    assert (model.flat_grad - ref).abs().max().item() <= 1e-4 * ref.abs().max().item()


@pytest.mark.parametrize('name', ['c2_mini', 'c2_mini_lowmemory', 'c2_mini_einsum', 'c4_mini', 'c3_mini_sdr'])
def test_graphed_train_step_matches_eager(cuda, name):
    """GraphedTrainStep (forward + CTC + backward in one hipGraph) computes the same
    loss and gradient as the eager process_train_step, and draws fresh dropout masks
    on every replay (device step counter)."""
    from srf_amd import train_helper, trainer_sr
    cfg = config_from_shape({'feat_dim': 123, 'enc_num': 3, 'iters': 3, 'lpad': 4, 'rpad': 4, 'ph': 8,
                             'pd': 16, 'ch': 8, 'cd': 16, 'vd': 16, 'context': False})
    model, sh, z = _build(name, cuda)
    inputs = (torch.tensor(z['feats'], dtype=torch.float32, device=cuda), torch.tensor(z['labels'], device=cuda),
              torch.tensor(z['inp_len'], dtype=torch.int32), torch.tensor(z['tar_len'], device=cuda))
    opt = train_helper.get_optimizer(cfg)   # lr(0) = 0: the first update leaves the parameters
    eager_nll = trainer_sr.process_train_step(4, inputs, model, opt, None, None, 1, sh.class_n - 1, None).clone()
    eager_grad = model.flat_grad.clone()
    model2, _, _ = _build(name, cuda)
    g = trainer_sr.GraphedTrainStep(4, inputs, model2, train_helper.get_optimizer(cfg), 1, sh.class_n - 1, warmup=1)
    try:
        model2.load_params({k: v for k, v in zip(*_params_of(model))})
        for p in model2.params.values():   # poison every gradient slice (not the alignment padding)
            p.grad.fill_(float('nan'))
        nll = g().clone()
        torch.cuda.synchronize()
        assert torch.allclose(nll, eager_nll, rtol=1e-5, atol=1e-5), (nll, eager_nll)
        err = (model2.flat_grad - eager_grad).abs().max().item()
        assert err <= 1e-4 * eager_grad.abs().max().item(), err
        # dropout on: consecutive replays see different masks
        model2.dropout_enabled = True
        g2 = trainer_sr.GraphedTrainStep(4, inputs, model2, train_helper.get_optimizer(cfg), 1, sh.class_n - 1,
                                         warmup=1)
        a = g2().clone()
        b = g2().clone()
        assert torch.isfinite(a).all() and not torch.equal(a, b)
        g2.close()
    finally:
        g.close()


def _params_of(model):
    names = list(model.params.keys())
    return names, [model.params[k].detach().clone() for k in names]


def test_graphed_dropout_gradient_matches_finite_difference(cuda):
    """Dropout on, GraphedTrainStep: the replayed gradient must be the gradient of
    the loss under the SAME dropout masks.  The forward and the backward kernels
    both rebuild their masks from (per-call seed, device step counter); the
    backward runs on torch's autograd device thread, so the counter must be seen
    there too (a per-thread counter would leave the backward on other masks).
    Checked with central differences of the graphed step's own loss along the
    gradient direction and along a random direction (fp32, 2 % tolerance)."""
    from srf_amd import ctc, train_helper, trainer_sr
    cfg = config_from_shape({'feat_dim': 123, 'enc_num': 3, 'iters': 3, 'lpad': 4, 'rpad': 4, 'ph': 8,
                             'pd': 16, 'ch': 8, 'cd': 16, 'vd': 16, 'context': False})
    model, sh, z = _build('c2_mini', cuda)
    model.dropout_enabled = True
    inputs = (torch.tensor(z['feats'], dtype=torch.float32, device=cuda), torch.tensor(z['labels'], device=cuda),
              torch.tensor(z['inp_len'], dtype=torch.int32), torch.tensor(z['tar_len'], device=cuda))
    g = trainer_sr.GraphedTrainStep(4, inputs, model, train_helper.get_optimizer(cfg), 1, sh.class_n - 1, warmup=1)
    try:
        cap_calls = model._calls             # the captured forward drew seed number cap_calls
        g.graph.replay()                     # counter -> c + 1; gradient into flat_grad
        torch.cuda.synchronize()
        grad = model.flat_grad.clone()
        B = inputs[0].shape[0]

        @torch.no_grad()
        def loss():
            model._calls = cap_calls - 1     # same per-call seed as the captured step
            logits = model(g.feats, input_lengths=g.inp_len, training=True)
            nll = ctc.ctc_loss(g.labels, logits, g.tar_len, g.logit_len, blank_index=sh.class_n - 1)
            return float(nll.double().sum()) / B

        assert abs(loss() - float(g.nll.double().sum()) / B) <= 1e-4 * abs(loss())
        p0 = model.flat_params.clone()
        gen = torch.Generator(device=cuda).manual_seed(7)
        rnd = torch.randn(p0.shape, device=cuda, generator=gen) * (grad != 0)
        for d in (grad / grad.norm(), rnd / rnd.norm()):
            h = 1e-3    # calibrated (scripts/dbg_fd.py): |p| ~ 131, |g| ~ 160; h = 1e-1 is too coarse
            model.flat_params.copy_(p0 + h * d)
            lp = loss()
            model.flat_params.copy_(p0 - h * d)
            lm = loss()
            model.flat_params.copy_(p0)
            fd, an = (lp - lm) / (2 * h), float((grad * d).sum())
            assert abs(fd - an) <= 0.02 * abs(float(grad.norm())), (fd, an, float(grad.norm()))
    finally:
        g.close()


@pytest.mark.parametrize('name,chunks,cs,store', [('c3_mini_sdr', 1, True, None), ('c3_mini_sdr', 3, True, None),
                                                  ('c3_mini_sdr', 64, True, None), ('c3_real', 4, True, None),
                                                  ('c3_real', 4, False, None), ('c3_real', 4, True, 0),
                                                  ('c5_real', 3, True, None), ('c5_real', 3, True, 0),
                                                  ('c3_mini_sdr_lowmemory', 2, True, None)])
def test_sdr_stack_matches_layer_by_layer(cuda, name, chunks, cs, store):
    """The layer-pipelined SDR stack (ops.SdrStack: frame ranges of every layer as a
    wavefront) against the layer-by-layer path (model.sdr_stack = False): the same
    logits and gradients to fp32 reassociation, for one range, several, and one frame
    per range (64 > T'); its backward from the forward's stored couplings
    (store_couplings) and recomputing them; u kept from the forward (default) and
    recomputed per range (store_u_bytes = 0)."""
    from srf_amd import ctc
    outs = []
    for stack in (True, False):
        model, sh, z = _build(name, cuda)
        model.sdr_stack = stack
        model.sdr_options = dict(n_chunks=chunks, store_couplings=cs, store_u_bytes=store)
        feats = torch.tensor(z['feats'], dtype=torch.float32, device=cuda)
        inp_len = torch.tensor(z['inp_len'], device=cuda)
        model.zero_grad()
        logits = model(feats, input_lengths=inp_len, training=True)
        nll = ctc.ctc_loss(torch.tensor(z['labels'], device=cuda), logits, torch.tensor(z['tar_len'], device=cuda),
                           (inp_len + 3) // 4, blank_index=sh.class_n - 1)
        (nll.sum() / feats.shape[0]).backward()
        torch.cuda.synchronize()
        outs.append((logits.detach().clone(), model.flat_grad.clone()))
    (la, ga), (lb, gb) = outs
    assert (la - lb).abs().max().item() <= 1e-5 * (1 + lb.abs().max().item())
    assert (ga - gb).abs().max().item() <= 1e-4 * gb.abs().max().item()
