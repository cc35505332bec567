"""The captured multi-stream SDR step at the bench size, in every schedule variant.

Round 5 saw one host SIGSEGV inside ``torch.cuda.CUDAGraph.replay`` of a graphed
``wsj_c3`` bench step (``gpurun_out/r05j/b3.log``) on an intermediate tree while the
stack's capture order was being reworked; the variant's flags were not logged
("Graph-replay crash").  This test captures the C3 training
step (B = 28, T = 800: 20 frame ranges per layer, three streams, the last layer's
backward grouped) under each schedule the bench can select -- the default (last
layer's gx / gW on a third stream), that launch inline, separate gx and gW launches,
one LN launch per layer, and the last layer's recurrence ungrouped or grouped both
ways, and the opt-in gu factors (ops.SDR_GU_FACTORS) -- replays it several times, and checks every replay against eager
``process_train_step`` of the same schedule.

The routing weights are scaled to half the reference init, where the step's gradient
stays finite (at the reference init the SDR backward overflows on these inputs, DESIGN
section 3.5).  The forward is deterministic (no atomics; group partials are summed in a
fixed order), so the per-utterance NLL must agree to fp32 rounding.  The gradient is not
bitwise reproducible (g_emb's window adjoint adds with float atomics, and the SDR
recurrence amplifies the difference through the layers below), so each replay's
gradient is held to 10x the distance between two eager runs of the same schedule
(plus 1e-6 relative).  conftest checks that no grouped launch set the fault word.

References: trainer_sr.py:41-75 (the step), sequence_router_naive.py:162-170,
212-245 (the SDR frame loop).
"""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

class _NoUpdate:
    """optimizer stand-in: the gradient is compared, the parameters stay as they are"""

    def apply_gradients(self, model):
        pass


VARIANTS = {
    'default': {},
    'last_gxw_inline': {'SDR_LAST_GXW_SIDE': False},
    'separate_gxgw': {'SDR_FUSED_GXGW': False},
    'capsnorm_per_layer': {'SDR_CAPSNORM_BATCHED': False},
    'last_ungrouped': {'last_group': (1, 1)},
    'last_grouped_both': {'last_group': (2, 2)},
    'gu_factors': {'SDR_GU_FACTORS': True},   # recurrence writes gu factors, gx / gW form gu
}


@pytest.fixture(scope='module')
def c3_model(cuda):
    sys.path.insert(0, ROOT)
    import bench
    from srf_amd.sequence_router import SequenceRouter
    kw, class_n, B, T = bench.WORKLOADS['wsj_c3']
    cfg = bench.make_config(kw)
    model = SequenceRouter(cfg, None, class_n, device=cuda, seed=1234)
    model.dropout_enabled = False
    # routing weights at half the reference init (as the c3_real fixture): at the reference
    # init the SDR backward through 200 frames overflows (max|g| ~ 1e26, NaN in the CNN-FE
    # gradient; scripts/dbg/grad_finite.py), which would hide a wrong replay
    with torch.no_grad():
        for l in range(model.enc_num):
            model.params[f'W{l}'].mul_(0.5)
    batch = bench.synthetic_batch(B, T, class_n, 0, cuda)
    return cfg, model, batch, class_n


@pytest.mark.parametrize('variant', list(VARIANTS))
def test_c3_graphed_step_replays_in_every_schedule(cuda, c3_model, variant):
    from srf_amd import ops, trainer_sr
    cfg, model, batch, class_n = c3_model
    opts = dict(VARIANTS[variant])
    group = opts.pop('last_group', None)
    saved = {k: getattr(ops, k) for k in opts}
    saved_group = model.sdr_options.get('last_group')
    try:
        for k, v in opts.items():
            setattr(ops, k, v)
        if group is not None:
            model.sdr_options['last_group'] = group
        else:
            model.sdr_options.pop('last_group', None)
        for key in [k for k in model._geoms if k[0] == 'sdr_stack']:
            del model._geoms[key]   # the stack plan reads last_group when it is built
        p0 = model.flat_params.clone()

        def eager():
            nll = trainer_sr.process_train_step(4, batch, model, _NoUpdate(), None, None, 1, class_n - 1,
                                                None).clone()
            return nll, model.flat_grad.clone()
        nll_e, g_e = eager()
        nll_e2, g_e2 = eager()
        assert torch.equal(model.flat_params, p0)
        assert torch.allclose(nll_e2, nll_e, rtol=2e-6, atol=1e-5)
        noise = (g_e2 - g_e).norm().item()
        scale = g_e.norm().item()
        assert torch.isfinite(g_e).all() and scale > 0
        g = trainer_sr.GraphedTrainStep(4, batch, model, _NoUpdate(), 1, class_n - 1, warmup=1)
        try:
            for rep in range(5):
                g.graph.replay()     # forward + CTC + backward only: no Adam, the parameters stay
                torch.cuda.synchronize()
                nll = g.nll.clone()
                assert torch.allclose(nll, nll_e, rtol=2e-6, atol=1e-5), (variant, rep, (nll - nll_e).abs().max())
                err = (model.flat_grad - g_e).norm().item()
                assert err <= 10.0 * noise + 1e-6 * scale, (variant, rep, err, noise, scale)
        finally:
            g.close()
        assert torch.equal(model.flat_params, p0)
    finally:
        for k, v in saved.items():
            setattr(ops, k, v)
        if saved_group is None:
            model.sdr_options.pop('last_group', None)
        else:
            model.sdr_options['last_group'] = saved_group
