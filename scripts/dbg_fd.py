"""Finite-difference calibration of the dropout-on gradient (graphed vs eager)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from tests.helpers import config_from_shape, load_model_fixture
from srf_amd import ctc, train_helper, trainer_sr
from srf_amd.sequence_router import SequenceRouter

cuda = torch.device('cuda:0')
kw, sh, P, z = load_model_fixture('c2_mini')
cfg = config_from_shape(kw)
model = SequenceRouter(cfg, None, sh.class_n, device=cuda)
model.load_params(P)
inputs = (torch.tensor(z['feats'], dtype=torch.float32, device=cuda), torch.tensor(z['labels'], device=cuda),
          torch.tensor(z['inp_len'], dtype=torch.int32), torch.tensor(z['tar_len'], device=cuda))
B = inputs[0].shape[0]
il = inputs[2].to(cuda)
ll = trainer_sr.ceil_div(il, 4)


def run(mode):
    model.flat_grad.zero_()
    if mode == 'graph':
        g = trainer_sr.GraphedTrainStep(4, inputs, model, train_helper.get_optimizer(cfg), 1, sh.class_n - 1, warmup=1)
        cap = model._calls
        g.graph.replay()
    else:
        cap = model._calls + 1
        logits = model(inputs[0], input_lengths=il, training=True)
        _, gl = ctc.ctc_loss_and_grad(inputs[1], logits, inputs[3], ll, sh.class_n - 1, 1.0 / B)
        logits.backward(gl)
    torch.cuda.synchronize()
    grad = model.flat_grad.clone()

    @torch.no_grad()
    def loss():
        model._calls = cap - 1
        logits = model(inputs[0], input_lengths=il, training=True)
        nll = ctc.ctc_loss(inputs[1], logits, inputs[3], ll, blank_index=sh.class_n - 1)
        return float(nll.double().sum()) / B

    p0 = model.flat_params.clone()
    d = grad / grad.norm()
    print(mode, 'L', loss(), '|g|', float(grad.norm()), '|p|', float(p0.norm()))
    for h in (1e-1, 3e-2, 1e-2, 3e-3, 1e-3, 3e-4):
        model.flat_params.copy_(p0 + h * d); lp = loss()
        model.flat_params.copy_(p0 - h * d); lm = loss()
        model.flat_params.copy_(p0)
        print(f'  h={h:g} fd={(lp - lm) / (2 * h):.4f} an={float((grad * d).sum()):.4f}')
    if mode == 'graph':
        g.close()


for dropout in (False, True):
    model.dropout_enabled = dropout
    print('dropout', dropout)
    run('eager')
    run('graph')
