"""Which gradient slices does a GraphedTrainStep replay leave unwritten? (debug)"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from srf_amd import train_helper, trainer_sr
from tests.helpers import config_from_shape, load_model_fixture
from srf_amd.sequence_router import SequenceRouter
dev = torch.device('cuda:0')
kw, sh, P, z = load_model_fixture('c2_mini')
cfg = config_from_shape(kw)
m = SequenceRouter(cfg, None, sh.class_n, device=dev)
m.load_params(P)
m.dropout_enabled = False
inputs = (torch.tensor(z['feats'], dtype=torch.float32, device=dev), torch.tensor(z['labels'], device=dev),
          torch.tensor(z['inp_len'], dtype=torch.int32), torch.tensor(z['tar_len'], device=dev))
g = trainer_sr.GraphedTrainStep(4, inputs, m, train_helper.get_optimizer(cfg), 1, sh.class_n - 1, warmup=1)
ok = {k: (p.grad is not None and p.grad.data_ptr() >= m.flat_grad.data_ptr() and
          p.grad.data_ptr() < m.flat_grad.data_ptr() + m.flat_grad.numel() * 4) for k, p in m.params.items()}
print('grad views intact:', all(ok.values()), [k for k, v in ok.items() if not v])
m.flat_grad.fill_(float('nan'))
g.graph.replay()
torch.cuda.synchronize()
for k, p in m.params.items():
    bad = torch.isnan(p.grad).sum().item()
    if bad:
        print('NaN grad slice:', k, bad, p.grad.numel())
g.close()
