"""Probe: multi-stream work inside an autograd backward during hipGraph capture.
python scripts/dbg/capture_probe2.py {torchbwd|torchbwd_relaxed|torchbwd_tl|step_relaxed|step_tl}"""
import functools
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
what = sys.argv[1]
dev = torch.device('cuda:0')
mode = 'relaxed' if what.endswith('relaxed') else ('thread_local' if what.endswith('_tl') else 'global')
if mode != 'global':
    torch.cuda.graph = functools.partial(torch.cuda.graph, capture_error_mode=mode)
S = [torch.cuda.Stream() for _ in range(3)]
EV = [torch.cuda.Event() for _ in range(3)]


class Fork(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x * 2

    @staticmethod
    def backward(ctx, g):
        main = torch.cuda.current_stream()
        outs = []
        for s in S:
            s.wait_stream(main)
        for i, s in enumerate(S):
            if i:
                s.wait_event(EV[i - 1])
            with torch.cuda.stream(s):
                outs.append(g * (i + 1))
            EV[i].record(s)
        for s in S:
            main.wait_stream(s)
        return outs[0] + outs[1] + outs[2]


if what == 'torch2fork':   # the same side streams forked twice in one capture
    x = torch.randn(1 << 16, device=dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        main = torch.cuda.current_stream()
        tot = x * 0
        for rep in range(2):
            for s in S:
                s.wait_stream(main)
            outs = []
            for i, s in enumerate(S):
                with torch.cuda.stream(s):
                    outs.append(x * (i + rep))
            for s in S:
                main.wait_stream(s)
            tot = tot + outs[0] + outs[1] + outs[2]
    g.replay()
    torch.cuda.synchronize()
    print(what, 'ok', float(tot.sum()))
elif what.startswith('torchbwd'):
    x = torch.randn(1 << 16, device=dev, requires_grad=True)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        Fork.apply(x).sum().backward()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    x.grad = None
    with torch.cuda.graph(g):
        Fork.apply(x).sum().backward()
    g.replay()
    torch.cuda.synchronize()
    print(what, 'ok', float(x.grad.sum()))
else:
    from tests.helpers import config_from_shape, load_model_fixture
    from srf_amd.sequence_router import SequenceRouter
    from srf_amd import train_helper, trainer_sr
    kw, sh, P, z = load_model_fixture('c3_mini_sdr')
    model = SequenceRouter(config_from_shape(kw), None, sh.class_n, device=dev)
    model.load_params(P)
    model.dropout_enabled = False
    feats = torch.tensor(z['feats'], dtype=torch.float32, device=dev)
    il = torch.tensor(z['inp_len'], dtype=torch.int32)
    inputs = (feats, torch.tensor(z['labels'], device=dev), il, torch.tensor(z['tar_len'], device=dev))
    g = trainer_sr.GraphedTrainStep(4, inputs, model, train_helper.get_optimizer(config_from_shape(kw)), 1,
                                    sh.class_n - 1, warmup=1)
    nll = g()
    torch.cuda.synchronize()
    print(what, 'ok', nll)
