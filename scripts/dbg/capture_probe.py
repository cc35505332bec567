"""Probe: multi-stream hipGraph capture (fork/join with events) -- which piece crashes.
python scripts/dbg/capture_probe.py {torch|stackfwd|step}"""
import sys
import os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
what = sys.argv[1]
dev = torch.device('cuda:0')
if what == 'torch':
    x = torch.randn(1 << 20, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    ev = [torch.cuda.Event() for _ in range(4)]
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        main = torch.cuda.current_stream()
        s1.wait_stream(main); s2.wait_stream(main)
        with torch.cuda.stream(s1):
            y = x * 2
        ev[0].record(s1)
        s2.wait_event(ev[0])
        with torch.cuda.stream(s2):
            z = y + 1
        main.wait_stream(s1); main.wait_stream(s2)
        w = z.sum()
    g.replay(); torch.cuda.synchronize()
    print('torch ok', float(w))
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
    ild = il.to(dev)
    if what == 'stackfwd':
        with torch.no_grad():
            model(feats, input_lengths=ild, training=True)
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                model(feats, input_lengths=ild, training=True)
            torch.cuda.current_stream().wait_stream(side)
            with torch.cuda.graph(g):
                out = model(feats, input_lengths=ild, training=True)
        g.replay(); torch.cuda.synchronize()
        print('stackfwd ok', float(out.abs().sum()))
    else:
        inputs = (feats, torch.tensor(z['labels'], device=dev), il, torch.tensor(z['tar_len'], device=dev))
        cfg = config_from_shape(kw)
        g = trainer_sr.GraphedTrainStep(4, inputs, model, train_helper.get_optimizer(cfg), 1, sh.class_n - 1, warmup=1)
        nll = g()
        torch.cuda.synchronize()
        print('step ok', nll)
