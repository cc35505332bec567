"""The RCCL leg of the data-parallel step, once, at world size 1 (the 8-GPU node is
the driver's): a child process of tests/test_dp_gpu.py that brings up an ``nccl``
(= RCCL on ROCm) process group with device_id, then takes the c2_mini fixture
through process_train_step with the flat all-reduce, with the bucketed all-reduce
issued from the backward (GradBuckets, force=True: the collectives run at world 1),
and through GraphedTrainStep with those bucketed collectives captured in the graph.
A SUM over one rank is the identity, so all three gradients must equal the
fixture's.  Prints one JSON line; exit status 0 unless it crashed.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    from srf_amd import train_helper, trainer_sr
    from srf_amd.sequence_router import SequenceRouter
    from tests.helpers import config_from_shape, gradient_mismatches, load_model_fixture

    dev = torch.device('cuda:0')
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', device_id=dev)
    out = {'backend': dist.get_backend(), 'world': dist.get_world_size()}
    kw, sh, P, z = load_model_fixture('c2_mini')
    cfg = config_from_shape(kw)
    inputs = (torch.tensor(z['feats'], dtype=torch.float32, device=dev), torch.tensor(z['labels'], device=dev),
              torch.tensor(z['inp_len'], dtype=torch.int32), torch.tensor(z['tar_len'], device=dev))

    def build():
        m = SequenceRouter(cfg, None, sh.class_n, device=dev, seed=1234)
        m.load_params(P)
        m.dropout_enabled = False
        return m

    def check(model, what):
        torch.cuda.synchronize()
        out[what] = [list(map(str, b)) for b in
                     gradient_mismatches(z, lambda p: model.P(p).grad.detach().cpu().double().numpy())]

    m0 = build()
    trainer_sr.process_train_step(4, inputs, m0, train_helper.get_optimizer(cfg), None, None, 1, sh.class_n - 1,
                                  None)
    check(m0, 'flat_bad')
    m1 = build()
    b = trainer_sr.use_grad_buckets(m1, bucket_mb=0.05, force=True)
    out['n_buckets'] = len(b.buckets)
    trainer_sr.process_train_step(4, inputs, m1, train_helper.get_optimizer(cfg), None, None, 1, sh.class_n - 1,
                                  None)
    check(m1, 'bucketed_bad')
    out['launched_collectives'] = len(b.buckets)
    m2 = build()
    trainer_sr.use_grad_buckets(m2, bucket_mb=0.05, force=True)
    g = trainer_sr.GraphedTrainStep(4, inputs, m2, train_helper.get_optimizer(cfg), 1, sh.class_n - 1, warmup=1)
    out['captured_collectives'] = g.buckets is not None
    for p in m2.params.values():
        p.grad.fill_(float('nan'))
    g()
    check(m2, 'graphed_bad')
    g.close()
    dist.barrier()
    dist.destroy_process_group()
    print('RESULT ' + json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
