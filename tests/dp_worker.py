"""One replica of the data-parallel GPU test (tests/test_dp_gpu.py): a child
process, rank RANK of WORLD_SIZE over gloo, all on cuda:0.

It runs the real model step on its slice of a DP fixture's global batch
(srf_amd.data_helper.split_global_batch): crop to the local longest utterance,
forward, CTC with the loss scaled by 1/(B_local * n_gpus), backward, all-reduce
(SUM) of the flat gradient, Adam (trainer_sr.py:41-75 under MirroredStrategy),
eagerly and through GraphedTrainStep, and checks the all-reduced gradient against
the fixture (the sum over replicas of each replica's gradient, computed by the
float64 oracle).  It then checks that the replicas draw different dropout masks.
Prints one JSON line with its findings; exit status 0 unless it crashed.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    from srf_amd import data_helper, train_helper, trainer_sr
    from srf_amd.sequence_router import SequenceRouter
    from tests.helpers import config_from_shape, gradient_mismatches, load_model_fixture

    name = sys.argv[1]
    dist.init_process_group('gloo')
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device('cuda:0')
    torch.cuda.set_device(dev)
    kw, sh, P, z = load_model_fixture(name)
    assert int(z['world']) == world
    cfg = config_from_shape(kw)
    feats, labels, inp_len, tar_len = data_helper.split_global_batch(
        (z['feats'], z['labels'], z['inp_len'], z['tar_len']), rank, world)
    inputs = (torch.tensor(feats, dtype=torch.float32, device=dev), torch.tensor(labels, device=dev),
              torch.tensor(inp_len, dtype=torch.int32), torch.tensor(tar_len, device=dev))
    out = {'rank': rank, 'B_local': int(len(inp_len))}

    def build():
        m = SequenceRouter(cfg, None, sh.class_n, device=dev, seed=1234)
        m.load_params(P)
        m.dropout_enabled = False
        return m

    def grad_of(model):
        return lambda p: model.P(p).grad.detach().cpu().double().numpy()

    # eager process_train_step (its Adam step at lr(0) = 0 leaves the parameters)
    model = build()
    nll = trainer_sr.process_train_step(4, inputs, model, train_helper.get_optimizer(cfg), None, None, world,
                                        sh.class_n - 1, None)
    torch.cuda.synchronize()
    lo, hi = data_helper.replica_slice(len(z['inp_len']), rank, world)
    ref_nll = z['nll'][lo:hi]
    out['nll_err'] = float(np.abs(nll.cpu().double().numpy() - ref_nll).max() / max(1.0, np.abs(ref_nll).max()))
    out['eager_bad'] = [list(map(str, b)) for b in gradient_mismatches(z, grad_of(model))]

    # bucketed all-reduce issued from the backward (GradBuckets), several buckets
    modelb = build()
    b = trainer_sr.use_grad_buckets(modelb, bucket_mb=0.02)
    out['n_buckets'] = len(b.buckets)
    trainer_sr.process_train_step(4, inputs, modelb, train_helper.get_optimizer(cfg), None, None, world,
                                  sh.class_n - 1, None)
    torch.cuda.synchronize()
    out['bucketed_bad'] = [list(map(str, x)) for x in gradient_mismatches(z, grad_of(modelb))]
    out['bucketed_vs_flat'] = float((modelb.flat_grad - model.flat_grad).abs().max() /
                                    model.flat_grad.abs().max())
    # a gloo group cannot be captured: the graphed step falls back to the flat form
    gb = trainer_sr.GraphedTrainStep(4, inputs, modelb, train_helper.get_optimizer(cfg), world, sh.class_n - 1,
                                     warmup=1)
    out['graphed_bucket_fallback'] = gb.buckets is None
    gb.close()

    # the same through the captured step
    model2 = build()
    g = trainer_sr.GraphedTrainStep(4, inputs, model2, train_helper.get_optimizer(cfg), world, sh.class_n - 1,
                                    warmup=1)
    for p in model2.params.values():
        p.grad.fill_(float('nan'))
    g()
    torch.cuda.synchronize()
    out['graphed_bad'] = [list(map(str, b)) for b in gradient_mismatches(z, grad_of(model2))]
    g.close()

    # dropout: every replica runs the same utterance with dropout on; the masks
    # (hence the logits) must differ between replicas, and agree with dropout off
    x = torch.tensor(z['feats'][:1, :int(z['inp_len'][0])], dtype=torch.float32, device=dev)
    il = torch.tensor(z['inp_len'][:1], dtype=torch.int32)
    with torch.no_grad():
        model.dropout_enabled = False
        off = model(x, input_lengths=il, training=True).cpu()
        model.dropout_enabled = True
        on = model(x, input_lengths=il, training=True).cpu()
    offs = [torch.zeros_like(off) for _ in range(world)]
    ons = [torch.zeros_like(on) for _ in range(world)]
    dist.all_gather(offs, off)
    dist.all_gather(ons, on)
    out['dropout_off_equal'] = all(torch.equal(offs[0], t) for t in offs)
    out['dropout_on_differs'] = all(not torch.equal(ons[0], t) for t in ons[1:])
    out['seed_base'] = str(model._seed_base)
    dist.barrier()
    dist.destroy_process_group()
    print('RESULT ' + json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
