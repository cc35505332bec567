"""Replays one captured training step (fwd + CTC + bwd, GraphedTrainStep's graph) many
times and compares every replay's gradient with the first eager step's, parameter by
parameter: a cross-stream race inside the graph shows as a replay whose gradient
differs.  World size 1 (the all-reduce is not part of the graph).

    python scripts/dbg/graph_race.py FIXTURE [REPLAYS] [--side]
(--side: the DR gW and CNN-FE wgrad launches on a side stream, ops.DR_GW_SIDE)
Prints one line per replay differing by more than 1e-4 relative and a summary line."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    from srf_amd import train_helper, trainer_sr
    from srf_amd.sequence_router import SequenceRouter
    from tests.helpers import config_from_shape, load_model_fixture

    from srf_amd import ops
    args = [a for a in sys.argv[1:] if not a.startswith('--')]
    name = args[0]
    n = int(args[1]) if len(args) > 1 else 100
    if '--cnnfe-inline' in sys.argv:
        ops.CNNFE_WGRAD_SIDE = False
    if '--gw-inline' in sys.argv:
        ops.DR_GW_SIDE = False
    dev = torch.device('cuda:0')
    kw, sh, P, z = load_model_fixture(name)
    cfg = config_from_shape(kw)
    model = SequenceRouter(cfg, None, sh.class_n, device=dev, seed=1234)
    model.load_params(P)
    model.dropout_enabled = False
    inputs = (torch.tensor(z['feats'], dtype=torch.float32, device=dev), torch.tensor(z['labels'], device=dev),
              torch.tensor(z['inp_len'], dtype=torch.int32), torch.tensor(z['tar_len'], device=dev))
    g = trainer_sr.GraphedTrainStep(4, inputs, model, train_helper.get_optimizer(cfg), 1, sh.class_n - 1, warmup=1)
    names = list(model.params.keys())
    ref = None
    bad, worst = 0, 0.0
    for k in range(n):
        model.flat_grad.fill_(float('nan'))
        g.graph.replay()
        torch.cuda.synchronize()
        cur = {p: model.P(p).grad.detach().clone() for p in names}
        if ref is None:
            ref = cur
            continue
        # float atomics reorder sums between replays: flag only differences far above
        # rounding (a race shows percent-level errors)
        diff = [(p, float((cur[p] - ref[p]).abs().max() / ref[p].abs().max().clamp_min(1e-30))) for p in names]
        worst = max(worst, max(d for _, d in diff))
        diff = [(p, d) for p, d in diff if not d <= 1e-4]
        if diff:
            bad += 1
            print(f'replay {k}: ' + ', '.join(f'{p} {d:.3g}' for p, d in diff[:6]), flush=True)
    print(f'SUMMARY {name} {sys.argv[3:]}: {bad} of {n - 1} replays differ from the first; max {worst:.3g}',
          flush=True)


if __name__ == '__main__':
    main()
