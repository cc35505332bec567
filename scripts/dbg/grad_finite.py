"""Per-parameter finiteness of one eager training-step gradient at a bench workload
(bench.py's model, init and synthetic batch; no optimizer update).
    python scripts/dbg/grad_finite.py [--workload wsj_c3]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
import bench  # noqa: E402


class _NoUpdate:
    def apply_gradients(self, model):
        pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--workload', default='wsj_c3')
    ap.add_argument('--dropout', action='store_true')
    a = ap.parse_args()
    from srf_amd import trainer_sr
    from srf_amd.sequence_router import SequenceRouter
    dev = torch.device('cuda:0')
    kw, class_n, B, T = bench.WORKLOADS[a.workload]
    cfg = bench.make_config(kw)
    model = SequenceRouter(cfg, None, class_n, device=dev, seed=1234)
    model.dropout_enabled = a.dropout
    batch = bench.synthetic_batch(B, T, class_n, 0, dev)
    for rep in range(2):
        model.flat_grad.fill_(float('nan'))
        nll = trainer_sr.process_train_step(4, batch, model, _NoUpdate(), None, None, 1, class_n - 1, None)
        torch.cuda.synchronize()
        print(f'rep {rep}: nll finite {bool(torch.isfinite(nll).all())} mean {nll.mean().item():.4f}')
        for name, p in model.params.items():
            g = p.grad
            bad = (~torch.isfinite(g)).sum().item()
            if bad or rep == 0:
                print(f'  {name:24s} {tuple(g.shape)!s:22s} nonfinite {bad:8d} max|g| '
                      f'{g[torch.isfinite(g)].abs().max().item() if bad < g.numel() else float("nan"):.3e}')
        pad = torch.ones_like(model.flat_grad, dtype=torch.bool)
        for name, p in model.params.items():
            off = model.offsets[name]
            pad[off:off + p.numel()] = False
        print(f'  padding floats {pad.sum().item()}, nonfinite there {(~torch.isfinite(model.flat_grad[pad])).sum().item()}')


if __name__ == '__main__':
    main()
