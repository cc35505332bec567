"""Cost of the bucketed all-reduce inside the captured step at world size 1 (RCCL
group of one, GradBuckets(force=True)) against the flat all-reduce after the replay:
the collectives are trivial at world 1, so any difference is how the captured
multi-stream step executes.
    python scripts/dbg/bucket_capture.py [--workload wsj_c4] [--steps 10]"""
import argparse
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--workload', default='wsj_c4')
    ap.add_argument('--steps', type=int, default=10)
    a = ap.parse_args()
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29531')
    dev = torch.device('cuda:0')
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=dev)
    from srf_amd import train_helper, trainer_sr
    from srf_amd.sequence_router import SequenceRouter
    kw, class_n, B, T = bench.WORKLOADS[a.workload]
    cfg = bench.make_config(kw)
    batch = bench.synthetic_batch(B, T, class_n, 0, dev)
    for mode in ('flat', 'bucketed', 'flat', 'bucketed'):
        model = SequenceRouter(cfg, None, class_n, device=dev, seed=1234)
        if mode == 'bucketed':
            trainer_sr.use_grad_buckets(model, 25.0, force=True)
        opt = train_helper.get_optimizer(cfg)
        ls, fs, sm = trainer_sr.Mean(), trainer_sr.Mean(), trainer_sr.Sum()
        for _ in range(2):
            trainer_sr.process_train_step(4, batch, model, opt, ls, fs, 1, class_n - 1, sm)
        g = trainer_sr.GraphedTrainStep(4, batch, model, opt, 1, class_n - 1)
        for _ in range(3):
            g(ls, fs, sm)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.steps):
            g(ls, fs, sm)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / a.steps * 1e3
        print('%-9s %.3f ms/step' % (mode, ms), flush=True)
        g.close()
        del g, model, opt
        torch.cuda.empty_cache()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
