"""Host cost of replaying a captured training step: the CPU time of graph.replay()
(returns once every node is enqueued) against the GPU time of the step, for a bench
workload.  A replay whose enqueue takes longer than the GPU needs to reach a node
starts that node late.
    python scripts/dbg/replay_cpu.py [--workload wsj_c3] [--reps 5]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--workload', default='wsj_c3')
    ap.add_argument('--reps', type=int, default=5)
    a = ap.parse_args()
    from srf_amd import train_helper, trainer_sr
    from srf_amd.sequence_router import SequenceRouter
    dev = torch.device('cuda:0')
    kw, class_n, B, T = bench.WORKLOADS[a.workload]
    cfg = bench.make_config(kw)
    model = SequenceRouter(cfg, None, class_n, device=dev, seed=1234)
    opt = train_helper.get_optimizer(cfg)
    batch = bench.synthetic_batch(B, T, class_n, 0, dev)
    ls, fs, sm = trainer_sr.Mean(), trainer_sr.Mean(), trainer_sr.Sum()
    for _ in range(2):
        trainer_sr.process_train_step(4, batch, model, opt, ls, fs, 1, class_n - 1, sm)
    g = trainer_sr.GraphedTrainStep(4, batch, model, opt, 1, class_n - 1)
    for _ in range(2):
        g(ls, fs, sm)
    torch.cuda.synchronize()
    for i in range(a.reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        g.graph.replay()
        t1 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print('replay %d: enqueue %.2f ms (host), step %.2f ms (GPU events), host until done %.2f ms'
              % (i, (t1 - t0) * 1e3, e0.elapsed_time(e1), (t2 - t0) * 1e3))
    # the same replay behind a GPU spin that outlasts the enqueue: GPU time without host stalls
    for i in range(a.reps):
        torch.cuda.synchronize()
        torch.cuda._sleep(int(30e6))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        g.graph.replay()
        t1 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        print('behind spin %d: enqueue %.2f ms (host), step %.2f ms (GPU events)'
              % (i, (t1 - t0) * 1e3, e0.elapsed_time(e1)))


if __name__ == '__main__':
    main()
