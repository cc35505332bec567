"""Graphed training steps only (for rocprofv3 --kernel-trace): python scripts/stepprof.py [workload] [steps].
Pair with scripts/stepbreak.py to get the per-step kernel breakdown."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from srf_amd import train_helper, trainer_sr  # noqa: E402
from srf_amd.sequence_router import SequenceRouter  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else 'timit_c2'
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dev = torch.device('cuda:0')
kw, class_n, B, T = bench.WORKLOADS[wl]
cfg = bench.make_config(kw)
model = SequenceRouter(cfg, None, class_n, device=dev, seed=1234)
opt = train_helper.get_optimizer(cfg)
batch = bench.synthetic_batch(B, T, class_n, 0, dev)
trainer_sr.process_train_step(4, batch, model, opt, None, None, 1, class_n - 1, None)
g = trainer_sr.GraphedTrainStep(4, batch, model, opt, 1, class_n - 1)
for _ in range(3):
    g()
torch.cuda.synchronize()
for _ in range(steps):
    g()
torch.cuda.synchronize()
print('done', wl, steps)
