"""Data parallelism on the real model: two replica processes share
cuda:0 over gloo (the 8-GPU RCCL node is the driver's; the step code is the same,
only the process-group backend differs).  Each runs tests/dp_worker.py on its
slice of a world-2 DP fixture (oracle/gen_golden.py DP_CASES), eager and graphed.

Checked: the all-reduced flat gradient equals the fixture's -- the SUM over
replicas of sum(nll_local) / (B_local * n_gpus) gradients, each replica cropped to
its own longest utterance with its own BN batch statistics, as MirroredStrategy
computes it (trainer_sr.py:58-71) -- at the model-test tolerance
(2e-3 * max|ref| + 1e-5 per parameter); per-replica NLL within 1e-4; and the
replicas draw different dropout masks (equal logits with dropout off, different
with it on).  The bucketed all-reduce (trainer_sr.GradBuckets, issued from the
backward's tensor hooks) gives the flat form's gradient.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize('name', ['dp2_c2_mini', 'dp2_c4_mini'])
def test_two_replicas_allreduce_to_fixture_gradient(cuda, name):
    world = 2
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR='127.0.0.1',
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, '-u', os.path.join(HERE, 'dp_worker.py'), name], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            o, _ = p.communicate(timeout=240)
            outs.append((p.returncode, o))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    res = []
    for rc, o in outs:
        assert rc == 0, o[-3000:]
        line = [ln for ln in o.splitlines() if ln.startswith('RESULT ')]
        assert line, o[-3000:]
        res.append(json.loads(line[-1][7:]))
    res.sort(key=lambda d: d['rank'])
    assert [d['B_local'] for d in res] == [2, 2]
    for d in res:
        assert d['nll_err'] <= 1e-4, d
        assert not d['eager_bad'], d['eager_bad']
        assert not d['graphed_bad'], d['graphed_bad']
        assert d['n_buckets'] > 2 and not d['bucketed_bad'], d
        assert d['bucketed_vs_flat'] <= 1e-6, d
        assert d['graphed_bucket_fallback'], d
        assert d['dropout_off_equal'], d
        assert d['dropout_on_differs'], d
    assert res[0]['seed_base'] != res[1]['seed_base']


def test_rccl_world1_flat_bucketed_and_captured():
    """The nccl (RCCL) process group and its collectives, at world size 1 in a child
    process (tests/rccl_worker.py): flat, bucketed-from-the-backward and
    graph-captured bucketed all-reduce all leave the fixture's gradient."""
    env = dict(os.environ, RANK='0', WORLD_SIZE='1', LOCAL_RANK='0', MASTER_ADDR='127.0.0.1',
               MASTER_PORT=str(_free_port()))
    p = subprocess.run([sys.executable, '-u', os.path.join(HERE, 'rccl_worker.py')], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith('RESULT ')]
    assert line, p.stdout[-3000:]
    d = json.loads(line[-1][7:])
    assert d['backend'] == 'nccl' and d['world'] == 1, d
    assert d['n_buckets'] > 2, d
    assert not d['flat_bad'] and not d['bucketed_bad'] and not d['graphed_bad'], d
    assert d['captured_collectives'], d
