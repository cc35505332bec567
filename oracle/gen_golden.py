"""Generate the committed fixtures under tests/golden/ -- TEST INFRASTRUCTURE ONLY.

Run in the build container (needs /root/reference for the flag fixtures):
    python -m oracle.gen_golden

* flags_*.json: argv -> parsed namespace produced by the REFERENCE parser
  (tfsr/helper/common_helper.py, TF-free, imported read-only from
  /root/reference).  The two .conf inputs are copied next to them as data.
* model_*.npz: SRF forward fixtures from the numpy float64 oracle
  (parity vs TF unpinned: TensorFlow is not installed), cross-checked at
  generation time against the float64 torch mirror; gradients from the mirror.
"""
import json
import os
import shutil
import sys
import tempfile

import numpy as np
import torch

from . import naive_mirror as nm
from . import srf_oracle as so

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, 'tests', 'golden')
REF = '/root/reference'

FLAG_CASES = {
    # train_srf_timit.sh:45-65 with the script defaults overridden to BASELINE C2
    'timit_c2': ['--config=timit.conf', '--train-lr-param-k=0.5', '--train-batch-frame=7000',
                 '--train-warmup-n=1200', '--train-es-tolerance=27', '--train-max-epoch=27',
                 '--model-caps-primary-num=8', '--model-caps-convolution-num=8', '--model-caps-primary-dim=16',
                 '--model-caps-convolution-dim=16', '--model-caps-class-dim=16', '--model-caps-type=naive',
                 '--model-caps-window-lpad=4', '--model-caps-window-rpad=4', '--model-caps-context=false',
                 '--model-caps-iter=3', '--model-encoder-num=3'],
    # train_srf_wsj.sh:36-54 (BASELINE C3: SDR)
    'wsj_c3': ['--config=wsj.conf', '--train-lr-param-k=0.6', '--train-es-tolerance=15', '--train-max-epoch=15',
               '--model-caps-type=naive', '--model-caps-primary-num=16', '--model-caps-convolution-num=16',
               '--model-caps-primary-dim=32', '--model-caps-convolution-dim=32', '--model-caps-class-dim=32',
               '--model-caps-window-lpad=2', '--model-caps-window-rpad=2', '--model-caps-context=True',
               '--model-caps-iter=3', '--model-encoder-num=6'],
    'defaults_only': ['--model-caps-type=naive'],
    'buckets': ['--config=timit.conf', '--train-batch-buckets="[241, 391, 541]"', '--train-batch-dynamic=false',
                '--model-caps-context=no'],
}

MODEL_CASES = {
    # name: (SrfShape kwargs, B, lengths, label_len, seed)
    'c1_mini': (dict(feat_dim=123, enc_num=1, iters=1, lpad=0, rpad=0, ph=4, pd=8, ch=4, cd=8, vd=8,
                     class_n=63, context=False), 2, [41, 30], [6, 4], 11),
    'c2_mini': (dict(feat_dim=123, enc_num=3, iters=3, lpad=4, rpad=4, ph=8, pd=16, ch=8, cd=16, vd=16,
                     class_n=63, context=False), 2, [37, 29], [5, 3], 12),
    'c3_mini_sdr': (dict(feat_dim=123, enc_num=2, iters=3, lpad=2, rpad=2, ph=4, pd=8, ch=4, cd=8, vd=8,
                         class_n=32, context=True), 2, [26, 19], [4, 2], 13),
    # the other two reference variants (trainer_sr.py:188-199), C2-shaped but smaller
    'c2_mini_einsum': (dict(feat_dim=123, enc_num=2, iters=3, lpad=2, rpad=2, ph=8, pd=8, ch=8, cd=8, vd=8,
                            class_n=63, context=False, caps_type='einsum'), 2, [37, 29], [5, 3], 14),
    'c2_mini_lowmemory': (dict(feat_dim=123, enc_num=2, iters=3, lpad=2, rpad=2, ph=8, pd=8, ch=8, cd=8, vd=8,
                               class_n=63, context=False, caps_type='lowmemory'), 2, [37, 29], [5, 3], 15),
    'c3_mini_sdr_lowmemory': (dict(feat_dim=123, enc_num=2, iters=3, lpad=2, rpad=2, ph=4, pd=8, ch=4, cd=8, vd=8,
                                   class_n=32, context=True, caps_type='lowmemory'), 2, [26, 19], [4, 2], 16),
    # C4-shaped DR (DIM 32, WSJ classes): the din-32 split-fp16 routing path, with two
    # row tiles per wave in the inner layer (J*dout = 128) and four in the last (1024)
    'c4_mini': (dict(feat_dim=123, enc_num=2, iters=3, lpad=2, rpad=2, ph=4, pd=32, ch=4, cd=32, vd=32,
                     class_n=32, context=False), 2, [34, 27], [4, 3], 17),
}


def gen_flags():
    sys.path.insert(0, REF)
    from tfsr.helper.common_helper import Logger, ParseOption  # reference parser, read-only
    logger = Logger(name='golden', level=Logger.CRITICAL).logger
    for conf in ('timit.conf', 'wsj.conf'):
        shutil.copy(os.path.join(REF, 'egs', 'conf', conf), os.path.join(GOLD, conf))
    base = tempfile.mkdtemp()
    for name, argv in FLAG_CASES.items():
        full = ['prog', '--path-base=' + base] + [a.replace('--config=', '--config=' + GOLD + '/') for a in argv]
        args = vars(ParseOption(full, logger, is_print_opts=False).args)
        args['path_base'] = '<BASE>'
        if args.get('config'):
            args['config'] = os.path.basename(args['config'])
        with open(os.path.join(GOLD, f'flags_{name}.json'), 'w') as fh:
            json.dump({'argv': argv, 'parsed': args}, fh, indent=1, sort_keys=True)


def gen_models(only=()):
    for name, (kw, B, lens, tlens, seed) in MODEL_CASES.items():
        if only and name not in only:
            continue
        sh = so.SrfShape(**kw)
        P = so.init_params(sh, seed=seed)
        rng = np.random.default_rng(seed + 100)
        T = max(lens)
        feats = rng.standard_normal((B, T, sh.feat_dim))
        for b, l in enumerate(lens):
            feats[b, l:] = 0.0   # padded_batch zero padding (load_speech_data.py:151-156)
        inp_len = np.array(lens, dtype=np.int32)
        tar_len = np.array(tlens, dtype=np.int32)
        L = max(tlens)
        labels = np.zeros((B, L), dtype=np.int32)
        for b, l in enumerate(tlens):
            labels[b, :l] = rng.integers(1, sh.class_n - 1, size=l)
        logits = so.srf_forward(P, sh, feats, inp_len)
        nll = so.ctc_batch(logits, labels, inp_len, tar_len, sh.class_n)
        greedy = so.greedy_decode(logits, np.ceil(inp_len / 4).astype(int), sh.class_n - 1)
        # gradients of loss = sum(nll)/B from the float64 torch mirror
        m = nm.NaiveMirror(sh, P)
        lt = m(torch.tensor(feats), torch.tensor(inp_len))
        assert np.abs(lt.detach().numpy() - logits).max() < 1e-10, 'oracle/mirror disagree'
        pe = nm.ctc_per_utt(lt, torch.tensor(labels), torch.tensor(inp_len), torch.tensor(tar_len), sh.class_n)
        assert np.abs(pe.detach().numpy() - nll).max() < 1e-9, 'ctc oracle/torch disagree'
        (pe.sum() / B).backward()
        # no gradient (lowmemory DR W/b, unused by the graph): TF's apply_gradients skips them, stored as 0
        grads = {'grad.' + k.replace('__', '.'): (p.grad.numpy() if p.grad is not None else np.zeros(p.shape))
                 for k, p in m.p.items()}
        out = {'shape_json': np.array(json.dumps(kw)), 'feats': feats, 'inp_len': inp_len, 'labels': labels,
               'tar_len': tar_len, 'logits': logits, 'nll': nll,
               'greedy_json': np.array(json.dumps(greedy))}
        # parameters are regenerated from the seed by the tests (so.init_params);
        # per-parameter checksums pin that regeneration, gradients kept in fp32.
        out['seed'] = np.array(seed)
        out.update({'psum.' + k: np.array([v.sum(), np.square(v).sum()]) for k, v in P.items()})
        out.update({k: v.astype(np.float32) for k, v in grads.items()})
        np.savez_compressed(os.path.join(GOLD, f'model_{name}.npz'), **out)
        print(name, logits.shape, nll)


if __name__ == '__main__':
    os.makedirs(GOLD, exist_ok=True)
    only = sys.argv[1:]   # optional model case names: regenerate just those
    if not only:
        gen_flags()
    gen_models(only)
