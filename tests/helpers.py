"""Shared test helpers (fixture loading, config construction)."""
import argparse
import json
import os

import numpy as np

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def config_from_shape(kw, **over):
    """argparse.Namespace with the reference flag names for an SrfShape kwargs dict."""
    ns = argparse.Namespace(
        feat_dim=kw['feat_dim'], model_conv_filter_num=64, model_conv_layer_num=2, model_conv_stride=2,
        model_encoder_num=kw['enc_num'], model_caps_iter=kw['iters'], model_caps_window_lpad=kw['lpad'],
        model_caps_window_rpad=kw['rpad'], model_caps_context=kw['context'], model_caps_primary_num=kw['ph'],
        model_caps_primary_dim=kw['pd'], model_caps_convolution_num=kw['ch'], model_caps_convolution_dim=kw['cd'],
        model_caps_class_dim=kw['vd'], model_caps_type=kw.get('caps_type', 'naive'), model_initializer='fan_avg',
        train_inp_dropout=0.1, train_inn_dropout=0.1, model_dimension=1, train_lr_param_k=0.5,
        train_warmup_n=1200, train_lr_max=1e3, train_adam_beta1=0.9, train_adam_beta2=0.98,
        train_adam_epsilon=1e-9, train_opti_type=None)
    for k, v in over.items():
        setattr(ns, k, v)
    return ns


def load_model_fixture(name):
    """Returns (shape kwargs, oracle params, arrays) with params (and, for the
    full-size fixtures, feats) regenerated from the fixture seed and verified
    against the stored checksums."""
    from oracle import gen_golden as gg
    from oracle import srf_oracle as so
    z = np.load(os.path.join(GOLD, f'model_{name}.npz'), allow_pickle=False)
    kw = json.loads(str(z['shape_json']))
    sh = so.SrfShape(**kw)
    P = so.init_params(sh, seed=int(z['seed']))
    if 'w_scale' in z.files:
        P = gg.scale_w(P, float(z['w_scale']))
    for k, v in P.items():
        ref = z['psum.' + k]
        got = np.array([v.sum(), np.square(v).sum()])
        assert np.allclose(got, ref, rtol=1e-12, atol=1e-12), f'param regeneration drifted for {k}'
    arrays = {k: z[k] for k in z.files}
    if 'feats_seed' in z.files:
        feats = gg.regen_feats(int(z['feats_seed']), [int(x) for x in z['inp_len']], sh.feat_dim)
        got = np.array([feats.sum(), np.square(feats).sum()])
        assert np.allclose(got, z['feats_sum'], rtol=1e-12), 'feats regeneration drifted'
        arrays['feats'] = feats
    if 'greedy_json' in z.files:
        arrays['greedy'] = json.loads(str(z['greedy_json']))
    return kw, sh, P, arrays


def gradient_mismatches(z, grad_of, rel=2e-3, abs_=1e-5):
    """Compare a model's parameter gradients with a fixture's: full arrays
    ('grad.<name>') or seeded samples ('gidx.'/'gval.' + 'gstat.' = max|g|, L2 norm).
    Tolerance per parameter: |got - ref| <= rel * max|ref| + abs_, and for sampled
    fixtures also |norm(got) - norm(ref)| <= rel * norm(ref) + abs_.
    ``grad_of(pname)`` returns the gradient as a float64 numpy array.  Returns the
    list of (name, error, scale) that fail."""
    bad = []
    for key in z:
        if key.startswith('grad.'):
            pname = key[5:].replace('.', '_')
            ref = z[key].astype(np.float64)
            got = grad_of(pname)
            err, scale = np.abs(got - ref).max(), np.abs(ref).max()
            if err > rel * scale + abs_:
                bad.append((pname, err, scale))
        elif key.startswith('gidx.'):
            name = key[5:]
            pname = name.replace('.', '_')
            got = grad_of(pname).reshape(-1)
            ref = z['gval.' + name].astype(np.float64)
            gmax, gnorm = z['gstat.' + name]
            err = np.abs(got[z[key]] - ref).max()
            if err > rel * gmax + abs_:
                bad.append((pname, err, gmax))
            nerr = abs(np.sqrt(np.square(got).sum()) - gnorm)
            if nerr > rel * gnorm + abs_:
                bad.append((pname + ' (norm)', nerr, gnorm))
    return bad
