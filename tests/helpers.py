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
    """Returns (shape kwargs, oracle params, arrays) with params regenerated
    from the fixture seed and verified against the stored checksums."""
    from oracle import srf_oracle as so
    z = np.load(os.path.join(GOLD, f'model_{name}.npz'), allow_pickle=False)
    kw = json.loads(str(z['shape_json']))
    sh = so.SrfShape(**kw)
    P = so.init_params(sh, seed=int(z['seed']))
    for k, v in P.items():
        ref = z['psum.' + k]
        got = np.array([v.sum(), np.square(v).sum()])
        assert np.allclose(got, ref, rtol=1e-12, atol=1e-12), f'param regeneration drifted for {k}'
    arrays = {k: z[k] for k in z.files}
    arrays['greedy'] = json.loads(str(z['greedy_json']))
    return kw, sh, P, arrays
