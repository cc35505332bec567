"""CPU checks of the oracle itself (no GPU): the numpy float64 restatement and
the torch mirror must reproduce the committed golden fixtures and each other,
the CTC restatement must match torch's, and the backward of the mirror must
match finite differences."""
import numpy as np
import pytest
import torch

from oracle import naive_mirror as nm
from oracle import srf_oracle as so
from tests.helpers import load_model_fixture


@pytest.mark.parametrize('name', ['c1_mini', 'c2_mini', 'c3_mini_sdr'])
def test_oracle_reproduces_fixture(name):
    kw, sh, P, z = load_model_fixture(name)
    logits = so.srf_forward(P, sh, z['feats'], z['inp_len'])
    assert np.abs(logits - z['logits']).max() < 1e-9
    nll = so.ctc_batch(logits, z['labels'], z['inp_len'], z['tar_len'], sh.class_n)
    assert np.abs(nll - z['nll']).max() < 1e-8
    assert so.greedy_decode(logits, np.ceil(z['inp_len'] / 4).astype(int), sh.class_n - 1) == z['greedy']


def test_mirror_matches_oracle_sdr_and_dr():
    for ctx in (False, True):
        sh = so.SrfShape(enc_num=2, iters=2, lpad=1, rpad=2, ph=4, pd=8, ch=4, cd=8, vd=8, class_n=9, context=ctx)
        P = so.init_params(sh, seed=5)
        rng = np.random.default_rng(6)
        feats = rng.standard_normal((2, 23, 123))
        inp_len = np.array([23, 17])
        feats[1, 17:] = 0
        a = so.srf_forward(P, sh, feats, inp_len)
        b = nm.NaiveMirror(sh, P)(torch.tensor(feats), torch.tensor(inp_len)).detach().numpy()
        assert np.abs(a - b).max() < 1e-10


def test_same_padding_rule():
    # TF 'SAME': pad_before = total // 2
    assert so.same_pad(123, 3, 2) == (62, 1, 1)
    assert so.same_pad(62, 3, 2) == (31, 0, 1)
    assert so.same_pad(320, 3, 2) == (160, 0, 1)
    assert so.same_pad(37, 3, 2) == (19, 1, 1)
    assert so.same_pad(80, 3, 1) == (80, 1, 1)


def test_dr_mask_makes_capsule0_exactly_zero():
    rng = np.random.default_rng(0)
    u = rng.standard_normal((1, 3, 5, 4, 8))
    v = so.dynamic_routing(u, 3, True)
    assert np.all(v[..., 0, :] == 0.0)


def test_ctc_oracle_matches_torch_with_repeats_and_blank_last():
    rng = np.random.default_rng(1)
    C, T = 7, 12
    logits = rng.standard_normal((2, T, C))
    labels = np.array([[1, 1, 2, 3], [4, 5, 5, 0]])
    tl = np.array([4, 3])
    il = np.array([T * 4, 9 * 4])
    ours = so.ctc_batch(logits, labels, il, tl, C)
    ref = nm.ctc_per_utt(torch.tensor(logits), torch.tensor(labels), torch.tensor(il), torch.tensor(tl), C).numpy()
    assert np.abs(ours - ref).max() < 1e-10


def test_ctc_infeasible_is_inf():
    logits = np.zeros((3, 5))
    assert np.isinf(so.ctc_nll(logits, np.array([1, 1, 1]), 4))   # needs >= 5 frames


def test_mirror_gradient_finite_difference():
    sh = so.SrfShape(enc_num=1, iters=2, lpad=1, rpad=0, ph=2, pd=8, ch=2, cd=8, vd=8, class_n=5, nfilt=4)
    P = so.init_params(sh, seed=3)
    rng = np.random.default_rng(4)
    feats = rng.standard_normal((1, 9, 123))
    inp_len = np.array([9])
    m = nm.NaiveMirror(sh, P)
    out = m(torch.tensor(feats), torch.tensor(inp_len))
    wvec = torch.tensor(rng.standard_normal(out.shape))
    (out * wvec).sum().backward()
    g = m.P('W0').grad.numpy().copy()
    idx = (1, 3, 2, 5)
    eps = 1e-6
    for sgn in (1, -1):
        P2 = dict(P)
        P2['W0'] = P['W0'].copy()
        P2['W0'][idx] += sgn * eps
        val = (so.srf_forward(P2, sh, feats, inp_len) * wvec.numpy()).sum()
        if sgn == 1:
            plus = val
        else:
            minus = val
    fd = (plus - minus) / (2 * eps)
    assert abs(fd - g[idx]) < 1e-6 * max(1.0, abs(fd))
