"""CTC prefix beam search (srf_ctc_beam_search in libsrf_data.so), the decoder of
process_test_step (trainer_sr.py:109-112, tf.nn.ctc_beam_search_decoder with
top_paths=1, blank = C-1).

Parity against TF is unpinned (TensorFlow is not importable here); the algorithm is
pinned instead by exhaustive search: with a beam wide enough to keep every prefix,
prefix beam search is exact, so its result must be the labelling of maximum CTC
probability among all labellings (each scored by an independent CTC forward), with
the same log probability.
"""
import itertools

import numpy as np
import pytest
import torch

from srf_amd import ctc


def _ctc_logp(logp, labels, blank):
    """log p(labels | x) by torch's CTC forward (independent of the decoder)."""
    T = logp.shape[0]
    lp = torch.tensor(logp, dtype=torch.float64).unsqueeze(1)
    tgt = torch.tensor([labels if labels else [0]], dtype=torch.long)
    nll = torch.nn.functional.ctc_loss(lp, tgt, torch.tensor([T]), torch.tensor([len(labels)]), blank=blank,
                                       reduction='none', zero_infinity=False)
    return -float(nll[0])


def _log_softmax(x):
    x = x - x.max(axis=-1, keepdims=True)
    return x - np.log(np.exp(x).sum(axis=-1, keepdims=True))


@pytest.mark.parametrize('seed,T,C', [(0, 4, 4), (1, 5, 3), (2, 5, 4), (3, 3, 5)])
def test_wide_beam_is_exact_map_labelling(seed, T, C):
    rng = np.random.default_rng(seed)
    logits = rng.standard_normal((1, T, C)).astype(np.float32) * 2.0
    blank = C - 1
    lp = _log_softmax(logits[0].astype(np.float64))
    best, best_lp = None, -np.inf
    for n in range(T + 1):
        for lab in itertools.product(range(C - 1), repeat=n):
            v = _ctc_logp(lp, list(lab), blank)
            if v > best_lp:
                best, best_lp = list(lab), v
    hyps, logp = ctc.beam_search_decode(torch.tensor(logits), [T], blank, beam_width=10000)
    assert hyps[0] == best
    assert abs(logp[0] - best_lp) < 1e-4


def test_beam_never_worse_than_best_path_and_respects_lengths():
    rng = np.random.default_rng(7)
    B, T, C = 4, 30, 8
    logits = torch.tensor(rng.standard_normal((B, T, C)).astype(np.float32) * 3.0)
    lens = torch.tensor([30, 17, 1, 0])
    blank = C - 1
    hyps, logp = ctc.beam_search_decode(logits, lens, blank, beam_width=16)
    greedy = ctc.greedy_decode(logits, lens, blank)
    for b in range(B):
        t = int(lens[b])
        assert len(hyps[b]) <= t and all(0 <= k < C - 1 for k in hyps[b])
        if t == 0:
            assert hyps[b] == [] and logp[b] == 0.0
            continue
        lp = _log_softmax(logits[b, :t].double().numpy())
        # the reported score is the CTC probability of the returned labelling when the
        # beam is wide, and beam search never scores below the best-path labelling
        assert _ctc_logp(lp, hyps[b], blank) >= _ctc_logp(lp, greedy[b], blank) - 1e-4


def test_beam_rejects_bad_arguments():
    with pytest.raises(ValueError):
        ctc.beam_search_decode(torch.zeros(1, 3, 4), [3], 4, beam_width=8)   # blank out of range
    with pytest.raises(ValueError):
        ctc.beam_search_decode(torch.zeros(1, 3, 4), [3], 3, beam_width=0)
