"""CTC loss and decoding at the trainer boundary (trainer_sr.py:64-66, :109-112).

``ctc_loss`` keeps tf.nn.ctc_loss's calling convention as the reference uses it
(dense labels, batch-major logits, explicit blank index) and returns the
per-utterance negative log likelihood.  This revision computes it with
the HIP kernel srf_ctc_loss (loss and logit gradient in one launch).
"""
import ctypes

import numpy as np
import torch

from . import ops


def ctc_loss(labels, logits, label_length, logit_length, logits_time_major=False, blank_index=0):
    if logits_time_major:
        logits = logits.transpose(0, 1)
    return ops.ctc_loss(logits.contiguous(), labels, label_length, logit_length, blank_index)


def ctc_loss_and_grad(labels, logits, label_length, logit_length, blank_index, grad_scale):
    """Per-utterance NLL and grad_scale * d(sum nll)/d logits from one launch
    (batch-major logits); the training step's loss head."""
    return ops.ctc_loss_and_grad(logits.contiguous(), labels, label_length, logit_length, blank_index, grad_scale)


def greedy_decode(logits, lengths, blank_index):
    """Best-path decoding: per-frame argmax, merge repeats, drop blanks.
    logits [B, T, C] batch-major; returns a list of label lists."""
    best = torch.argmax(logits, dim=-1).cpu()
    lengths = lengths.cpu()
    out = []
    for b in range(best.shape[0]):
        seq, prev = [], -1
        for k in best[b, :int(lengths[b])].tolist():
            if k != prev and k != blank_index:
                seq.append(k)
            prev = k
        out.append(seq)
    return out


def beam_search_decode(logits, lengths, blank_index, beam_width=100):
    """tf.nn.ctc_beam_search_decoder(time-major logits, lengths, beam_width,
    top_paths=1) as process_test_step calls it (trainer_sr.py:109-112), on the host
    prefix beam search of libsrf_data.so.  logits [B, T, C] batch-major (device or
    host); returns (list of label lists, numpy log probabilities)."""
    from . import load_speech_data as lsd
    L = lsd.lib()
    x = np.ascontiguousarray(logits.detach().float().cpu().numpy())
    lens = [int(v) for v in torch.as_tensor(lengths).cpu().tolist()]
    B, T, C = x.shape
    out, logp = [], np.zeros(B, np.float64)
    buf = np.zeros(max(T, 1), np.int32)
    n = ctypes.c_int()
    lp = ctypes.c_float()
    for b in range(B):
        t = max(0, min(lens[b], T))
        row = x[b]
        rc = L.srf_ctc_beam_search(row.ctypes.data, t, C, int(blank_index), int(beam_width), buf.ctypes.data,
                                   ctypes.byref(n), ctypes.byref(lp))
        if rc != 0:
            raise ValueError(f'srf_ctc_beam_search: bad argument (T={t}, C={C}, blank={blank_index}, beam={beam_width})')
        out.append(buf[:n.value].tolist())
        logp[b] = lp.value
    return out, logp
