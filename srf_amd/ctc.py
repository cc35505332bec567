"""CTC loss and decoding at the trainer boundary (trainer_sr.py:64-66, :109-112).

``ctc_loss`` keeps tf.nn.ctc_loss's calling convention as the reference uses it
(dense labels, batch-major logits, explicit blank index) and returns the
per-utterance negative log likelihood.  This revision computes it with
torch's device CTC (a HIP CTC kernel is the next row in DESIGN.md).
"""
import torch
import torch.nn.functional as F


def ctc_loss(labels, logits, label_length, logit_length, logits_time_major=False, blank_index=0):
    if logits_time_major:
        logits = logits.transpose(0, 1)
    log_probs = torch.log_softmax(logits, dim=-1).transpose(0, 1)   # [T, B, C]
    return F.ctc_loss(log_probs, labels.long(), logit_length.long(), label_length.long(), blank=blank_index,
                      reduction='none', zero_infinity=False)


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
