"""Optimizer, LR schedule and length bucketing (tfsr/helper/train_helper.py)."""
import ctypes
import math

import numpy as np
import torch

from . import _lib


class CustomSchedule:
    """train_helper.py:32-57: lr(step) = min(k * rsqrt(d_model) * min(step^-0.5,
    step * warmup^-1.5), max_lr).  Note lr(0) == 0."""

    def __init__(self, train_lr_param_k, d_model, warmup_steps, max_lr=10):
        self.train_lr_param_k = train_lr_param_k
        self.d_model = float(d_model)
        self.warmup_steps = warmup_steps
        self.max_lr = max_lr

    def __call__(self, step):
        step = float(step)
        arg1 = math.inf if step == 0 else 1.0 / math.sqrt(step)
        arg2 = step * self.warmup_steps ** -1.5
        return min(self.train_lr_param_k / math.sqrt(self.d_model) * min(arg1, arg2), self.max_lr)

    def get_config(self):
        return {'model_dimension': self.d_model, 'train_lr_param_k': self.train_lr_param_k,
                'warmup_steps': self.warmup_steps}


class SrfAdam:
    """Keras Adam (train_helper.py:60-70) over a model's flat parameter buffer,
    applied by one fused HIP launch (srf_adam_step).  The schedule is evaluated at
    the 0-based iteration count, the bias correction at iterations + 1, as Keras'
    OptimizerV2 does."""

    def __init__(self, learning_rate, beta_1=0.9, beta_2=0.98, epsilon=1e-9):
        self.lr = learning_rate
        self.beta_1, self.beta_2, self.epsilon = beta_1, beta_2, epsilon
        self.iterations = 0
        self._m = self._v = None

    def current_lr(self):
        return self.lr(self.iterations) if callable(self.lr) else float(self.lr)

    def apply_gradients(self, model):
        if self._m is None:
            self._m = torch.zeros_like(model.flat_params)
            self._v = torch.zeros_like(model.flat_params)
        lr = self.current_lr()
        t = self.iterations + 1
        alpha = lr * math.sqrt(1 - self.beta_2 ** t) / (1 - self.beta_1 ** t)
        vp = ctypes.c_void_p
        rc = _lib.lib().srf_adam_step(vp(model.flat_params.data_ptr()), vp(model.flat_grad.data_ptr()),
                                      vp(self._m.data_ptr()), vp(self._v.data_ptr()), model.n_flat, alpha,
                                      self.beta_1, self.beta_2, self.epsilon,
                                      vp(torch.cuda.current_stream().cuda_stream))
        _lib.check(rc, 'srf_adam_step')
        self.iterations += 1


def get_optimizer(config):
    """train_helper.py:60-75 (the SRF scripts use the default branch)."""
    if config.train_opti_type is None or config.train_opti_type not in ('adam', 'sgd'):
        sched = CustomSchedule(config.train_lr_param_k, config.model_dimension, config.train_warmup_n,
                               config.train_lr_max)
        return SrfAdam(sched, config.train_adam_beta1, config.train_adam_beta2, config.train_adam_epsilon)
    if config.train_opti_type == 'adam':
        return SrfAdam(config.train_lr_param_k)
    raise NotImplementedError('sgd is not on the SRF path')


def get_bucket_info(batch_total_size, num_gpus, min_bkt, max_bkt, step, step_for_bucket_size=False,
                    manual_bucket_batch_sizes=None):
    """train_helper.py:269-320: (bucket_boundaries, bucket_batch_sizes) for
    length bucketing with ~batch_total_size frames per global batch."""
    bounds, sizes = [], []
    if step_for_bucket_size and manual_bucket_batch_sizes is None:
        for bs in range(int(np.floor(batch_total_size / min_bkt)), num_gpus, -step):
            boundary = int(np.floor(batch_total_size / bs))
            if bs <= num_gpus:
                break
            sizes.append(bs)
            bounds.append(min(boundary, max_bkt))
            if boundary >= max_bkt:
                break
    else:
        cands = manual_bucket_batch_sizes if manual_bucket_batch_sizes else range(min_bkt, max_bkt + step, step)
        for boundary in cands:
            bs = int(np.floor(batch_total_size / boundary))
            if bs <= num_gpus:
                break
            sizes.append(bs)
            bounds.append(boundary)
    sizes.append(num_gpus)
    # drop buckets whose batch size repeats the next one's (train_helper.py:311-318)
    prev = -1
    for i in reversed(range(len(bounds))):
        if sizes[i] == prev:
            bounds.pop(i)
            sizes.pop(i)
        prev = sizes[i]
    return bounds, sizes
