"""Checkpoints of the SRF path: TF object-graph names, manager, averaging.

Mirrors the reference's checkpoint surface:
  * ``tf.train.Checkpoint(optimizer=optimizer, model=model)`` +
    ``tf.train.CheckpointManager`` with ``ckpt-N`` prefixes and the ``checkpoint``
    state file, ``load_checkpoint`` returning (manager, epoch_offset)
    (tfsr/helper/misc_helper.py:139-163);
  * checkpoint averaging of the last ``model_average_num`` checkpoints into
    ``path_ckpt/avg`` (tfsr/utils/average_ckpt_sr.py:100-179).

Every tensor is stored under the key TF2's object-based checkpoint would give
it (``model/<attribute path>/.ATTRIBUTES/VARIABLE_VALUE``, optimizer slots as
``.../.OPTIMIZER_SLOT/optimizer/{m,v}/...``), following the attribute names of
sequence_router_naive.py:68-118 and sequence_router.py:44-63, so a checkpoint
converts to or from a TF bundle by renaming nothing.  Files are TF TensorBundles
by default -- ``ckpt-N.index`` + ``ckpt-N.data-00000-of-00001``, the layout
tf.train.CheckpointManager writes, through tf_bundle.py -- or safetensors
(``ckpt-N.srf.safetensors``, ``fmt='safetensors'``); readers take either.

Parity note: TensorFlow is not installed here, so the key scheme restates TF2's
documented object-path convention; no TF-written checkpoint ships in the
reference to pin it (parity unpinned).
"""
import os
import re

import numpy as np
import torch

from safetensors.numpy import load_file, save_file

VALUE = '.ATTRIBUTES/VARIABLE_VALUE'
SAVE_COUNTER = 'save_counter/' + VALUE


def tf_variable_map(model):
    """our parameter / buffer name -> (TF object path, TF shape).

    CapsulationLayer keeps conv_layers[j][k] and uses conv_layers[0][k] and
    conv_layers[1][k] for the two maxout halves of conv stage k
    (sequence_router.py:52-60, 76-77): ours conv{k}a / conv{k}b.
    W%d / b%d carry the reference's leading (1, 1) and trailing 1 axes
    (naive:97-103); the einsum variant stores W as (in, out, od, id) and the bias as
    (1, 1, in, out, od) (einsum:93-97), lowmemory as (1, in, out, od, id) and
    (1, in, out, od, 1) (lowmemory:94-98).  Same values in the same order."""
    caps_type = getattr(model, 'caps_type', 'naive')
    m = {}
    for k in range(model.cnn_n):
        for j, ab in enumerate('ab'):
            for t in ('kernel', 'bias'):
                m[f'conv{k}{ab}_{t}'] = (f'model/conv/conv_layers/{j}/{k}/{t}/{VALUE}', None)
        for t in ('gamma', 'beta'):
            m[f'bn{k}_{t}'] = (f'model/conv/bn_layers/{k}/{t}/{VALUE}', None)
        m[f'bn{k}_moving_mean'] = (f'model/conv/bn_layers/{k}/moving_mean/{VALUE}', None)
        m[f'bn{k}_moving_var'] = (f'model/conv/bn_layers/{k}/moving_variance/{VALUE}', None)
    for t in ('kernel', 'bias'):
        m[f'proj_{t}'] = (f'model/proj_pe/{t}/{VALUE}', None)
        for e in (1, 2):
            m[f'encaps{e}_{t}'] = (f'model/ecs/{e - 1}/{t}/{VALUE}', None)
    for t in ('gamma', 'beta'):
        m[f'ln_input_{t}'] = (f'model/ln_i/{t}/{VALUE}', None)
        m[f'ln_output_{t}'] = (f'model/ln_o/{t}/{VALUE}', None)
    for l, (in_n, out_n, out_d, in_d) in enumerate(model.layer_shapes):
        if caps_type == 'einsum':
            ws, bs = (in_n, out_n, out_d, in_d), (1, 1, in_n, out_n, out_d)
        elif caps_type == 'lowmemory':
            ws, bs = (1, in_n, out_n, out_d, in_d), (1, in_n, out_n, out_d, 1)
        else:
            ws, bs = (1, 1, in_n, out_n, out_d, in_d), (1, 1, in_n, out_n, out_d, 1)
        m[f'W{l}'] = (f'model/wgt/{l}/{VALUE}', ws)
        m[f'b{l}'] = (f'model/bias/{l}/{VALUE}', bs)
        for t in ('gamma', 'beta'):
            m[f'ln_mid{l + 1}_{t}'] = (f'model/ln_m/{l}/{t}/{VALUE}', None)
    return m


def _slot_key(tf_key, slot):
    return tf_key.replace(VALUE, f'.OPTIMIZER_SLOT/optimizer/{slot}/{VALUE}')


def model_state(model, overrides=None):
    """All model tensors (parameters + BN moving statistics) under TF names.
    ``overrides`` maps our names to tensors saved in place of the model's own (the
    replica-mean BN moving statistics of trainer_sr.replica_mean_moving_statistics)."""
    out = {}
    overrides = overrides or {}
    for name, (key, shape) in tf_variable_map(model).items():
        t = overrides.get(name)
        if t is None:
            t = model.params[name] if name in model.params else getattr(model, name)
        a = t.detach().cpu().numpy().astype(np.float32)
        out[key] = a.reshape(shape) if shape else a
    return out


def load_model_state(model, state, strict=True):
    """Inverse of model_state; returns the TF keys it did not use."""
    used = set()
    with torch.no_grad():
        for name, (key, _) in tf_variable_map(model).items():
            if key not in state:
                if strict:
                    raise KeyError(f'checkpoint lacks {key} ({name})')
                continue
            dst = model.params[name] if name in model.params else getattr(model, name)
            src = np.asarray(state[key], np.float32)
            if src.size != dst.numel():
                raise ValueError(f'{key}: {src.shape} does not fit {tuple(dst.shape)}')
            dst.copy_(torch.from_numpy(src.reshape(tuple(dst.shape))).to(dst.device))
            used.add(key)
    return sorted(set(state) - used)


def optimizer_state(model, optimizer):
    out = {'optimizer/iter/' + VALUE: np.array(optimizer.iterations, np.int64)}
    if optimizer._m is not None:
        for name, (key, shape) in tf_variable_map(model).items():
            if name not in model.offsets:
                continue
            off, n = model.offsets[name], model.params[name].numel()
            for slot, buf in (('m', optimizer._m), ('v', optimizer._v)):
                a = buf[off:off + n].detach().cpu().numpy()
                out[_slot_key(key, slot)] = a.reshape(shape) if shape else a.reshape(tuple(model.params[name].shape))
    return out


def load_optimizer_state(model, optimizer, state):
    key_iter = 'optimizer/iter/' + VALUE
    if key_iter in state:
        optimizer.iterations = int(np.asarray(state[key_iter]).reshape(-1)[0])
    slots = [k for k in state if '.OPTIMIZER_SLOT/' in k]
    if not slots:
        return
    optimizer._m = torch.zeros_like(model.flat_params)
    optimizer._v = torch.zeros_like(model.flat_params)
    for name, (key, _) in tf_variable_map(model).items():
        if name not in model.offsets:
            continue
        off, n = model.offsets[name], model.params[name].numel()
        for slot, buf in (('m', optimizer._m), ('v', optimizer._v)):
            sk = _slot_key(key, slot)
            if sk in state:
                buf[off:off + n].copy_(torch.from_numpy(np.asarray(state[sk], np.float32).reshape(-1)))


class CheckpointManager:
    """tf.train.CheckpointManager(ckpt, directory, max_to_keep): ``ckpt-N``
    prefixes, N = save counter; the ``checkpoint`` text file lists them like TF's
    CheckpointState (model_checkpoint_path / all_model_checkpoint_paths).

    ``save_counter`` is tf.train.Checkpoint's save_counter: 0 for a fresh
    checkpoint object, set by a restore to the value stored in the restored
    checkpoint, and advanced by one on every save, which numbers the file unless
    an explicit checkpoint_number is given.  Resuming from ckpt-3 while ckpt-5
    exists therefore writes ckpt-4 next, as TF does."""

    SUFFIX = '.srf.safetensors'
    FORMATS = ('tf', 'safetensors')

    def __init__(self, model, optimizer, directory, max_to_keep=5, fmt='tf'):
        if fmt not in self.FORMATS:
            raise ValueError(f'checkpoint format must be one of {self.FORMATS}')
        self.model, self.optimizer, self.directory = model, optimizer, directory
        self.max_to_keep = max_to_keep
        self.fmt = fmt
        self.save_counter = 0
        os.makedirs(directory, exist_ok=True)
        self._ckpts = self._read_state()

    @property
    def checkpoints(self):
        return [os.path.join(self.directory, c) for c in self._ckpts]

    @property
    def latest_checkpoint(self):
        return os.path.join(self.directory, self._ckpts[-1]) if self._ckpts else None

    def _read_state(self):
        path = os.path.join(self.directory, 'checkpoint')
        if not os.path.exists(path):
            return []
        names = re.findall(r'all_model_checkpoint_paths:\s*"([^"]+)"', open(path).read())
        return [n for n in names if checkpoint_files(os.path.join(self.directory, n))]

    def _write_state(self):
        lines = []
        if self._ckpts:
            lines.append(f'model_checkpoint_path: "{self._ckpts[-1]}"')
        lines += [f'all_model_checkpoint_paths: "{c}"' for c in self._ckpts]
        with open(os.path.join(self.directory, 'checkpoint'), 'w') as f:
            f.write('\n'.join(lines) + '\n')

    def save(self, checkpoint_number=None, overrides=None):
        """``overrides``: see model_state (data-parallel runs pass the replica-mean
        BN moving statistics, which is what a MirroredStrategy checkpoint holds).
        Raises first if a grouped SDR recurrence timed out since the last check
        (ops.check_faults): no checkpoint of parameters the run cannot vouch for."""
        fp = getattr(self.model, 'flat_params', None)
        if fp is not None and fp.is_cuda:
            from . import ops
            ops.check_faults()
        self.save_counter += 1
        n = self.save_counter if checkpoint_number is None else int(checkpoint_number)
        name = f'ckpt-{n}'
        state = model_state(self.model, overrides)
        if self.optimizer is not None:
            state.update(optimizer_state(self.model, self.optimizer))
        state[SAVE_COUNTER] = np.array(self.save_counter, np.int64)
        prefix = os.path.join(self.directory, name)
        for f in checkpoint_files(prefix):   # re-saving a number replaces it in either format
            os.remove(f)
        if self.fmt == 'tf':
            from . import tf_bundle
            tf_bundle.save_checkpoint(prefix, state)
        else:
            save_file(state, prefix + self.SUFFIX)
        self._ckpts = [c for c in self._ckpts if c != name] + [name]
        if self.max_to_keep is not None and self.max_to_keep > 0:
            while len(self._ckpts) > self.max_to_keep:
                old = self._ckpts.pop(0)
                for f in checkpoint_files(os.path.join(self.directory, old)):
                    os.remove(f)
        self._write_state()
        return prefix


def checkpoint_files(prefix):
    """The files of checkpoint ``prefix`` on disk (TF bundle or safetensors), [] if none."""
    import glob
    if os.path.exists(prefix + '.index'):
        return [prefix + '.index'] + sorted(glob.glob(glob.escape(prefix) + '.data-*-of-*'))
    if os.path.exists(prefix + CheckpointManager.SUFFIX):
        return [prefix + CheckpointManager.SUFFIX]
    return []


def read_checkpoint(prefix):
    """{TF key: array} of checkpoint ``prefix``, from a TF bundle (``.index``) or safetensors."""
    if os.path.exists(prefix + '.index'):
        from . import tf_bundle
        return tf_bundle.load_checkpoint(prefix)
    return load_file(prefix + CheckpointManager.SUFFIX)


def restore(prefix, model, optimizer=None, expect_partial=True):
    """tf.train.Checkpoint(...).restore(prefix).expect_partial(); returns the
    restored save_counter (0 when the checkpoint holds none)."""
    state = read_checkpoint(prefix)
    load_model_state(model, state, strict=not expect_partial)
    if optimizer is not None:
        load_optimizer_state(model, optimizer, state)
    return int(np.asarray(state[SAVE_COUNTER]).reshape(-1)[0]) if SAVE_COUNTER in state else 0


def load_checkpoint(config, logger, model, optimizer):
    """misc_helper.py:139-163: restore ckpt-<path_ckpt_epoch> or the latest one;
    returns (manager, epoch_offset)."""
    max_to_keep = config.model_ckpt_max_to_keep
    if max_to_keep is not None and max_to_keep < 0:
        max_to_keep = None
    manager = CheckpointManager(model, optimizer, config.path_ckpt, max_to_keep=max_to_keep)
    loaded = ''
    if config.path_ckpt_epoch is not None and config.path_ckpt_epoch > 0:
        loaded = os.path.join(config.path_ckpt, 'ckpt-%d' % config.path_ckpt_epoch)
    elif manager.latest_checkpoint:
        loaded = manager.latest_checkpoint
    if 'ckpt' in loaded:
        epoch_offset = int(loaded.split('-')[-1])
        manager.save_counter = restore(loaded, model, optimizer)
    else:
        epoch_offset = 0
        loaded = None
    if logger is not None:
        logger.info('Loaded ckpt: %s', loaded)
    return manager, epoch_offset


def average_checkpoints(config, logger, model_fn, optimizer=None):
    """average_ckpt_sr.py:91-179: element-wise mean of the model weights of the
    last ``model_average_num`` checkpoints in ``path_ckpt`` among those numbered
    <= ``train_max_epoch`` (all of them when it is 0, :91-96), saved through a
    max_to_keep=1 manager into ``path_ckpt/avg`` (replaced if present)."""
    import shutil
    ckpts = CheckpointManager(model_fn(), None, config.path_ckpt, max_to_keep=None).checkpoints
    max_epoch = getattr(config, 'train_max_epoch', 0) or 0
    ckpts = [c for c in ckpts if max_epoch == 0 or int(c.split('-')[-1]) <= max_epoch]
    chosen = ckpts[-config.model_average_num:]
    if not chosen:
        raise FileNotFoundError(f'no checkpoints in {config.path_ckpt}')
    states = []
    for c in chosen:
        if logger is not None:
            logger.info(c)
        states.append(model_state(_restored(model_fn, c)))
    if logger is not None:
        logger.info('Total %d models were loaded.', len(states))
    avg = {k: np.mean(np.stack([s[k] for s in states]), axis=0).astype(np.float32) for k in states[0]}
    model = model_fn()
    load_model_state(model, avg)
    out_dir = os.path.join(config.path_ckpt, 'avg')
    if os.path.exists(out_dir):
        shutil.rmtree(out_dir)
    path = CheckpointManager(model, optimizer, out_dir, max_to_keep=1).save()
    if logger is not None:
        logger.info('Saved to %s', path)
    return path, model


def _restored(model_fn, prefix):
    m = model_fn()
    restore(prefix, m)
    return m
