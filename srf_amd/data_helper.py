"""Dataset construction with the reference's config surface (TF-free).

Mirrors tfsr/helper/data_helper.py: get_data_len :30-47,
create_ds_for_evaluation :49-69, create_ds_for_training :71-125, on the
TFRecord pipeline of srf_amd/load_speech_data.py.
"""
import glob
import os

from . import load_speech_data
from . import train_helper as th


def _count(pattern):
    return sum(sum(1 for _ in load_speech_data.read_tfrecord(f)) for f in sorted(glob.glob(pattern)))


def get_data_len(config):
    """data_helper.py:30-47: utterance counts, counted from the records when the
    config does not give them."""
    train_num, valid_num, test_num = config.prep_data_num_train, config.prep_data_num_valid, config.prep_data_num_test
    if config.path_train_ptrn and train_num is None:
        train_num = _count(os.path.join(config.path_base, config.path_train_ptrn))
    if config.path_valid_ptrn and valid_num is None:
        valid_num = _count(os.path.join(config.path_base, config.path_valid_ptrn))
    if config.path_test_ptrn and test_num is None:
        test_num = _count(os.path.join(config.path_base, config.path_test_ptrn))
    return train_num, valid_num, test_num


def create_ds_for_evaluation(config, logger):
    """data_helper.py:49-69: batch size 1, utt ids kept."""
    test_file_ptrn = os.path.join(config.path_base, config.path_test_ptrn)
    if logger is not None:
        logger.info('Batch size for test will be set to 1')
    test_ds = load_speech_data.create_ds_batch_for_test(file_pattern=test_file_ptrn, batch_size=1,
                                                        max_inp=config.prep_max_inp, max_tar=config.prep_max_tar)
    return test_ds.map(load_speech_data.map_data_for_transformer_utt_id_fn, config.feat_dim)


def replica_slice(batch_size, rank, world):
    """[lo, hi) of replica ``rank``'s share of a global batch: batch_size // world
    utterances each, the first batch_size % world replicas one more, in order --
    how tf.distribute rebatches a global batch over the replicas of
    MirroredStrategy.experimental_distribute_dataset (trainer_sr.py:147-153,168)."""
    if not 0 <= rank < world:
        raise ValueError(f'rank {rank} outside world {world}')
    q, r = divmod(batch_size, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def split_global_batch(batch, rank, world):
    """Replica ``rank``'s sub-batch of one global batch (a tuple of arrays whose
    first axis is the utterance).  Padding is left as the global batch had it:
    process_train_step crops each replica to its own longest utterance
    (trainer_sr.py:59-60), as the reference's replicas do."""
    lo, hi = replica_slice(len(batch[0]), rank, world)
    return tuple(c[lo:hi] for c in batch)


def distribute_dataset(dataset, rank, world):
    """strategy.experimental_distribute_dataset (trainer_sr.py:168) for one process
    per GPU: every rank iterates the same global batches (same files, same shuffle
    seed) and keeps its own slice.  The reference forces every bucket batch size
    above num_gpus (train_helper.py:289-296,301-309), so no replica is empty."""
    if world <= 1:
        return dataset
    return load_speech_data.Dataset(lambda: (split_global_batch(b, rank, world) for b in dataset))


def _shared_seed(seed, world):
    """All ranks must shuffle identically: an explicit seed, or rank 0's draw
    broadcast over the process group."""
    if seed is not None or world <= 1:
        return seed
    import numpy as np
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        raise ValueError('create_ds_for_training with world > 1 needs a seed or an initialised process group')
    t = torch.tensor([int(np.random.default_rng().integers(0, 2 ** 31 - 1))], dtype=torch.int64)
    if dist.get_backend() == 'nccl':
        t = t.cuda()
    dist.broadcast(t, src=0)
    return int(t.item())


def _dist_rank_world():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def create_ds_for_training(config, logger, num_gpus, manual_bucket_batch_sizes=None, seed=None, rank=None,
                           world=None):
    """data_helper.py:71-125: length-bucketed batches of ~train_batch_frame
    frames (buckets from get_bucket_info(frames, num_gpus, 241, 10000, 150)) or
    fixed-size batches.

    ``rank`` / ``world`` (defaults: the process group's rank and size, or 0 and 1
    without one) give the per-process view of MirroredStrategy's distributed
    dataset: each yielded batch is this replica's slice of a global batch
    (distribute_dataset).  ``num_gpus`` sizes the buckets only, as in the reference
    (get_bucket_info), so a single process asking for num_gpus > 1 gets whole
    global batches, never a silent 1/num_gpus slice."""
    g_rank, g_world = _dist_rank_world()
    world = g_world if world is None else world
    rank = g_rank if rank is None else rank
    seed = _shared_seed(seed, world)
    train_ds, valid_ds = _create_global(config, logger, num_gpus, manual_bucket_batch_sizes, seed)
    return distribute_dataset(train_ds, rank, world), distribute_dataset(valid_ds, rank, world)


def _create_global(config, logger, num_gpus, manual_bucket_batch_sizes, seed):
    train_file_ptrn = os.path.join(config.path_base, config.path_train_ptrn)
    valid_file_ptrn = os.path.join(config.path_base, config.path_valid_ptrn)
    if config.train_batch_dynamic:
        assert config.train_batch_frame is not None and config.train_batch_frame > 0
        bounds, sizes = th.get_bucket_info(config.train_batch_frame, num_gpus, 241, 10000, 150,
                                           step_for_bucket_size=False,
                                           manual_bucket_batch_sizes=manual_bucket_batch_sizes)
        if logger is not None:
            logger.info('bucket_boundaries: [%s]', ', '.join(map(str, bounds)))
            logger.info('bucket_batch_sizes: [%s]', ', '.join(map(str, sizes)))
        train_ds = load_speech_data.create_ds_bucket(train_file_ptrn, True, 1, bounds, sizes, config.prep_max_inp,
                                                     config.prep_max_tar, seed=seed)
        valid_ds = load_speech_data.create_ds_bucket(valid_file_ptrn, False, 1, bounds, sizes, config.prep_max_inp,
                                                     config.prep_max_tar)
    else:
        assert config.train_batch_size is not None and config.train_batch_size > 0
        train_ds = load_speech_data.create_ds_batch_for_train(train_file_ptrn, True, 1, config.train_batch_size,
                                                              config.prep_max_inp, config.prep_max_tar, seed=seed)
        valid_ds = load_speech_data.create_ds_batch_for_train(valid_file_ptrn, False, 1, config.train_batch_size,
                                                              config.prep_max_inp, config.prep_max_tar)
    fn = load_speech_data.map_data_for_transformer_fn
    return train_ds.map(fn, config.feat_dim), valid_ds.map(fn, config.feat_dim)
