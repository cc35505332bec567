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


def create_ds_for_training(config, logger, num_gpus, manual_bucket_batch_sizes=None, seed=None):
    """data_helper.py:71-125: length-bucketed batches of ~train_batch_frame
    frames (buckets from get_bucket_info(frames, num_gpus, 241, 10000, 150)) or
    fixed-size batches."""
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
