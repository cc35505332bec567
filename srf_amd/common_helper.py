"""Flag surface of tfsr (``tfsr/helper/common_helper.py``), re-implemented.

Same flag names, types, defaults, ``@file.conf`` loading and merge rule as the
reference's ``ParseOption`` (common_helper.py:134-194): keys given on the
command line (as ``--key=value``) win, every other key comes from the
``--config`` file.  ``sanity_check`` mirrors :222-268 and failures exit with the
reference's ``ExitCode`` values.  Parity is pinned by
``tests/golden/flags_*.json``, produced by the reference parser itself
(``oracle/gen_golden.py``).
"""
import argparse
import logging
import os
import sys
from enum import Enum


class Constants:
    """Subset of common_helper.py:41-81 used on the SRF path."""
    PAD_CHAR = 'p'
    PAD_WORD = '<PADDING_SYMBOL>'
    SPACE = '<SPACE>'
    UNK = '<unk>'
    EOS = '$'
    BOS = '@'
    EPS = 1e-14
    INF = 1e9
    SM_NEIGHBOR = 'neighbor'
    SM_LABEL = 'label'
    INIT_GLOROT = 'glorot_uniform'
    INIT_FANAVG = 'fan_avg'
    INIT_UNIFORM = 'uniform'


class ExitCode(Enum):
    """common_helper.py:83-95."""
    NO_DATA = 0
    NOT_SUPPORTED = 1
    INVALID_OPTION = 11
    INVALID_CONVERSION = 12
    INVALID_NAME = 13
    INVALID_NAME_OF_CONFIGURATION_FILE = 14
    INVALID_FILE_PATH = 15
    INVALID_DICTIONARY = 16
    INVALID_CONDITION = 17


class Logger:
    """TF-style log lines (common_helper.py:97-132)."""
    DEBUG, INFO, WARN, ERROR, CRITICAL = (logging.DEBUG, logging.INFO, logging.WARN, logging.ERROR,
                                          logging.CRITICAL)
    NOTSET = logging.NOTSET

    def __init__(self, name='__default__', level=logging.NOTSET):
        self.logger = logging.getLogger(name)
        self.logger.setLevel(level)
        if not self.logger.handlers:
            h = logging.StreamHandler()
            h.setLevel(level)
            fmt = logging.Formatter('%(asctime)s: %(levelname).1s %(filename)s:%(lineno)d] %(message)s')
            fmt.default_msec_format = '%s.%06d'
            h.setFormatter(fmt)
            self.logger.addHandler(h)
        self.logger.propagate = False


def str2bool(s):
    return s.lower() in ('yes', 'true', 't', '1')


def str2list_int(s):
    if s is None:
        return None
    return [int(x) for x in s.replace('"', '').replace('[', '').replace(']', '').split(',')]


# (group, flag, type, default) -- the reference's parser table (common_helper.py:288-459)
_B, _L = str2bool, str2list_int
_FLAGS = [
    ('training', 'train-inp-dropout', float, 0.1), ('training', 'train-inn-dropout', float, 0.1),
    ('training', 'train-att-dropout', float, 0.1), ('training', 'train-res-dropout', float, 0.1),
    ('training', 'train-ckpt-saving-per', int, 1), ('training', 'train-es-min-delta', float, 0.001),
    ('training', 'train-es-tolerance', int, 1), ('training', 'train-lr-param-k', float, None),
    ('training', 'train-max-epoch', int, None), ('training', 'train-adam-beta1', float, 0.9),
    ('training', 'train-adam-beta2', float, 0.98), ('training', 'train-adam-epsilon', float, 1e-09),
    ('training', 'train-warmup-n', int, 25000), ('training', 'train-ppl-step', int, 1),
    ('training', 'train-max-step', int, 0), ('training', 'train-opti-type', str, None),
    ('training', 'train-smoothing-confidence', float, 0.0),
    ('training', 'train-smoothing-type', str, Constants.SM_NEIGHBOR),
    ('training', 'train-schedule-prob', float, None), ('training', 'train-batch-size', int, 26),
    ('training', 'train-batch-frame', int, 20000), ('training', 'train-lr-max', float, 1e3),
    ('training', 'train-batch-dynamic', _B, 'False'), ('training', 'train-is-mwer', _B, 'false'),
    ('training', 'train-batch-buckets', _L, None),
    ('prep', 'prep-data-shard', int, 100), ('prep', 'prep-data-name', str, 'wsj'),
    ('prep', 'prep-data-unit', str, 'char'), ('prep', 'prep-data-bos', _B, 'True'),
    ('prep', 'prep-data-pad-space', _B, 'True'), ('prep', 'prep-max-tar', int, -1),
    ('prep', 'prep-max-inp', int, -1), ('prep', 'prep-data-num-train', int, None),
    ('prep', 'prep-data-num-valid', int, None), ('prep', 'prep-data-num-test', int, None),
    ('path', 'path-base', str, None), ('path', 'path-ckpt', str, None), ('path', 'path-ckpt-epoch', int, 0),
    ('path', 'path-cmvn-ptrn', str, None), ('path', 'path-vocab', str, None), ('path', 'path-hyp', str, None),
    ('path', 'path-train-ptrn', str, None), ('path', 'path-test-ptrn', str, None),
    ('path', 'path-valid-ptrn', str, None), ('path', 'path-train-json', str, None),
    ('path', 'path-valid-json', str, None), ('path', 'path-test-json', str, None),
    ('path', 'path-wrt-tfrecord', str, None),
    ('feature', 'feat-type', str, None), ('feature', 'feat-dim', int, None), ('feature', 'feat-dim1', int, None),
    ('feature', 'feat-dim2', int, None),
    ('model', 'model-encoder-num', int, None), ('model', 'model-decoder-num', int, None),
    ('model', 'model-res-enc', int, 1), ('model', 'model-res-dec', int, 1), ('model', 'model-dimension', int, 1),
    ('model', 'model-inner-dim', int, 2048), ('model', 'model-inner-num', int, 3),
    ('model', 'model-att-head-num', int, 4), ('model', 'model-conv-filter-num', int, 64),
    ('model', 'model-conv-layer-num', int, 2), ('model', 'model-conv-stride', int, 2),
    ('model', 'model-ckpt-max-to-keep', int, -1), ('model', 'model-shared-embed', _B, 'False'),
    ('model', 'model-conv-mask-type', int, None), ('model', 'model-ap-scale', float, None),
    ('model', 'model-ap-width-zero', int, None), ('model', 'model-ap-width-stripe', int, None),
    ('model', 'model-average-num', int, None), ('model', 'model-ap-encoder', _B, 'False'),
    ('model', 'model-ap-decoder', _B, 'False'), ('model', 'model-ap-encdec', _B, 'False'),
    ('model', 'model-type', str, 'srf'), ('model', 'model-initializer', str, None),
    ('model', 'model-emb-sqrt', _B, 'True'), ('model', 'model-caps-context', _B, 'True'),
    ('model', 'model-lstm-is-cnnfe', _B, 'False'), ('model', 'model-lstm-merge', str, 'ave'),
    ('model', 'model-caps-type', str, 'lowmemory'), ('model', 'model-caps-iter', int, 2),
    ('model', 'model-caps-primary-num', int, 3), ('model', 'model-caps-primary-dim', int, 2),
    ('model', 'model-caps-convolution-num', int, 4), ('model', 'model-caps-convolution-dim', int, 4),
    ('model', 'model-caps-class-dim', int, 64), ('model', 'model-caps-window-lpad', int, None),
    ('model', 'model-caps-window-rpad', int, None), ('model', 'model-caps-layer-num', int, 2),
    ('model', 'model-caps-layer-time', int, None), ('model', 'model-caps-res-connection', _B, 'False'),
    ('model', 'model-conv-is-mp', _B, 'False'), ('model', 'model-conv-inp-nfilt', int, 64),
    ('model', 'model-conv-inn-nfilt', int, 128), ('model', 'model-conv-proj-num', int, 3),
    ('model', 'model-conv-proj-dim', int, 512),
    ('decoding', 'decoding-beam-width', int, None), ('decoding', 'decoding-lp-alpha', float, None),
    ('decoding', 'decoding-from-npy', _B, 'False'),
]


def build_parser():
    parser = argparse.ArgumentParser(description='MI355X Sequential Routing Framework', fromfile_prefix_chars='@')
    parser.add_argument('--config', help='options can be loaded from this config file')
    groups = {}
    for group, flag, typ, default in _FLAGS:
        grp = groups.get(group)
        if grp is None:
            grp = groups[group] = parser.add_argument_group(title=group)
        kw = {'default': default}
        if typ is not str:
            kw['type'] = typ
        grp.add_argument('--' + flag, **kw)
    return parser


class ParseOption:
    """``ParseOption(argv, logger).args`` (common_helper.py:134-194)."""

    def __init__(self, argv, logger, is_print_opts=True):
        self.logger = logger
        parser = build_parser()
        if len(argv) <= 1:
            logger.critical('No options..')
            sys.exit(ExitCode.INVALID_OPTION)
        # The reference derives the set of command-line keys from '--key=value'
        # tokens (common_helper.py:143-145); a bare '--key value' pair loses its
        # last character there, and we keep that behaviour.
        cmd_keys = {a.replace('-', '_')[2:a.find('=')] for a in argv[1:]}
        cmd = parser.parse_args(argv[1:])
        if cmd.config is not None and not cmd.config.endswith('.conf'):
            logger.critical('The the extension of configuration file must be conf, but %s' % cmd.config)
            sys.exit(ExitCode.INVALID_NAME_OF_CONFIGURATION_FILE)
        merged = vars(cmd)
        if cmd.config:
            path = cmd.config
            if cmd.path_base and not os.path.exists(path):
                path = cmd.path_base + '/' + path
            from_file = vars(parser.parse_args(['@' + path]))
            if 'config' not in cmd_keys:
                logger.critical('"config" is a required option for the command line.')
                sys.exit(ExitCode.INVALID_OPTION)
            for k in merged:
                if k not in cmd_keys:
                    merged[k] = from_file[k]
        args = argparse.Namespace(**merged)
        if not self.sanity_check(args):
            sys.exit(ExitCode.INVALID_OPTION)
        if is_print_opts:
            self.print_args(args)
        self._args = args

    @property
    def args(self):
        return self._args

    str2bool = staticmethod(str2bool)
    str2list_int = staticmethod(str2list_int)

    def sanity_check(self, args):
        """common_helper.py:222-268."""
        log = self.logger
        if args.model_caps_type not in ('lowmemory', 'einsum', 'naive'):
            log.critical('model-caps-type must be lowmemory, einsum or naivebut %s', args.model_caps_type)
            return False
        if not args.path_base:
            log.critical('the following arguments are required: paths-data-path')
            return False
        if not os.path.isdir(args.path_base) or os.path.isfile(args.path_base):
            log.critical('A data path must exist, please check the data path option : %s' % args.path_base)
            return False
        if args.train_schedule_prob is not None and not 0 <= args.train_schedule_prob < 2:
            log.critical('Prob. for scheduled sampling must be within [0, 2)')
            return False
        if args.train_smoothing_type not in (Constants.SM_LABEL, Constants.SM_NEIGHBOR):
            log.critical('Please check smoothing type %s' % args.train_smoothing_type)
            return False
        if not args.train_is_mwer and (args.prep_max_inp > 0 or args.prep_max_tar > 0):
            log.warning('Please do not set max length unless you use mwer, but prep-max-inp %d, prep-max-tar %d'
                        % (args.prep_max_inp, args.prep_max_tar))
        return True

    def print_args(self, args):
        log = self.logger
        log.info('********************************************')
        log.info('        Sequential Routing Framework        ')
        log.info('********************************************')
        prev = ''
        for k in sorted(vars(args)):
            head = k.split('_')[0]
            if head != prev:
                log.info('. %s' % head.upper())
                prev = head
            log.info('- %s=%s' % (k, getattr(args, k)))
        log.info('*********************************************')


def load_vocab(vocab_path, logger=None):
    """``Util.load_vocab`` (misc_helper.py:77-108): returns (vocab, str_to_int,
    dec_in_dim, dec_out_dim).  The trainer uses class_n = dec_in_dim + 1 and
    blank = dec_in_dim (trainer_sr.py:130-134)."""
    vocab = []
    with open(vocab_path) as fh:
        for line in fh:
            tok = line.strip()
            vocab.append(' ' if tok == Constants.SPACE else tok)
    if vocab[-1] != Constants.BOS:
        msg = 'Last index must be BOS: %s, but %s' % (Constants.BOS, vocab[-1])
        (logger.critical(msg) if logger else print(msg))
    s2i = {t: i for i, t in enumerate(vocab)}
    dec_in = len(vocab)
    dec_out = dec_in - 1 if Constants.BOS in s2i else dec_in
    msg = 'Decoder Input Dim: %d, Output Dim %d' % (dec_in, dec_out)
    (logger.info(msg) if logger else print(msg))
    return vocab, s2i, dec_in, dec_out
