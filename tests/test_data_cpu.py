"""TF-free input pipeline (libsrf_data.so + srf_amd/load_speech_data.py) against
independent oracles:
  * CRC-32C known answers (RFC 3720 B.4 / the iSCSI check value of "123456789");
  * tf.train.Example wire bytes from google.protobuf with descriptors built from
    tensorflow/core/example/{feature,example}.proto (field numbers restated here),
    serialised deterministically -- the reference's save path is
    tf.train.Example(...).SerializeToString() (save_speech_data.py:178-186);
  * TFRecord framing restated in Python (length, masked CRCs);
  * dataset semantics (filter, padded_batch, bucket_by_sequence_length) restated
    in plain Python from load_speech_data.py:24-181 and TF's documented semantics.
TensorFlow itself is not installed, so these are the pins (no TF-produced file
ships in the reference)."""
import struct

import numpy as np
import pytest

from srf_amd import load_speech_data as lsd
from srf_amd import data_helper, train_helper


def crc32c_py(data):
    c = 0xFFFFFFFF
    for b in data:
        c ^= b
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
    return c ^ 0xFFFFFFFF


def masked(c):
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def test_crc32c_known_answers():
    L = lsd.lib()
    cases = [(b'123456789', 0xE3069283), (b'', 0x0), (bytes(32), 0x8A9136AA), (b'\xff' * 32, 0x62A8AB43),
             (bytes(range(32)), 0x46DD794E), (bytes(range(31, -1, -1)), 0x113FDB5C)]
    for data, want in cases:
        assert L.srf_crc32c(data, len(data)) == want, data
    rng = np.random.default_rng(0)
    for n in (1, 7, 8, 9, 63, 1000):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert L.srf_crc32c(data, n) == crc32c_py(data)
        assert L.srf_crc32c_masked(data, n) == masked(crc32c_py(data))


def _example_classes():
    """tf.train.Example / Features / Feature / *List from the public .proto field
    numbers (feature.proto: BytesList=1, FloatList=2 packed, Int64List=3 packed,
    Feature oneof kind {bytes_list=1, float_list=2, int64_list=3}, Features map
    feature=1; example.proto: Example features=1)."""
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    fd = descriptor_pb2.FileDescriptorProto(name='srf_test_example.proto', package='tfx', syntax='proto3')
    F = descriptor_pb2.FieldDescriptorProto

    def msg(name, fields, nested=None):
        m = fd.message_type.add(name=name)
        for fname, num, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = tname
        return m
    rep, opt = F.LABEL_REPEATED, F.LABEL_OPTIONAL
    msg('BytesList', [('value', 1, F.TYPE_BYTES, rep, None)])
    msg('FloatList', [('value', 1, F.TYPE_FLOAT, rep, None)])
    msg('Int64List', [('value', 1, F.TYPE_INT64, rep, None)])
    feat = msg('Feature', [('bytes_list', 1, F.TYPE_MESSAGE, opt, '.tfx.BytesList'),
                           ('float_list', 2, F.TYPE_MESSAGE, opt, '.tfx.FloatList'),
                           ('int64_list', 3, F.TYPE_MESSAGE, opt, '.tfx.Int64List')])
    feat.oneof_decl.add(name='kind')
    for f in feat.field:
        f.oneof_index = 0
    feats = msg('Features', [('feature', 1, F.TYPE_MESSAGE, rep, '.tfx.Features.FeatureEntry')])
    entry = feats.nested_type.add(name='FeatureEntry')
    entry.field.add(name='key', number=1, type=F.TYPE_STRING, label=opt)
    entry.field.add(name='value', number=2, type=F.TYPE_MESSAGE, label=opt, type_name='.tfx.Feature')
    entry.options.map_entry = True
    msg('Example', [('features', 1, F.TYPE_MESSAGE, opt, '.tfx.Features')])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = message_factory.GetMessageClass
    return {n: get(pool.FindMessageTypeByName('tfx.' + n)) for n in ('Example', 'Feature', 'FloatList', 'Int64List',
                                                                      'BytesList')}


def _pb_example(C, feats, labels, utt):
    ex = C['Example']()
    fm = ex.features.feature
    fm['input_speech'].float_list.value.extend(np.asarray(feats, np.float32).reshape(-1).tolist())
    fm['target_label'].int64_list.value.extend([int(v) for v in labels])
    fm['input_length'].int64_list.value.append(int(np.asarray(feats).shape[0]))
    fm['target_length'].int64_list.value.append(len(labels))
    if utt is not None:
        fm['utt_id'].bytes_list.value.append(utt)
    return ex


def _frame(payload):
    hdr = struct.pack('<Q', len(payload))
    return hdr + struct.pack('<I', masked(crc32c_py(hdr))) + payload + struct.pack('<I', masked(crc32c_py(payload)))


def test_writer_bytes_match_protobuf_serialisation(tmp_path):
    C = _example_classes()
    rng = np.random.default_rng(1)
    path = str(tmp_path / 'w.tfrecord')
    expected = b''
    with lsd.TFRecordWriter(path) as w:
        for k in range(4):
            T = int(rng.integers(1, 9))
            feats = rng.standard_normal((T, 5)).astype(np.float32)
            labels = rng.integers(1, 62, int(rng.integers(0, 6)))
            utt = f'spk{k}-utt{k}'.encode() if k % 2 == 0 else None
            w.write_example(feats, labels, utt_id=utt)
            expected += _frame(_pb_example(C, feats, labels, utt).SerializeToString(deterministic=True))
    assert open(path, 'rb').read() == expected


def test_reader_parses_protobuf_records(tmp_path):
    """protobuf-serialised Examples (deterministic and default map order, extra
    unknown feature) framed in Python, read back by the C++ reader."""
    C = _example_classes()
    rng = np.random.default_rng(2)
    path = str(tmp_path / 'r.tfrecord')
    ref = []
    with open(path, 'wb') as f:
        for k in range(5):
            T = int(rng.integers(1, 12))
            feats = rng.standard_normal((T, 3)).astype(np.float32)
            labels = rng.integers(1, 30, int(rng.integers(1, 8)))
            ex = _pb_example(C, feats, labels, f'u{k}'.encode())
            ex.features.feature['ignored_extra'].float_list.value.append(1.5)
            f.write(_frame(ex.SerializeToString(deterministic=(k % 2 == 0))))
            ref.append((feats, labels, f'u{k}'.encode()))
    got = list(lsd.read_tfrecord(path, is_utt_id=True))
    assert len(got) == len(ref)
    for (feats, labels, utt), (gf, gl, a, b, gu) in zip(ref, got):
        np.testing.assert_array_equal(gf, feats.reshape(-1))
        np.testing.assert_array_equal(gl, labels)
        assert a == feats.shape[0] and b == len(labels) and gu == utt


def test_reader_accepts_unpacked_lists_and_detects_corruption(tmp_path):
    # unpacked float (wire type 5) and int64 (wire type 0) encodings, hand-built
    def ld(field, body):
        return bytes([(field << 3) | 2]) + _varint(len(body)) + body

    floats = b''.join(bytes([(1 << 3) | 5]) + struct.pack('<f', v) for v in (1.0, -2.5))
    ints = b''.join(bytes([(1 << 3) | 0]) + _varint(v) for v in (3, 300))
    one = bytes([(1 << 3) | 0]) + _varint(1)
    two = bytes([(1 << 3) | 0]) + _varint(2)

    def entry(key, feature):
        return ld(1, ld(1, key.encode()) + ld(2, feature))
    feats = (entry('input_speech', ld(2, floats)) + entry('target_label', ld(3, ints))
             + entry('input_length', ld(3, one)) + entry('target_length', ld(3, two)))
    payload = ld(1, feats)
    x, y, a, b = lsd.parse_example(payload, is_utt_id=False)
    np.testing.assert_array_equal(x, [1.0, -2.5])
    np.testing.assert_array_equal(y, [3, 300])
    assert (a, b) == (1, 2)
    path = str(tmp_path / 'bad.tfrecord')
    rec = bytearray(_frame(payload))
    rec[20] ^= 0x40
    open(path, 'wb').write(bytes(rec))
    with pytest.raises(lsd.TFRecordError, match='CRC'):
        list(lsd.read_tfrecord(path))


def _varint(v):
    out = b''
    while v >= 0x80:
        out += bytes([(v & 0x7F) | 0x80])
        v >>= 7
    return out + bytes([v])


def _write_corpus(tmp_path, n_utt, feat_dim, shards=3, seed=3):
    rng = np.random.default_rng(seed)
    paths = lsd.tfrecord_shard_paths(str(tmp_path), 'tfr', 'timit', 'train', 'fbank', feat_dim, shards)
    (tmp_path / 'tfr').mkdir()
    utts = []
    writers = [lsd.TFRecordWriter(p) for p in paths]
    for k in range(n_utt):
        T = int(rng.integers(5, 60))
        feats = rng.standard_normal((T, feat_dim)).astype(np.float32)
        labels = rng.integers(1, 61, int(rng.integers(1, T // 2 + 2)))
        writers[k % shards].write_example(feats, labels, utt_id=f'utt{k:03d}')   # round robin (:133-135)
        utts.append((feats, labels))
    for w in writers:
        w.close()
    return paths, utts


def test_shard_names():
    p = lsd.tfrecord_shard_paths('/d', 'tfrecord', 'timit', 'train', 'fbank', 123, 2)
    assert p == ['/d/tfrecord/timit-train-fbank-123-00001-of-00002', '/d/tfrecord/timit-train-fbank-123-00002-of-00002']


def test_create_ds_order_filter_and_padding(tmp_path):
    paths, utts = _write_corpus(tmp_path, 14, 4)
    pattern = str(tmp_path / 'tfr' / '*')
    ds = lsd.create_ds(pattern, False, max_inp=40, max_tar=-1)
    got = list(ds)
    # round-robin over the sorted shards, one record each: utt order 0..13
    want = [u for u in utts if u[0].shape[0] <= 40]
    assert len(got) == len(want)
    for (f, l), (gf, gl, a, b) in zip(want, got):
        np.testing.assert_array_equal(gf, f.reshape(-1))
        assert a == f.shape[0] and b == len(l)
    batches = list(lsd.create_ds_batch_for_train(pattern, False, 1, 3, -1, -1).map(
        lsd.map_data_for_transformer_fn, 4))
    assert len(batches) == 14 // 3   # drop_remainder=True
    x, y, a, b = batches[0]
    assert x.shape == (3, int(a.max()), 4) and x.dtype == np.float32 and y.dtype == np.int32
    for i in range(3):
        np.testing.assert_array_equal(x[i, :a[i]], utts[i][0])
        assert np.all(x[i, a[i]:] == 0) and np.all(y[i, b[i]:] == 0)


def test_bucket_by_sequence_length_semantics(tmp_path):
    paths, utts = _write_corpus(tmp_path, 40, 2, shards=1, seed=4)
    pattern = str(tmp_path / 'tfr' / '*')
    bounds, sizes = [20, 35], [4, 3, 2]
    got = list(lsd.create_ds_bucket(pattern, False, 1, bounds, sizes, -1, -1))
    # restatement: bucket k holds [b_{k-1}, b_k); a bucket emits when full; partials dropped
    pending, want = [[], [], []], []
    for k, (f, l) in enumerate(utts):
        T = f.shape[0]
        bk = 0 if T < 20 else (1 if T < 35 else 2)
        pending[bk].append(k)
        if len(pending[bk]) == sizes[bk]:
            want.append(pending[bk])
            pending[bk] = []
    assert len(got) == len(want)
    for batch, idx in zip(got, want):
        x, y, a, b = batch
        assert list(a) == [utts[i][0].shape[0] for i in idx]
        assert x.shape == (len(idx), max(a) * 2)


def test_training_datasets_from_config(tmp_path):
    from srf_amd.common_helper import build_parser
    _write_corpus(tmp_path, 30, 3, shards=2, seed=5)
    cfg = build_parser().parse_args([])
    cfg.path_base = str(tmp_path)
    cfg.path_train_ptrn = cfg.path_valid_ptrn = 'tfr/*'
    cfg.feat_dim = 3
    cfg.train_batch_dynamic = True
    cfg.train_batch_frame = 700
    train_ds, valid_ds = data_helper.create_ds_for_training(cfg, None, 1, seed=0)
    bounds, sizes = train_helper.get_bucket_info(700, 1, 241, 10000, 150)
    n_frames = [int(a.sum()) for _, _, a, _ in valid_ds]
    for (x, y, a, b) in valid_ds:
        k = int(np.searchsorted(bounds, int(a.max()), side='right'))
        assert x.shape[0] == sizes[k] and x.shape[2] == 3
    n_train = 0
    for (x, y, a, b) in train_ds:
        k = int(np.searchsorted(bounds, int(a.max()), side='right'))
        assert x.shape[0] == sizes[k]
        n_train += 1
    assert n_train > 0 and len(n_frames) > 0
    assert data_helper.get_data_len(cfg)[:2] == (30, 30)


def test_data_library_exports_every_header_symbol():
    import ctypes
    import os
    import re
    hdr = open(os.path.join(os.path.dirname(__file__), '..', 'include', 'srf_data.h')).read()
    hdr = re.sub(r'/\*.*?\*/', '', hdr, flags=re.S)
    declared = set(re.findall(r'^(?:int|void\*|uint32_t|const char\*|const uint8_t\*)\s+(srf_\w+)\(', hdr, re.M))
    assert len(declared) == 14, declared
    lib = ctypes.CDLL(lsd.DATA_LIB_PATH)
    for name in declared:
        assert hasattr(lib, name), name
    assert declared == set(lsd.exported_symbols())


def test_replica_slices_cover_the_global_batch_in_order():
    """tf.distribute rebatching (trainer_sr.py:147-153,168): B // world each, the
    first B % world replicas one more, contiguous and in order."""
    for B in range(1, 40):
        for world in (1, 2, 3, 4, 8):
            sl = [data_helper.replica_slice(B, r, world) for r in range(world)]
            assert sl[0][0] == 0 and sl[-1][1] == B
            assert all(a[1] == b[0] for a, b in zip(sl, sl[1:]))
            sizes = [hi - lo for lo, hi in sl]
            assert max(sizes) - min(sizes) <= 1 and sizes == sorted(sizes, reverse=True)
    assert [hi - lo for lo, hi in (data_helper.replica_slice(17, r, 8) for r in range(8))] == [3] + [2] * 7


def test_training_datasets_split_per_replica(tmp_path):
    """create_ds_for_training(..., rank, world): every rank sees the same global
    batch sequence (shared shuffle seed) and keeps its own slice; the slices of all
    ranks rebuild each global batch, padded like it (each replica crops later)."""
    from srf_amd.common_helper import build_parser
    _write_corpus(tmp_path, 60, 3, shards=2, seed=6)
    cfg = build_parser().parse_args([])
    cfg.path_base = str(tmp_path)
    cfg.path_train_ptrn = cfg.path_valid_ptrn = 'tfr/*'
    cfg.feat_dim = 3
    cfg.train_batch_dynamic = True
    cfg.train_batch_frame = 1400
    world = 2
    glob_train, _ = data_helper.create_ds_for_training(cfg, None, world, seed=3, rank=0, world=1)
    parts = [data_helper.create_ds_for_training(cfg, None, world, seed=3, rank=r, world=world)[0]
             for r in range(world)]
    glob = list(glob_train)
    per_rank = [list(p) for p in parts]
    assert len(glob) > 0 and all(len(p) == len(glob) for p in per_rank)
    for k, g in enumerate(glob):
        assert g[0].shape[0] > world     # bucket sizes are forced above num_gpus
        for comp in range(4):
            np.testing.assert_array_equal(np.concatenate([p[k][comp] for p in per_rank]), g[comp])
    with pytest.raises(ValueError):
        data_helper.create_ds_for_training(cfg, None, world, seed=None, rank=0, world=world)
    # no process group: one replica (whole global batches), whatever num_gpus says
    single = list(data_helper.create_ds_for_training(cfg, None, world, seed=3)[0])
    assert len(single) == len(glob)
    for a, b in zip(single, glob):
        np.testing.assert_array_equal(a[0], b[0])
