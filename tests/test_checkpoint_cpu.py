"""Checkpoint surface of the SRF path (srf_amd/checkpoint.py) on CPU tensors:
TF object-path naming and shapes (naive:68-118, sequence_router.py:44-63),
CheckpointManager semantics (ckpt-N, max_to_keep, the `checkpoint` state file,
misc_helper.py:139-163) and averaging (average_ckpt_sr.py:135-179)."""
import argparse
import os

import numpy as np
import pytest
import torch

from srf_amd import checkpoint as ck
from srf_amd.sequence_router import SequenceRouter
from srf_amd.train_helper import CustomSchedule, SrfAdam
from tests.helpers import config_from_shape

KW = dict(feat_dim=40, enc_num=2, iters=2, lpad=1, rpad=1, ph=4, pd=8, ch=4, cd=8, vd=8, context=False)


def _model(seed):
    return SequenceRouter(config_from_shape(KW), None, 12, device=torch.device('cpu'), seed=seed)


def test_tf_names_and_shapes():
    m = _model(0)
    st = ck.model_state(m)
    in_n = 4 * 3
    assert st['model/wgt/0/.ATTRIBUTES/VARIABLE_VALUE'].shape == (1, 1, in_n, 4, 8, 8)
    assert st['model/bias/1/.ATTRIBUTES/VARIABLE_VALUE'].shape == (1, 1, in_n, 12, 8, 1)
    assert st['model/conv/conv_layers/1/0/kernel/.ATTRIBUTES/VARIABLE_VALUE'].shape == (3, 3, 1, 64)
    assert st['model/conv/bn_layers/1/moving_variance/.ATTRIBUTES/VARIABLE_VALUE'].shape == (64,)
    assert st['model/ln_m/1/gamma/.ATTRIBUTES/VARIABLE_VALUE'].shape == (12 * 8,)
    assert st['model/proj_pe/kernel/.ATTRIBUTES/VARIABLE_VALUE'].shape == (10 * 64, 4)
    # every parameter and BN statistic is named exactly once
    assert len(st) == len(m.params) + 2 * m.cnn_n
    np.testing.assert_array_equal(st['model/wgt/0/.ATTRIBUTES/VARIABLE_VALUE'].reshape(in_n, 4, 8, 8),
                                  m.params['W0'].detach().numpy())


def test_tf_shapes_per_variant():
    """einsum:91-97 and lowmemory:94-98 store W / bias without the naive (1, 1)
    prefix or with a single leading 1; values keep the same order."""
    in_n = 4 * 3
    for caps_type, ws, bs in (('einsum', (in_n, 4, 8, 8), (1, 1, in_n, 12, 8)),
                              ('lowmemory', (1, in_n, 4, 8, 8), (1, in_n, 12, 8, 1))):
        m = SequenceRouter(config_from_shape(dict(KW, caps_type=caps_type)), None, 12, device=torch.device('cpu'),
                           seed=0)
        st = ck.model_state(m)
        assert st['model/wgt/0/.ATTRIBUTES/VARIABLE_VALUE'].shape == ws
        assert st['model/bias/1/.ATTRIBUTES/VARIABLE_VALUE'].shape == bs
        m2 = SequenceRouter(config_from_shape(dict(KW, caps_type=caps_type)), None, 12, device=torch.device('cpu'),
                            seed=5)
        ck.load_model_state(m2, st)
        assert torch.equal(m2.params['b1'], m.params['b1'])


@pytest.mark.parametrize('fmt', ['tf', 'safetensors'])
def test_manager_save_restore_rotation(tmp_path, fmt):
    m, opt = _model(1), SrfAdam(CustomSchedule(0.5, 1, 1200))
    opt._m = torch.randn(m.n_flat)
    opt._v = torch.rand(m.n_flat)
    opt.iterations = 17
    mgr = ck.CheckpointManager(m, opt, str(tmp_path), max_to_keep=2, fmt=fmt)
    for _ in range(3):
        with torch.no_grad():
            m.flat_params.add_(1.0)
        path = mgr.save()
    assert path.endswith('ckpt-3') and mgr.latest_checkpoint == path
    if fmt == 'tf':   # tf.train.CheckpointManager's file layout (the default)
        assert sorted(os.listdir(tmp_path)) == ['checkpoint', 'ckpt-2.data-00000-of-00001', 'ckpt-2.index',
                                                'ckpt-3.data-00000-of-00001', 'ckpt-3.index']
        from srf_amd import tf_bundle
        names = {n for n, _, _ in tf_bundle.list_variables(str(tmp_path / 'ckpt-3'))}
        assert 'model/wgt/0/' + ck.VALUE in names and ck.SAVE_COUNTER in names
    else:
        assert sorted(os.listdir(tmp_path)) == ['checkpoint', 'ckpt-2.srf.safetensors', 'ckpt-3.srf.safetensors']
    state_file = open(tmp_path / 'checkpoint').read()
    assert 'model_checkpoint_path: "ckpt-3"' in state_file and 'all_model_checkpoint_paths: "ckpt-2"' in state_file
    m2, opt2 = _model(2), SrfAdam(CustomSchedule(0.5, 1, 1200))
    cfg = argparse.Namespace(model_ckpt_max_to_keep=-1, path_ckpt=str(tmp_path), path_ckpt_epoch=0)
    mgr2, epoch = ck.load_checkpoint(cfg, None, m2, opt2)
    assert epoch == 3 and opt2.iterations == 17
    for k in m.params:
        torch.testing.assert_close(m2.params[k], m.params[k], rtol=0, atol=0)
    for a, b in ((opt2._m, opt._m), (opt2._v, opt._v)):
        for name in m.params:
            off, n = m.offsets[name], m.params[name].numel()
            torch.testing.assert_close(a[off:off + n], b[off:off + n], rtol=0, atol=0)
    cfg.path_ckpt_epoch = 2
    m3 = _model(3)
    assert ck.load_checkpoint(cfg, None, m3, None)[1] == 2
    torch.testing.assert_close(m3.params['W1'], m.params['W1'] - 1.0, rtol=0, atol=1e-6)


def test_resume_numbers_from_restored_save_counter(tmp_path):
    """tf.train.Checkpoint restores save_counter with the model: resuming from
    ckpt-3 while ckpt-5 exists writes ckpt-4 next (and the epoch offset of the
    following resume is 4, not 6)."""
    m = _model(1)
    mgr = ck.CheckpointManager(m, None, str(tmp_path), max_to_keep=None)
    for _ in range(5):
        mgr.save()
    assert mgr.save_counter == 5
    cfg = argparse.Namespace(model_ckpt_max_to_keep=-1, path_ckpt=str(tmp_path), path_ckpt_epoch=3)
    mgr2, epoch = ck.load_checkpoint(cfg, None, _model(2), None)
    assert epoch == 3 and mgr2.save_counter == 3
    assert mgr2.save().endswith('ckpt-4')
    assert int(ck.read_checkpoint(os.path.join(str(tmp_path), 'ckpt-4'))[ck.SAVE_COUNTER]) == 4
    # a fresh checkpoint object (no restore) counts from 0, as TF's does
    assert ck.CheckpointManager(m, None, str(tmp_path / 'other'), max_to_keep=None).save().endswith('ckpt-1')


def test_average_checkpoints(tmp_path):
    models = [_model(10 + k) for k in range(3)]
    mgr = ck.CheckpointManager(models[0], None, str(tmp_path), max_to_keep=None)
    for mk in models:
        mgr.model = mk
        mgr.save()
    cfg = argparse.Namespace(path_ckpt=str(tmp_path), model_average_num=2, train_max_epoch=0)
    path, avg = ck.average_checkpoints(cfg, None, lambda: _model(99))
    assert path == os.path.join(str(tmp_path), 'avg', 'ckpt-1')
    for k in avg.params:
        want = (models[1].params[k].detach() + models[2].params[k].detach()) / 2
        torch.testing.assert_close(avg.params[k].detach(), want, rtol=1e-6, atol=1e-7)
    back = _model(5)
    ck.restore(path, back)
    torch.testing.assert_close(back.params['b0'], avg.params['b0'], rtol=0, atol=0)
    # average_ckpt_sr.py:91-96: only ckpt-N with N <= train_max_epoch take part
    cfg.train_max_epoch = 2
    _, avg2 = ck.average_checkpoints(cfg, None, lambda: _model(99))
    for k in avg2.params:
        want = (models[0].params[k].detach() + models[1].params[k].detach()) / 2
        torch.testing.assert_close(avg2.params[k].detach(), want, rtol=1e-6, atol=1e-7)


def _masked_crc(b):
    from tests.test_data_cpu import crc32c_py, masked
    return masked(crc32c_py(b))


def test_tf_bundle_reads_hand_built_table(tmp_path):
    """A LevelDB-format table assembled byte by byte from the format spec
    (entries: varint shared/non_shared/value_len + key delta + value; restart
    array; block trailer type + masked CRC; index block of BlockHandles; 48-byte
    footer with magic) and a BundleEntryProto written field by field."""
    import struct
    from srf_amd import tf_bundle as tb
    val = np.arange(6, dtype=np.float32).reshape(2, 3)
    raw = val.tobytes()
    dims = bytes([0x12, 2, 0x08, 2]) + bytes([0x12, 2, 0x08, 3])          # dim{size:2} dim{size:3}
    entry = (bytes([0x08, 1]) + bytes([0x12, len(dims)]) + dims            # dtype=DT_FLOAT, shape
             + bytes([0x28, len(raw)]) + bytes([0x35]) + struct.pack('<I', _masked_crc(raw)))
    header = bytes([0x08, 1])                                              # num_shards=1
    # data block: key "" -> header, key "w" -> entry (shared 0, restart at 0 only)
    body = bytes([0, 0, len(header)]) + header + bytes([0, 1, len(entry)]) + b'w' + entry
    body += struct.pack('<I', 0) + struct.pack('<I', 1)
    f = bytearray(body)
    f += b'\x00' + struct.pack('<I', _masked_crc(body + b'\x00'))
    meta_off = len(f)
    meta = struct.pack('<I', 0) + struct.pack('<I', 1)
    f += meta + b'\x00' + struct.pack('<I', _masked_crc(meta + b'\x00'))
    idx_off = len(f)
    handle = bytes([0, len(body)])
    idx = bytes([0, 1, len(handle)]) + b'w' + handle + struct.pack('<I', 0) + struct.pack('<I', 1)
    f += idx + b'\x00' + struct.pack('<I', _masked_crc(idx + b'\x00'))
    footer = bytes([meta_off, len(meta), idx_off, len(idx)])
    f += footer + b'\x00' * (40 - len(footer)) + struct.pack('<Q', 0xdb4775248b80fb57)
    prefix = str(tmp_path / 'hand')
    open(prefix + '.index', 'wb').write(bytes(f))
    open(prefix + '.data-00000-of-00001', 'wb').write(raw)
    assert tb.list_variables(prefix) == [('w', [2, 3], 1)]
    np.testing.assert_array_equal(tb.load_checkpoint(prefix)['w'], val)


def test_tf_bundle_export_import_round_trip(tmp_path):
    from srf_amd import tf_bundle as tb
    m, opt = _model(7), SrfAdam(CustomSchedule(0.5, 1, 1200))
    opt._m = torch.randn(m.n_flat)
    opt._v = torch.rand(m.n_flat)
    opt.iterations = 5
    prefix = str(tmp_path / 'tf' / 'ckpt-4')
    tb.export_to_tf(prefix, m, opt)
    names = [n for n, _, _ in tb.list_variables(prefix)]
    assert names == sorted(names) and 'model/wgt/1/.ATTRIBUTES/VARIABLE_VALUE' in names
    m2, opt2 = _model(8), SrfAdam(CustomSchedule(0.5, 1, 1200))
    unused = tb.restore_from_tf(prefix, m2, opt2)
    assert unused and all(k.startswith('optimizer/') or '.OPTIMIZER_SLOT/' in k for k in unused)
    for k in m.params:
        torch.testing.assert_close(m2.params[k], m.params[k], rtol=0, atol=0)
    assert opt2.iterations == 5
    torch.testing.assert_close(opt2._v[m.offsets['W0']:m.offsets['W0'] + 10], opt._v[m.offsets['W0']:m.offsets['W0'] + 10])


def _trackable_classes():
    """TrackableObjectGraph from the public trackable_object_graph.proto field numbers
    (TrackableObject: children = 1, attributes = 2, slot_variables = 3;
    ObjectReference: node_id = 1, local_name = 2; SerializedTensor: name = 1,
    full_name = 2, checkpoint_key = 3; SlotVariableReference:
    original_variable_node_id = 1, slot_name = 2, slot_variable_node_id = 3)."""
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    fd = descriptor_pb2.FileDescriptorProto(name='srf_test_trackable.proto', package='tft', syntax='proto3')
    F = descriptor_pb2.FieldDescriptorProto
    rep, opt = F.LABEL_REPEATED, F.LABEL_OPTIONAL
    g = fd.message_type.add(name='TrackableObjectGraph')
    g.field.add(name='nodes', number=1, type=F.TYPE_MESSAGE, label=rep,
                type_name='.tft.TrackableObjectGraph.TrackableObject')
    t = g.nested_type.add(name='TrackableObject')
    base = '.tft.TrackableObjectGraph.TrackableObject.'
    t.field.add(name='children', number=1, type=F.TYPE_MESSAGE, label=rep, type_name=base + 'ObjectReference')
    t.field.add(name='attributes', number=2, type=F.TYPE_MESSAGE, label=rep, type_name=base + 'SerializedTensor')
    t.field.add(name='slot_variables', number=3, type=F.TYPE_MESSAGE, label=rep,
                type_name=base + 'SlotVariableReference')
    o = t.nested_type.add(name='ObjectReference')
    o.field.add(name='node_id', number=1, type=F.TYPE_INT32, label=opt)
    o.field.add(name='local_name', number=2, type=F.TYPE_STRING, label=opt)
    st = t.nested_type.add(name='SerializedTensor')
    for n, k in (('name', 1), ('full_name', 2), ('checkpoint_key', 3)):
        st.field.add(name=n, number=k, type=F.TYPE_STRING, label=opt)
    sv = t.nested_type.add(name='SlotVariableReference')
    sv.field.add(name='original_variable_node_id', number=1, type=F.TYPE_INT32, label=opt)
    sv.field.add(name='slot_name', number=2, type=F.TYPE_STRING, label=opt)
    sv.field.add(name='slot_variable_node_id', number=3, type=F.TYPE_INT32, label=opt)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName('tft.TrackableObjectGraph'))


def test_bundle_object_graph_restorable_by_path(tmp_path):
    """The TF bundles carry a _CHECKPOINTABLE_OBJECT_GRAPH that protobuf parses as a
    TrackableObjectGraph and re-serialises to the same bytes; walking the root's
    children by the names of each key's object path (what tf.train.Checkpoint.restore
    does, misc_helper.py:141-156) reaches a node whose VARIABLE_VALUE attribute is
    exactly that key, for every model, optimizer and save-counter tensor; and every
    Adam m / v slot is referenced from the optimizer node with its own key."""
    from srf_amd import tf_bundle
    model, opt = _model(1), SrfAdam(CustomSchedule(0.5, 1, 1200))
    opt._m = torch.randn(model.n_flat)
    opt._v = torch.rand(model.n_flat)
    opt.iterations = 5
    mgr = ck.CheckpointManager(model, opt, str(tmp_path / 'ck'), max_to_keep=2)
    prefix = mgr.save()
    raw = tf_bundle.read_object_graph(prefix, raw=True)
    G = _trackable_classes()
    g = G()
    g.ParseFromString(raw)
    assert g.SerializeToString() == raw
    keys = [k for k, _, _ in tf_bundle.list_variables(prefix) if k != tf_bundle.OBJECT_GRAPH_KEY]
    nodes = g.nodes
    assert {c.local_name for c in nodes[0].children} == {'model', 'optimizer', 'save_counter'}
    seen = set()
    for k in keys:
        if '.OPTIMIZER_SLOT' in k:
            continue
        nid = 0
        for part in k[:-len('/.ATTRIBUTES/VARIABLE_VALUE')].split('/'):
            nid = next(c.node_id for c in nodes[nid].children if c.local_name == part)
        assert [a.checkpoint_key for a in nodes[nid].attributes] == [k]
        assert nodes[nid].attributes[0].name == 'VARIABLE_VALUE'
        seen.add(k)
    opt_node = next(c.node_id for c in nodes[0].children if c.local_name == 'optimizer')
    slots = nodes[opt_node].slot_variables
    slot_keys = sorted(k for k in keys if '.OPTIMIZER_SLOT' in k)
    assert len(slots) == len(slot_keys) > 0
    for s in slots:
        sk = nodes[s.slot_variable_node_id].attributes[0].checkpoint_key
        orig = nodes[s.original_variable_node_id].attributes[0].checkpoint_key
        assert sk == orig.replace('/.ATTRIBUTES/', f'/.OPTIMIZER_SLOT/optimizer/{s.slot_name}/.ATTRIBUTES/')
        seen.add(sk)
    assert seen == set(keys)
    # the graph round-trips through our own decoder too, and restore still reads the tensors
    assert tf_bundle.decode_object_graph(raw) == tf_bundle.object_graph(keys)
    model2, opt2 = _model(9), SrfAdam(CustomSchedule(0.5, 1, 1200))
    assert ck.restore(prefix, model2, opt2) == 1
    for k in model.params:
        torch.testing.assert_close(model2.params[k], model.params[k], rtol=0, atol=0)
    assert opt2.iterations == 5
