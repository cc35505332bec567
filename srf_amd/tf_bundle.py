"""TF checkpoint (TensorBundle) reader/writer without TensorFlow.

Lets a reference user bring a ``tf.train.Checkpoint`` of the SRF model
(misc_helper.py:139-163, average_ckpt_sr.py:168-179) into this framework and
write one back:
  * ``<prefix>.index``: a LevelDB-format table (TF core/lib/io/table): data blocks
    of prefix-compressed (key, value) entries with restart arrays, an index block
    of BlockHandles, a 48-byte footer ending in magic 0xdb4775248b80fb57; every
    block followed by a 1-byte compression type and a masked CRC-32C.
    Key "" holds BundleHeaderProto, every other key a BundleEntryProto
    (dtype=1, shape=2, shard_id=3, offset=4, size=5, crc32c=6 (masked), slices=7);
  * ``<prefix>.data-SSSSS-of-NNNNN``: raw little-endian tensor bytes.
Numeric dense tensors are decoded, and the scalar DT_STRING tensor
``_CHECKPOINTABLE_OBJECT_GRAPH`` (read_object_graph); only uncompressed tables
(TF writes its bundles uncompressed).  Written bundles carry that object graph --
a TrackableObjectGraph (trackable_object_graph.proto) whose children follow the
object paths of the keys (``model/conv/conv_layers/0/0/kernel`` ...), with the
optimizer's slot variables -- so ``tf.train.Checkpoint(optimizer=, model=)
.restore(prefix)`` (misc_helper.py:141-156, average_ckpt_sr.py:122-123) can match
them to the live objects by attribute name.

Parity: restated from the public table / tensor_bundle.proto /
trackable_object_graph.proto formats; no TF-written bundle ships in the reference
and TF is not installed, so it is pinned by its own round trip, hand-built tables
and protobuf's own serialisation of the object graph (parity against TF unpinned).
"""
import os
import struct

import numpy as np

from . import load_speech_data as _data

MAGIC = 0xdb4775248b80fb57
_DTYPES = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8, 9: np.int64,
           10: np.bool_, 17: np.uint16, 19: np.float16, 22: np.uint32, 23: np.uint64}
_DTYPE_IDS = {np.dtype(v): k for k, v in _DTYPES.items()}
DT_STRING = 7


def _crc_masked(b):
    return _data.lib().srf_crc32c_masked(bytes(b), len(b))


def _varint(buf, pos):
    v, s = 0, 0
    while True:
        b = buf[pos]
        pos += 1
        v |= (b & 0x7F) << s
        if not b & 0x80:
            return v, pos
        s += 7


def _put_varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


# ---------------------------------------------------------------- protobuf (tiny)
def _fields(buf):
    pos, out = 0, []
    while pos < len(buf):
        tag, pos = _varint(buf, pos)
        f, w = tag >> 3, tag & 7
        if w == 0:
            v, pos = _varint(buf, pos)
        elif w == 1:
            v = buf[pos:pos + 8]
            pos += 8
        elif w == 2:
            n, pos = _varint(buf, pos)
            v = buf[pos:pos + n]
            pos += n
        elif w == 5:
            v = buf[pos:pos + 4]
            pos += 4
        else:
            raise ValueError(f'unsupported wire type {w}')
        out.append((f, w, v))
    return out


def _parse_entry(buf):
    e = {'dtype': 0, 'shape': [], 'shard_id': 0, 'offset': 0, 'size': 0, 'crc32c': None}
    for f, w, v in _fields(buf):
        if f == 1:
            e['dtype'] = v
        elif f == 2:
            for sf, _, sv in _fields(v):
                if sf == 2:
                    size = 0
                    for df, _, dv in _fields(sv):
                        if df == 1:
                            size = dv
                    e['shape'].append(size)
        elif f == 3:
            e['shard_id'] = v
        elif f == 4:
            e['offset'] = v
        elif f == 5:
            e['size'] = v
        elif f == 6:
            e['crc32c'] = struct.unpack('<I', v)[0]
        elif f == 7:
            raise ValueError('sliced (partitioned) variables are not supported')
    return e


def _ld(field, body):
    return _put_varint((field << 3) | 2) + _put_varint(len(body)) + body


def _vi(field, v):
    return _put_varint(field << 3) + _put_varint(v) if v else b''


def _encode_entry(dtype, shape, shard_id, offset, size, crc):
    dims = b''.join(_ld(2, _vi(1, int(d)) if d else b'') for d in shape)
    return (_vi(1, dtype) + _ld(2, dims) + _vi(3, shard_id) + _vi(4, offset) + _vi(5, size)
            + _put_varint((6 << 3) | 5) + struct.pack('<I', crc))


# ---------------------------------------------------------------- table
def _read_block(data, off, size):
    body = data[off:off + size]
    ctype, crc = data[off + size], struct.unpack('<I', data[off + size + 1:off + size + 5])[0]
    if ctype != 0:
        raise ValueError('compressed table blocks are not supported')
    if _crc_masked(data[off:off + size + 1]) != crc:
        raise ValueError('table block CRC mismatch')
    n_restarts = struct.unpack('<I', body[-4:])[0]
    end = len(body) - 4 - 4 * n_restarts
    pos, key, out = 0, b'', []
    while pos < end:
        shared, pos = _varint(body, pos)
        non_shared, pos = _varint(body, pos)
        vlen, pos = _varint(body, pos)
        key = key[:shared] + body[pos:pos + non_shared]
        pos += non_shared
        out.append((bytes(key), bytes(body[pos:pos + vlen])))
        pos += vlen
    return out


def _read_table(path):
    data = open(path, 'rb').read()
    if len(data) < 48 or struct.unpack('<Q', data[-8:])[0] != MAGIC:
        raise ValueError(f'{path} is not a TF table (bad footer magic)')
    footer = data[-48:]
    _, pos = _varint(footer, 0)
    _, pos = _varint(footer, pos)
    idx_off, pos = _varint(footer, pos)
    idx_size, pos = _varint(footer, pos)
    out = []
    for _, handle in _read_block(data, idx_off, idx_size):
        off, p = _varint(handle, 0)
        size, _ = _varint(handle, p)
        out += _read_block(data, off, size)
    return out


def _block(entries, restart_interval=16):
    body, restarts, prev = bytearray(), [], b''
    for k, (key, value) in enumerate(entries):
        shared = 0
        if k % restart_interval == 0:
            restarts.append(len(body))
        else:
            while shared < min(len(prev), len(key)) and prev[shared] == key[shared]:
                shared += 1
        body += _put_varint(shared) + _put_varint(len(key) - shared) + _put_varint(len(value))
        body += key[shared:] + value
        prev = key
    if not restarts:
        restarts = [0]
    for r in restarts:
        body += struct.pack('<I', r)
    body += struct.pack('<I', len(restarts))
    return bytes(body)


def _write_table(path, entries, block_size=4096):
    out = bytearray()

    def emit(block):
        off = len(out)
        out.extend(block)
        trailer = b'\x00'
        out.extend(trailer + struct.pack('<I', _crc_masked(block + trailer)))
        return _put_varint(off) + _put_varint(len(block))

    index, cur, cur_bytes = [], [], 0
    for key, value in entries:
        cur.append((key, value))
        cur_bytes += len(key) + len(value) + 8
        if cur_bytes >= block_size:
            index.append((cur[-1][0], emit(_block(cur))))
            cur, cur_bytes = [], 0
    if cur:
        index.append((cur[-1][0], emit(_block(cur))))
    meta = emit(_block([]))
    idx = emit(_block(index, restart_interval=1))
    footer = meta + idx
    footer += b'\x00' * (40 - len(footer)) + struct.pack('<Q', MAGIC)
    out.extend(footer)
    with open(path, 'wb') as f:
        f.write(bytes(out))


# ---------------------------------------------------------------- bundle API
def list_variables(prefix):
    """[(name, shape, dtype id)] like tf.train.list_variables."""
    return [(k.decode(), e['shape'], e['dtype']) for k, e in _entries(prefix) if k]


def _entries(prefix):
    out = []
    for key, value in _read_table(prefix + '.index'):
        out.append((key, _parse_entry(value) if key else None))
    return out


OBJECT_GRAPH_KEY = '_CHECKPOINTABLE_OBJECT_GRAPH'
_ATTR = '/.ATTRIBUTES/VARIABLE_VALUE'
_SLOT = '/.OPTIMIZER_SLOT/'


def _ls(field, text):
    return _ld(field, text.encode())


def object_graph(keys):
    """TrackableObjectGraph of a checkpoint whose variables sit at ``keys`` (TF2
    object paths ``<path>/.ATTRIBUTES/VARIABLE_VALUE``; optimizer slots as
    ``<variable path>/.OPTIMIZER_SLOT/<optimizer path>/<slot>/.ATTRIBUTES/...``).
    Returns [{'children': [(local_name, node)], 'attributes': [(name, full_name,
    checkpoint_key)], 'slots': [(original_node, slot_name, slot_node)]}], node 0 the
    root; nodes in breadth-first order of the object tree, slot variables last."""
    nodes = [{'children': [], 'attributes': [], 'slots': []}]
    index = {(): 0}

    def node(path):
        path = tuple(path)
        if path not in index:
            parent = node(path[:-1])
            index[path] = len(nodes)
            nodes.append({'children': [], 'attributes': [], 'slots': []})
            nodes[parent]['children'].append((path[-1], index[path]))
        return index[path]

    plain = sorted(k for k in keys if k.endswith(_ATTR) and _SLOT not in k)
    for depth in range(1, max((k.count('/') for k in plain), default=0) + 2):   # breadth first
        for k in plain:
            parts = k[:-len(_ATTR)].split('/')
            if len(parts) >= depth:
                node(parts[:depth])
    for k in plain:
        path = k[:-len(_ATTR)]
        nodes[node(path.split('/'))]['attributes'].append(('VARIABLE_VALUE', path, k))
    for k in sorted(k for k in keys if k.endswith(_ATTR) and _SLOT in k):
        var, rest = k[:-len(_ATTR)].split(_SLOT)
        opt, slot = rest.rsplit('/', 1)
        sid = len(nodes)
        nodes.append({'children': [], 'attributes': [('VARIABLE_VALUE', f'{var}/{slot}', k)], 'slots': []})
        nodes[node(opt.split('/'))]['slots'].append((node(var.split('/')), slot, sid))
    return nodes


def encode_object_graph(nodes):
    """Wire bytes of TrackableObjectGraph {repeated TrackableObject nodes = 1}, with
    TrackableObject {children = 1 (ObjectReference {node_id = 1, local_name = 2}),
    attributes = 2 (SerializedTensor {name = 1, full_name = 2, checkpoint_key = 3}),
    slot_variables = 3 (SlotVariableReference {original_variable_node_id = 1,
    slot_name = 2, slot_variable_node_id = 3})} -- fields in number order, as
    protobuf serialises them."""
    out = b''
    for n in nodes:
        body = b''.join(_ld(1, _vi(1, nid) + _ls(2, name)) for name, nid in n['children'])
        body += b''.join(_ld(2, _ls(1, a) + _ls(2, fn) + _ls(3, ck)) for a, fn, ck in n['attributes'])
        body += b''.join(_ld(3, _vi(1, o) + _ls(2, sl) + _vi(3, sn)) for o, sl, sn in n['slots'])
        out += _ld(1, body)
    return out


def decode_object_graph(buf):
    nodes = []
    for f, _, v in _fields(buf):
        if f != 1:
            continue
        n = {'children': [], 'attributes': [], 'slots': []}
        for g, _, w in _fields(v):
            d = {h: x for h, _, x in _fields(w)}
            if g == 1:
                n['children'].append((bytes(d.get(2, b'')).decode(), d.get(1, 0)))
            elif g == 2:
                n['attributes'].append(tuple(bytes(d.get(h, b'')).decode() for h in (1, 2, 3)))
            elif g == 3:
                n['slots'].append((d.get(1, 0), bytes(d.get(2, b'')).decode(), d.get(3, 0)))
        nodes.append(n)
    return nodes


def _string_tensor(values):
    """tensor_bundle.cc's DT_STRING data: varint64 lengths, the masked CRC-32C of the
    length bytes, then the strings; returns (bytes, masked crc of all of them)."""
    lens = b''.join(_put_varint(len(v)) for v in values)
    data = lens + struct.pack('<I', _crc_masked(lens)) + b''.join(values)
    return data, _crc_masked(data)


def read_object_graph(prefix, raw=False):
    """The decoded _CHECKPOINTABLE_OBJECT_GRAPH of a bundle (raw=True: its wire
    bytes), or None."""
    header = {}
    for key, value in _read_table(prefix + '.index'):
        if key == b'':
            header = {f: v for f, _, v in _fields(value)}
        elif key == OBJECT_GRAPH_KEY.encode():
            e = _parse_entry(value)
            n_shards = header.get(1, 1) or 1
            raw_bytes = raw
            raw = open(f'{prefix}.data-{e["shard_id"]:05d}-of-{n_shards:05d}', 'rb').read()[
                e['offset']:e['offset'] + e['size']]
            if e['crc32c'] is not None and _crc_masked(raw) != e['crc32c']:
                raise ValueError('object graph CRC mismatch')
            n, pos = _varint(raw, 0)
            if _crc_masked(raw[:pos]) != struct.unpack('<I', raw[pos:pos + 4])[0]:
                raise ValueError('object graph length CRC mismatch')
            graph = bytes(raw[pos + 4:pos + 4 + n])
            return graph if raw_bytes else decode_object_graph(graph)
    return None


def load_checkpoint(prefix, verify_crc=True):
    """{name: numpy array} of every numeric tensor in the bundle."""
    ents = _entries(prefix)
    header = {}
    for key, value in _read_table(prefix + '.index'):
        if key == b'':
            header = {f: v for f, _, v in _fields(value)}
    n_shards = header.get(1, 1) or 1
    shards = {}
    out = {}
    for key, e in ents:
        if not key or e['dtype'] == DT_STRING:
            continue
        if e['dtype'] not in _DTYPES:
            raise ValueError(f'{key!r}: unsupported dtype {e["dtype"]}')
        sid = e['shard_id']
        if sid not in shards:
            shards[sid] = open(f'{prefix}.data-{sid:05d}-of-{n_shards:05d}', 'rb').read()
        raw = shards[sid][e['offset']:e['offset'] + e['size']]
        if verify_crc and e['crc32c'] is not None and _crc_masked(raw) != e['crc32c']:
            raise ValueError(f'{key!r}: tensor CRC mismatch')
        out[key.decode()] = np.frombuffer(raw, dtype=_DTYPES[e['dtype']]).reshape(e['shape']).copy()
    return out


def save_checkpoint(prefix, tensors, with_object_graph=True):
    """Write {name: array} as a single-shard bundle (keys sorted, as TF's table needs),
    with the object graph of its keys (object_graph) unless with_object_graph=False."""
    os.makedirs(os.path.dirname(os.path.abspath(prefix)), exist_ok=True)
    data = bytearray()
    entries = [(b'', _vi(1, 1) + _vi(2, 0) + _ld(3, _vi(1, 1)))]   # num_shards=1, LITTLE, version{producer=1}
    names = sorted(tensors) + ([OBJECT_GRAPH_KEY] if with_object_graph else [])
    for name in sorted(names):
        if name == OBJECT_GRAPH_KEY:
            raw, crc = _string_tensor([encode_object_graph(object_graph(list(tensors)))])
            entries.append((name.encode(), _encode_entry(DT_STRING, (), 0, len(data), len(raw), crc)))
            data += raw
            continue
        a = np.asarray(tensors[name])
        a = a if a.flags['C_CONTIGUOUS'] else a.copy(order='C')   # scalars stay 0-d (TF scalar variables)
        dt = _DTYPE_IDS.get(a.dtype)
        if dt is None:
            raise ValueError(f'{name}: dtype {a.dtype} not supported')
        raw = a.tobytes()
        entries.append((name.encode(), _encode_entry(dt, a.shape, 0, len(data), len(raw), _crc_masked(raw))))
        data += raw
    with open(prefix + '.data-00000-of-00001', 'wb') as f:
        f.write(bytes(data))
    _write_table(prefix + '.index', entries)


def restore_from_tf(prefix, model, optimizer=None):
    """Load a TF-format bundle whose keys follow checkpoint.tf_variable_map."""
    from . import checkpoint
    state = load_checkpoint(prefix)
    unused = checkpoint.load_model_state(model, state, strict=False)
    if optimizer is not None:
        checkpoint.load_optimizer_state(model, optimizer, state)
    return unused


def export_to_tf(prefix, model, optimizer=None):
    from . import checkpoint
    state = checkpoint.model_state(model)
    if optimizer is not None:
        state.update(checkpoint.optimizer_state(model, optimizer))
    save_checkpoint(prefix, state)
