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
Only numeric dense tensors are decoded (DT_STRING entries such as
_CHECKPOINTABLE_OBJECT_GRAPH are listed but skipped), and only uncompressed
tables (TF writes its bundles uncompressed).  Written bundles carry no object
graph, so TF reads them with tf.train.load_checkpoint / list_variables rather
than Checkpoint.restore.

Parity: restated from the public table / tensor_bundle.proto formats; no
TF-written bundle ships in the reference and TF is not installed, so it is
pinned only by its own round trip and hand-built tables (parity unpinned).
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


def save_checkpoint(prefix, tensors):
    """Write {name: array} as a single-shard bundle (keys sorted, as TF's table needs)."""
    os.makedirs(os.path.dirname(os.path.abspath(prefix)), exist_ok=True)
    data = bytearray()
    entries = [(b'', _vi(1, 1) + _vi(2, 0) + _ld(3, _vi(1, 1)))]   # num_shards=1, LITTLE, version{producer=1}
    for name in sorted(tensors):
        a = np.ascontiguousarray(tensors[name])
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
