"""TensorFlow V2 checkpoint ("tensor bundle") reader and writer -- no tensorflow.

The reference converts Google's original BERT checkpoints with
``tf.train.list_variables`` / ``tf.train.load_variable``
(hetseq/bert_modeling.py:43-101, ``load_tf_weights_in_bert``), i.e. it needs a
full TensorFlow install.  TensorFlow is not available here, so the on-disk
format is decoded directly:

* ``<prefix>.index`` is an SSTable (LevelDB table layout): data blocks of
  prefix-compressed ``(key, value)`` entries with a restart array, a 5-byte
  block trailer (compression type + masked CRC32C), an index block of block
  handles, and a 48-byte footer ending in the magic ``0xdb4775248b80fb57``.
  Blocks may be Snappy-compressed (decoder below); TensorFlow writes bundles
  uncompressed.
* The entry with the empty key is a ``BundleHeaderProto`` (``num_shards``,
  ``endianness``); every other key is a variable name whose value is a
  ``BundleEntryProto`` (``dtype``, ``shape``, ``shard_id``, ``offset``,
  ``size``, masked ``crc32c``).
* ``<prefix>.data-SSSSS-of-NNNNN`` hold the raw little-endian tensor bytes.

Protobuf messages are decoded with a small wire-format parser (varint /
fixed32 / fixed64 / length-delimited), so no generated TF protos are needed.
Tensor payloads are memory-mapped, and the optional CRC check runs in the
native runtime (``_data_native.crc32c``, SSE4.2 when the host has it).

``write_tf_checkpoint`` produces the same layout (used to build test fixtures
and to export weights under TF names); parity against checkpoints written by
real TensorFlow is unpinned in this environment (no TF, no network).
"""
import os
import re
import struct

import numpy as np

MAGIC = 0xdb4775248b80fb57
BLOCK_TRAILER = 5
FOOTER_LEN = 48

# tensorflow/core/framework/types.proto
_DT_TO_NP = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8, 9: np.int64,
             10: np.bool_, 17: np.uint16, 19: np.float16, 22: np.uint32, 23: np.uint64}
DT_BFLOAT16 = 14
_NP_TO_DT = {np.dtype(v): k for k, v in _DT_TO_NP.items()}


# ----------------------------------------------------------------------------- checksums
def _py_crc32c(data, crc=0):
    tbl = _py_crc32c.table
    if tbl is None:
        tbl = []
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
            tbl.append(c)
        _py_crc32c.table = tbl
    crc ^= 0xFFFFFFFF
    for b in bytes(data):
        crc = tbl[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


_py_crc32c.table = None


def crc32c(data):
    """CRC32C (Castagnoli) of a bytes-like object; native when the extension is built."""
    try:
        from .. import _data_native
        fn = getattr(_data_native, 'crc32c', None)
    except ImportError:
        fn = None
    if fn is not None:
        return fn(np.frombuffer(memoryview(data).cast('B'), dtype=np.uint8))
    return _py_crc32c(data)


def mask_crc(crc):
    return (((crc >> 15) | (crc << 17)) + 0xa282ead8) & 0xFFFFFFFF


def unmask_crc(masked):
    rot = (masked - 0xa282ead8) & 0xFFFFFFFF
    return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF


# ----------------------------------------------------------------------------- wire format
def _varint(buf, pos):
    result, shift = 0, 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def _enc_varint(v):
    if v < 0:
        v += 1 << 64
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _signed64(v):
    return v - (1 << 64) if v >= 1 << 63 else v


def _pb_fields(buf):
    """Decode one protobuf message into a list of (field_number, value)."""
    pos, out = 0, []
    while pos < len(buf):
        key, pos = _varint(buf, pos)
        field, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from('<Q', buf, pos)[0]
            pos += 8
        elif wt == 2:
            n, pos = _varint(buf, pos)
            v = bytes(buf[pos:pos + n])
            pos += n
        elif wt == 5:
            v = struct.unpack_from('<I', buf, pos)[0]
            pos += 4
        else:
            raise ValueError('unsupported protobuf wire type {}'.format(wt))
        out.append((field, v))
    return out


def _pb_field(field, wt, payload):
    key = _enc_varint((field << 3) | wt)
    if wt == 0:
        return key + _enc_varint(payload)
    if wt == 2:
        return key + _enc_varint(len(payload)) + payload
    if wt == 5:
        return key + struct.pack('<I', payload)
    raise ValueError(wt)


# ----------------------------------------------------------------------------- snappy
def snappy_decompress(src):
    """Raw Snappy block decoder (the compression LevelDB tables may use)."""
    src = bytes(src)
    n, pos = _varint(src, 0)
    out = bytearray()
    while pos < len(src):
        tag = src[pos]
        pos += 1
        t = tag & 3
        if t == 0:
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(src[pos:pos + nb], 'little')
                pos += nb
            ln += 1
            out += src[pos:pos + ln]
            pos += ln
            continue
        if t == 1:
            ln = ((tag >> 2) & 7) + 4
            off = ((tag >> 5) << 8) | src[pos]
            pos += 1
        elif t == 2:
            ln = (tag >> 2) + 1
            off = int.from_bytes(src[pos:pos + 2], 'little')
            pos += 2
        else:
            ln = (tag >> 2) + 1
            off = int.from_bytes(src[pos:pos + 4], 'little')
            pos += 4
        if off == 0 or off > len(out):
            raise ValueError('corrupt snappy stream')
        start = len(out) - off
        if off >= ln:
            out += out[start:start + ln]
        else:                      # overlapping copy (run-length style)
            for i in range(ln):
                out.append(out[start + i])
    if len(out) != n:
        raise ValueError('snappy length mismatch')
    return bytes(out)


# ----------------------------------------------------------------------------- SSTable
def _read_block(f, offset, size, verify):
    f.seek(offset)
    raw = f.read(size + BLOCK_TRAILER)
    if len(raw) != size + BLOCK_TRAILER:
        raise ValueError('truncated table block')
    contents, ctype = raw[:size], raw[size]
    if verify:
        want = unmask_crc(struct.unpack_from('<I', raw, size + 1)[0])
        if crc32c(raw[:size + 1]) != want:
            raise ValueError('table block checksum mismatch')
    if ctype == 1:
        contents = snappy_decompress(contents)
    elif ctype != 0:
        raise ValueError('unsupported table block compression {}'.format(ctype))
    return contents


def _block_entries(data):
    n_restarts = struct.unpack_from('<I', data, len(data) - 4)[0]
    end = len(data) - 4 - 4 * n_restarts
    pos, key = 0, b''
    while pos < end:
        shared, pos = _varint(data, pos)
        non_shared, pos = _varint(data, pos)
        vlen, pos = _varint(data, pos)
        key = key[:shared] + bytes(data[pos:pos + non_shared])
        pos += non_shared
        yield key, bytes(data[pos:pos + vlen])
        pos += vlen


def read_table(path, verify=False):
    """All (key, value) pairs of an SSTable file, in key order."""
    with open(path, 'rb') as f:
        f.seek(0, os.SEEK_END)
        flen = f.tell()
        if flen < FOOTER_LEN:
            raise ValueError('{}: too small for a table'.format(path))
        f.seek(flen - FOOTER_LEN)
        footer = f.read(FOOTER_LEN)
        lo, hi = struct.unpack_from('<II', footer, 40)
        if (hi << 32) | lo != MAGIC:
            raise ValueError('{}: not an SSTable (bad magic)'.format(path))
        pos = 0
        _, pos = _varint(footer, pos)      # metaindex offset / size (unused)
        _, pos = _varint(footer, pos)
        idx_off, pos = _varint(footer, pos)
        idx_size, pos = _varint(footer, pos)
        out = []
        for _, handle in _block_entries(_read_block(f, idx_off, idx_size, verify)):
            off, p = _varint(handle, 0)
            size, _ = _varint(handle, p)
            out.extend(_block_entries(_read_block(f, off, size, verify)))
        return out


def _build_block(kvs, restart_interval=16):
    buf, restarts, last = bytearray(), [], b''
    for i, (k, v) in enumerate(kvs):
        shared = 0
        if i % restart_interval == 0:
            restarts.append(len(buf))
        else:
            while shared < min(len(last), len(k)) and last[shared] == k[shared]:
                shared += 1
        buf += _enc_varint(shared) + _enc_varint(len(k) - shared) + _enc_varint(len(v)) + k[shared:] + v
        last = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        buf += struct.pack('<I', r)
    buf += struct.pack('<I', len(restarts))
    return bytes(buf)


def write_table(path, kvs, block_size=4096):
    """Write (key, value) byte pairs as an uncompressed SSTable (sorted by key)."""
    kvs = sorted(kvs, key=lambda kv: kv[0])
    with open(path, 'wb') as f:
        def put_block(contents):
            off = f.tell()
            f.write(contents)
            f.write(b'\x00' + struct.pack('<I', mask_crc(crc32c(contents + b'\x00'))))
            return _enc_varint(off) + _enc_varint(len(contents))

        index, cur, cur_bytes = [], [], 0
        for k, v in kvs:
            cur.append((k, v))
            cur_bytes += len(k) + len(v) + 6
            if cur_bytes >= block_size:
                index.append((cur[-1][0], put_block(_build_block(cur))))
                cur, cur_bytes = [], 0
        if cur:
            index.append((cur[-1][0], put_block(_build_block(cur))))
        meta = put_block(_build_block([]))
        idx = put_block(_build_block(index, restart_interval=1))
        footer = meta + idx
        footer += b'\x00' * (40 - len(footer)) + struct.pack('<II', MAGIC & 0xFFFFFFFF, MAGIC >> 32)
        f.write(footer)


# ----------------------------------------------------------------------------- bundle
def _resolve_prefix(path):
    if path.endswith('.index'):
        return path[:-len('.index')]
    if os.path.isdir(path):
        state = os.path.join(path, 'checkpoint')
        if os.path.exists(state):
            with open(state, 'r', encoding='utf-8') as fh:
                m = re.search(r'^model_checkpoint_path:\s*"([^"]+)"', fh.read(), re.M)
            if m:
                p = m.group(1)
                return p if os.path.isabs(p) else os.path.join(path, p)
        cands = sorted(n[:-6] for n in os.listdir(path) if n.endswith('.index'))
        if len(cands) == 1:
            return os.path.join(path, cands[0])
        raise FileNotFoundError('{}: no unique TF checkpoint (.index) found'.format(path))
    return path


class TFCheckpointReader(object):
    """``list_variables()`` / ``get_tensor(name)`` over a TF V2 checkpoint."""

    def __init__(self, path, verify=False):
        self.prefix = _resolve_prefix(path)
        index = self.prefix + '.index'
        if not os.path.exists(index):
            raise FileNotFoundError('TF checkpoint index not found: {}'.format(index))
        self.verify = verify
        self.num_shards = 1
        self._entries = {}
        for key, val in read_table(index, verify=verify):
            if key == b'':
                for field, v in _pb_fields(val):
                    if field == 1:
                        self.num_shards = v
                    elif field == 2 and v != 0:
                        raise ValueError('big-endian TF checkpoints are not supported')
                continue
            self._entries[key.decode('utf-8')] = self._parse_entry(val)
        self._maps = {}

    @staticmethod
    def _parse_entry(val):
        e = {'dtype': 1, 'shape': (), 'shard_id': 0, 'offset': 0, 'size': 0, 'crc32c': None}
        for field, v in _pb_fields(val):
            if field == 1:
                e['dtype'] = v
            elif field == 2:
                dims = []
                for f2, d in _pb_fields(v):
                    if f2 == 2:
                        size = 0
                        for f3, s in _pb_fields(d):
                            if f3 == 1:
                                size = _signed64(s)
                        dims.append(size)
                e['shape'] = tuple(dims)
            elif field == 3:
                e['shard_id'] = v
            elif field == 4:
                e['offset'] = _signed64(v)
            elif field == 5:
                e['size'] = _signed64(v)
            elif field == 6:
                e['crc32c'] = v
            elif field == 7:
                e['sliced'] = True
        return e

    def list_variables(self):
        return [(n, list(e['shape'])) for n, e in sorted(self._entries.items())]

    def has_tensor(self, name):
        return name in self._entries

    def _shard(self, sid):
        m = self._maps.get(sid)
        if m is None:
            path = '{}.data-{:05d}-of-{:05d}'.format(self.prefix, sid, self.num_shards)
            m = np.memmap(path, dtype=np.uint8, mode='r') if os.path.getsize(path) else np.zeros(0, np.uint8)
            self._maps[sid] = m
        return m

    def get_tensor(self, name):
        e = self._entries[name]
        if e.get('sliced'):
            raise NotImplementedError('{}: partitioned (sliced) variables are not supported'.format(name))
        raw = self._shard(e['shard_id'])[e['offset']:e['offset'] + e['size']]
        if len(raw) != e['size']:
            raise ValueError('{}: tensor bytes past the end of its data shard'.format(name))
        if self.verify and e['crc32c'] is not None and crc32c(raw) != unmask_crc(e['crc32c']):
            raise ValueError('{}: tensor checksum mismatch'.format(name))
        if e['dtype'] == DT_BFLOAT16:
            u = np.frombuffer(raw.tobytes(), dtype='<u2').astype(np.uint32) << 16
            return u.view(np.float32).reshape(e['shape'])
        if e['dtype'] not in _DT_TO_NP:
            raise NotImplementedError('{}: TF dtype {} not supported'.format(name, e['dtype']))
        dt = np.dtype(_DT_TO_NP[e['dtype']]).newbyteorder('<')
        return np.frombuffer(raw.tobytes(), dtype=dt).reshape(e['shape'])


def list_variables(path):
    return TFCheckpointReader(path).list_variables()


def load_variable(path, name):
    return TFCheckpointReader(path).get_tensor(name)


def write_tf_checkpoint(prefix, tensors):
    """Write ``{name: ndarray}`` as a single-shard TF V2 checkpoint at ``prefix``
    (``prefix.index`` + ``prefix.data-00000-of-00001`` + a ``checkpoint`` state file)."""
    os.makedirs(os.path.dirname(os.path.abspath(prefix)), exist_ok=True)
    kvs = [(b'', _pb_field(1, 0, 1) + _pb_field(3, 2, _pb_field(1, 0, 1)))]   # num_shards, version{producer}
    with open(prefix + '.data-00000-of-00001', 'wb') as f:
        off = 0
        for name in sorted(tensors):
            a = np.asarray(tensors[name], order='C')   # (ascontiguousarray would make 0-d arrays 1-d)
            a = a.astype(a.dtype.newbyteorder('<'), copy=False)
            dt = _NP_TO_DT.get(np.dtype(a.dtype.str.replace('>', '<').replace('|', '<')),
                               _NP_TO_DT.get(a.dtype))
            if dt is None:
                raise TypeError('{}: dtype {} has no TF equivalent here'.format(name, a.dtype))
            b = a.tobytes()
            f.write(b)
            shape = b''.join(_pb_field(2, 2, _pb_field(1, 0, d)) for d in a.shape)
            entry = (_pb_field(1, 0, dt) + _pb_field(2, 2, shape) + _pb_field(4, 0, off) + _pb_field(5, 0, len(b))
                     + _pb_field(6, 5, mask_crc(crc32c(b))))
            kvs.append((name.encode('utf-8'), entry))
            off += len(b)
    write_table(prefix + '.index', kvs)
    with open(os.path.join(os.path.dirname(os.path.abspath(prefix)), 'checkpoint'), 'w', encoding='utf-8') as fh:
        fh.write('model_checkpoint_path: "{}"\n'.format(os.path.basename(prefix)))
