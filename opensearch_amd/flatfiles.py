"""Lucene99 flat vector files (.vec data + .vemf meta): the on-disk source of segment staging.

OpenSearch 3.3 keeps vector fields in Lucene's flat vectors format ([L] Lucene99FlatVectorsFormat,
lucene-core 10.3.0, un-vendored: gradle/libs.versions.toml:3) under its default codec
(S/index/codec/CodecService.java:75-99); `.vec` is memory-mapped and `.vem*` read through NIO under
hybridfs (S/index/IndexModule.java:215-233, S/index/store/FsDirectoryFactory.java:98-110).  A segment
opened by an NRT refresh (S/index/engine/InternalEngine.java:584-589) is staged into HBM once from
those files: `GpuFlatVectorsReader.from_files` reads the field's entry from `.vemf` here and hands the
`.vec` slice to `osk_seg_stage_file` (mmap → pinned staging ring → HBM, libosknn).

This module restates the published layout — PARITY UNPINNED: there is no Lucene jar or index fixture
in the reference or the image, so files written here are checked against this restatement only:

  header   CodecUtil.writeIndexHeader: BE int 0x3FD76C17, codec name (vInt length + UTF-8), BE int
           version, 16-byte segment id, suffix (byte length + bytes)
  .vec     header "Lucene99FlatVectorsFormatData"; per field: aligned to the element size, the rows
           little-endian (n × dim × 4 B float32 or n × dim B int8); for a sparse field the
           docsWithField IndexedDISI and the ord→doc DirectMonotonic block follow; footer
  .vemf    header "Lucene99FlatVectorsFormatMeta"; per field: int number, int encoding ordinal, int
           similarity ordinal, vLong data offset, vLong data length, vInt dimension, int count, then
           OrdToDocDISIReaderConfiguration (long docsWithFieldOffset: −2 empty, −1 dense, else the
           IndexedDISI offset in .vec; long its length; short jump-table entries; byte dense rank power;
           sparse only: long ord→doc offset, vInt block shift, DirectMonotonic meta, long its length);
           int −1 ends the fields; footer
  footer   CodecUtil.writeFooter: BE int ~0x3FD76C17, BE int 0, BE long CRC32 of everything before
  ints     DataOutput.writeInt/Short/Long are little-endian (Lucene ≥ 9)
  IndexedDISI  per 65536-doc block with docs: short block, short cardinality−1, then SPARSE
           (≤ 4095 docs: a short per doc), DENSE (a 2-byte big-endian rank entry per 512 docs, then
           1024 LE longs) or ALL (65536 docs: nothing); a NO_MORE_DOCS block (0x7FFF, 0xFFFF) ends it,
           then the jump table (int index, int offset per block up to the last one)
The ord→doc map of a sparse field is the IndexedDISI's iteration order (ord i = its i-th doc), which is
what the reader decodes; the DirectMonotonic copy is written for layout fidelity but not needed here.
"""
from __future__ import annotations

import ctypes as C
import os
import struct
import zlib
from dataclasses import dataclass

import numpy as np

CODEC_MAGIC = 0x3FD76C17
FOOTER_MAGIC = (~CODEC_MAGIC) & 0xFFFFFFFF
META_CODEC = "Lucene99FlatVectorsFormatMeta"
DATA_CODEC = "Lucene99FlatVectorsFormatData"
VERSION = 0
DIRECT_MONOTONIC_BLOCK_SHIFT = 16
DENSE_RANK_POWER = 9
BLOCK = 1 << 16
MAX_ARRAY_LENGTH = (1 << 12) - 1
NO_MORE_DOCS = 0x7FFFFFFF


class CorruptIndexError(ValueError):
    """[L] CorruptIndexException: a header, footer or checksum that does not match."""


# ------------------------------------------------------------------------------------------------
# DataOutput / DataInput primitives
# ------------------------------------------------------------------------------------------------
class _Out:
    def __init__(self):
        self.b = bytearray()

    def pos(self):
        return len(self.b)

    def byte(self, v):
        self.b += struct.pack("<b", v)

    def short(self, v):
        self.b += struct.pack("<h", v)

    def int_(self, v):
        self.b += struct.pack("<i", v)

    def long(self, v):
        self.b += struct.pack("<q", v)

    def be_int(self, v):
        self.b += struct.pack(">I", v & 0xFFFFFFFF)

    def be_long(self, v):
        self.b += struct.pack(">Q", v & 0xFFFFFFFFFFFFFFFF)

    def vlong(self, v):
        if v < 0:
            raise ValueError("negative vLong")
        while v >= 0x80:
            self.b.append((v & 0x7F) | 0x80)
            v >>= 7
        self.b.append(v)

    vint = vlong

    def string(self, s):
        raw = s.encode()
        self.vint(len(raw))
        self.b += raw

    def raw(self, data):
        self.b += data

    def align(self, n):
        while len(self.b) % n:
            self.b.append(0)


class _In:
    def __init__(self, data: bytes, pos: int = 0):
        self.d, self.p = data, pos

    def _take(self, n):
        if self.p + n > len(self.d):
            raise CorruptIndexError("read past EOF")
        v = self.d[self.p:self.p + n]
        self.p += n
        return v

    def byte(self):
        return struct.unpack("<b", self._take(1))[0]

    def short(self):
        return struct.unpack("<h", self._take(2))[0]

    def int_(self):
        return struct.unpack("<i", self._take(4))[0]

    def long(self):
        return struct.unpack("<q", self._take(8))[0]

    def be_int(self):
        return struct.unpack(">I", self._take(4))[0]

    def be_long(self):
        return struct.unpack(">Q", self._take(8))[0]

    def vlong(self):
        v, shift = 0, 0
        while True:
            b = self._take(1)[0]
            v |= (b & 0x7F) << shift
            if b < 0x80:
                return v
            shift += 7
            if shift > 63:
                raise CorruptIndexError("invalid vLong")

    vint = vlong

    def string(self):
        return self._take(self.vint()).decode()


def _write_header(o: _Out, codec: str, segment_id: bytes, suffix: str, version: int = VERSION):
    """[L] CodecUtil.writeIndexHeader: BE magic, codec name (vInt length + bytes), BE version, the
    16-byte segment id, suffix (one length byte + bytes)."""
    o.be_int(CODEC_MAGIC)
    o.string(codec)
    o.be_int(version)
    o.raw(segment_id)
    raw = suffix.encode()
    o.b.append(len(raw))
    o.raw(raw)


def _check_header(i: _In, codec: str, segment_id: bytes, suffix: str, min_version: int = VERSION,
                  max_version: int = VERSION) -> int:
    """[L] CodecUtil.checkIndexHeader; returns the version."""
    if i.be_int() != CODEC_MAGIC:
        raise CorruptIndexError("codec header mismatch")
    name = i.string()
    if name != codec:
        raise CorruptIndexError(f"codec mismatch: expected {codec!r}, got {name!r}")
    version = i.be_int()
    if not min_version <= version <= max_version:
        raise CorruptIndexError(f"unsupported version {version}")
    if i._take(16) != segment_id:
        raise CorruptIndexError("segment id mismatch")
    n = i._take(1)[0]
    if i._take(n).decode() != suffix:
        raise CorruptIndexError("segment suffix mismatch")
    return version


def _write_footer(o: _Out):
    o.be_int(FOOTER_MAGIC)
    o.be_int(0)
    o.be_long(zlib.crc32(bytes(o.b)))   # CRC32 of everything before it, footer magic and algorithm included


def _check_footer(data: bytes):
    if len(data) < 16:
        raise CorruptIndexError("file too short for a footer")
    magic, algo, crc = struct.unpack(">IIQ", data[-16:])
    if magic != FOOTER_MAGIC or algo != 0:
        raise CorruptIndexError("codec footer mismatch")
    if zlib.crc32(data[:-8]) != crc:
        raise CorruptIndexError("checksum failed")


# ------------------------------------------------------------------------------------------------
# IndexedDISI
# ------------------------------------------------------------------------------------------------
def _write_indexed_disi(o: _Out, docs: np.ndarray) -> int:
    """IndexedDISI.writeBitSet of ascending docs into o; returns the jump-table entry count."""
    start = o.pos()
    blocks = docs >> 16
    jumps = []   # (index of the block's first doc, offset of the block) for every block up to the last
    index = 0
    last_block = int(blocks[-1]) if len(docs) else -1
    uniq, first = np.unique(blocks, return_index=True)
    bounds = list(first) + [len(docs)]
    present = {int(b): (int(bounds[j]), int(bounds[j + 1])) for j, b in enumerate(uniq)}
    for blk in range(last_block + 1):
        jumps.append((index, o.pos() - start))
        if blk not in present:
            continue
        a, b = present[blk]
        lows = (docs[a:b] & 0xFFFF).astype(np.int64)
        card = b - a
        o.short(np.int16(np.uint16(blk)).item())
        o.short(np.int16(np.uint16(card - 1)).item())
        if card > MAX_ARRAY_LENGTH:
            if card != BLOCK:   # DENSE: rank table (BE shorts, one per 512 docs) + 1024 LE longs
                bits = np.zeros(BLOCK, bool)
                bits[lows] = True
                csum = np.concatenate([[0], np.cumsum(bits)])
                for r in range(0, BLOCK, 1 << DENSE_RANK_POWER):
                    o.raw(struct.pack(">H", int(csum[r]) & 0xFFFF))
                o.raw(np.packbits(bits, bitorder="little").tobytes())
        else:
            o.raw(lows.astype("<u2").tobytes())
        index += card
    o.short(np.int16(np.uint16(NO_MORE_DOCS >> 16)).item())
    o.short(np.int16(np.uint16(NO_MORE_DOCS & 0xFFFF)).item())
    if len(jumps) <= 1:
        return 0   # a single block needs no jump table
    for idx, off in jumps:
        o.int_(idx)
        o.int_(off)
    return len(jumps)


def read_indexed_disi(data: bytes, offset: int, length: int, rank_power: int) -> np.ndarray:
    """All docs of an IndexedDISI written at data[offset:offset+length], ascending (= ord order)."""
    i = _In(data, offset)
    end = offset + length
    out = []
    while i.p < end:
        blk = i.short() & 0xFFFF
        card = (i.short() & 0xFFFF) + 1
        if blk == NO_MORE_DOCS >> 16:
            break
        base = blk << 16
        if card > MAX_ARRAY_LENGTH:
            if card == BLOCK:
                out.append(np.arange(base, base + BLOCK, dtype=np.int64))
            else:
                if rank_power != -1:
                    i._take(2 * (BLOCK >> rank_power))
                words = np.frombuffer(i._take(BLOCK // 8), np.uint8)
                lows = np.nonzero(np.unpackbits(words, bitorder="little"))[0]
                if len(lows) != card:
                    raise CorruptIndexError("dense block cardinality mismatch")
                out.append(base + lows.astype(np.int64))
        else:
            lows = np.frombuffer(i._take(2 * card), "<u2").astype(np.int64)
            out.append(base + lows)
    return np.concatenate(out).astype(np.int32) if out else np.zeros(0, np.int32)


# ------------------------------------------------------------------------------------------------
# DirectMonotonic (written for layout fidelity: ord → doc, blocks of 2^shift values)
# ------------------------------------------------------------------------------------------------
def _write_direct_monotonic(meta: _Out, data: _Out, values: np.ndarray, shift: int):
    base = data.pos()
    for s in range(0, len(values), 1 << shift):
        v = values[s:s + (1 << shift)].astype(np.int64)
        n = len(v)
        avg = float(v[-1] - v[0]) / max(1, n - 1) if n > 1 else 0.0
        expected = (np.arange(n) * np.float32(avg)).astype(np.int64)
        deltas = v - expected
        mn = int(deltas.min())
        deltas = deltas - mn
        maxd = int(deltas.max())
        bpv = 0 if maxd == 0 else maxd.bit_length()
        meta.long(mn)
        meta.int_(struct.unpack("<i", struct.pack("<f", avg))[0])
        meta.long(data.pos() - base)
        meta.byte(bpv)
        if bpv:
            acc, nbits, buf = 0, 0, bytearray()
            for d in deltas.tolist():
                acc |= d << nbits
                nbits += bpv
                while nbits >= 8:
                    buf.append(acc & 0xFF)
                    acc >>= 8
                    nbits -= 8
            if nbits:
                buf.append(acc & 0xFF)
            data.raw(bytes(buf))


# ------------------------------------------------------------------------------------------------
# segment files
# ------------------------------------------------------------------------------------------------
@dataclass
class FieldEntry:
    """One field of a .vemf meta file ([L] Lucene99FlatVectorsReader.FieldEntry)."""
    number: int
    encoding: int            # 0 FLOAT32, 1 BYTE
    similarity: int          # VectorSimilarityFunction ordinal
    data_offset: int         # of the rows in .vec
    data_length: int
    dim: int
    size: int                # vectors (= ords)
    docs_with_field_offset: int   # −2 empty, −1 dense, else IndexedDISI offset in .vec
    docs_with_field_length: int
    jump_table_entries: int
    dense_rank_power: int


def write_segment(directory: str, name: str, segment_id: bytes, max_doc: int, fields, suffix: str = ""):
    """Write `name[_suffix].vec` / `.vemf` for fields = [(number, vectors ndarray [n, dim] f32|i8, similarity,
    docs ascending int array or None = dense)].  Returns (vec_path, vemf_path)."""
    if len(segment_id) != 16:
        raise ValueError("segment id is 16 bytes")
    base = name + (f"_{suffix}" if suffix else "")
    data, meta = _Out(), _Out()
    _write_header(data, DATA_CODEC, segment_id, suffix)
    _write_header(meta, META_CODEC, segment_id, suffix)
    for number, vectors, sim, docs in fields:
        v = np.ascontiguousarray(vectors)
        enc = 1 if v.dtype == np.int8 else 0
        if enc == 0:
            v = v.astype("<f4", copy=False)
        n, dim = v.shape
        data.align(4 if enc == 0 else 1)
        off = data.pos()
        data.raw(v.tobytes())
        length = data.pos() - off
        meta.int_(number)
        meta.int_(enc)
        meta.int_(int(sim))
        meta.vlong(off)
        meta.vlong(length)
        meta.vint(dim)
        meta.int_(n)
        if n == 0:
            meta.long(-2), meta.long(0), meta.short(-1), meta.byte(-1)
        elif docs is None or n == max_doc:
            meta.long(-1), meta.long(0), meta.short(-1), meta.byte(-1)
        else:
            d = np.asarray(docs, np.int64)
            if len(d) != n or np.any(np.diff(d) <= 0) or d[0] < 0 or d[-1] >= max_doc:
                raise ValueError("docs must be n ascending doc ids in [0, max_doc)")
            dwf = data.pos()
            meta.long(dwf)
            jumps = _write_indexed_disi(data, d)
            meta.long(data.pos() - dwf)
            meta.short(jumps)
            meta.byte(DENSE_RANK_POWER)
            start = data.pos()
            meta.long(start)
            meta.vint(DIRECT_MONOTONIC_BLOCK_SHIFT)
            _write_direct_monotonic(meta, data, d, DIRECT_MONOTONIC_BLOCK_SHIFT)
            meta.long(data.pos() - start)
    meta.int_(-1)
    _write_footer(data)
    _write_footer(meta)
    vec = os.path.join(directory, base + ".vec")
    vemf = os.path.join(directory, base + ".vemf")
    with open(vec, "wb") as f:
        f.write(bytes(data.b))
    with open(vemf, "wb") as f:
        f.write(bytes(meta.b))
    return vec, vemf


def read_meta(vemf_path: str, segment_id: bytes, suffix: str = "") -> list[FieldEntry]:
    """Parse a .vemf file (header, fields until −1, footer + CRC32 checked)."""
    data = open(vemf_path, "rb").read()
    _check_footer(data)
    i = _In(data)
    _check_header(i, META_CODEC, segment_id, suffix)
    out = []
    while True:
        number = i.int_()
        if number == -1:
            break
        enc, sim = i.int_(), i.int_()
        off, length, dim, size = i.vlong(), i.vlong(), i.vint(), i.int_()
        dwf_off, dwf_len, jumps, rank = i.long(), i.long(), i.short(), i.byte()
        if dwf_off >= 0:   # sparse: skip the ord→doc DirectMonotonic meta
            i.long()
            shift = i.vint()
            for _ in range((size + (1 << shift) - 1) >> shift):
                i.long(), i.int_(), i.long(), i.byte()
            i.long()
        elem = 4 if enc == 0 else 1
        if length != size * dim * elem:
            raise CorruptIndexError(f"field {number}: data length {length} != {size}×{dim}×{elem}")
        out.append(FieldEntry(number, enc, sim, off, length, dim, size, dwf_off, dwf_len, jumps, rank))
    if i.p != len(data) - 16:
        raise CorruptIndexError("trailing bytes before the footer")
    return out


def check_data_file(vec_path: str, segment_id: bytes, suffix: str = "") -> None:
    """[L] CodecUtil.checksumEntireFile on .vec: header and footer CRC32."""
    data = open(vec_path, "rb").read()
    _check_footer(data)
    _check_header(_In(data), DATA_CODEC, segment_id, suffix)


def ord_to_doc(vec_path: str, entry: FieldEntry, max_doc: int) -> np.ndarray | None:
    """None for a dense field (doc == ord); else the ascending docs of the IndexedDISI (ord order)."""
    if entry.docs_with_field_offset == -1:
        return None
    if entry.docs_with_field_offset == -2:
        return np.zeros(0, np.int32)
    with open(vec_path, "rb") as f:
        data = f.read()
    docs = read_indexed_disi(data, entry.docs_with_field_offset, entry.docs_with_field_length,
                             entry.dense_rank_power)
    if len(docs) != entry.size or (len(docs) and docs[-1] >= max_doc):
        raise CorruptIndexError("docsWithField does not match the field's size / maxDoc")
    return docs


def stage_field(vec_path: str, entry: FieldEntry, max_doc: int, device: int = 0) -> int:
    """osk_seg_stage_file of one field: the .vec slice mmapped, staged through pinned buffers into HBM.
    Returns the osk_seg handle."""
    from ._lib import check, lib, ptr
    o2d = ord_to_doc(vec_path, entry, max_doc)
    h = C.c_void_p()
    check(lib().osk_seg_stage_file(device, vec_path.encode(), entry.data_offset, entry.size, entry.dim, entry.encoding,
                                   entry.similarity, ptr(o2d), max_doc, C.byref(h)))
    return h.value
