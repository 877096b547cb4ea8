"""Lucene99 flat vector files (.vec / .vemf): the restated layout (opensearch_amd/flatfiles.py) written
and read back on CPU — headers, footers and CRC32, per-field entries, and the docsWithField IndexedDISI
of sparse fields (SPARSE, DENSE and ALL blocks, several 65536-doc blocks, jump tables).  Parity
unpinned: no Lucene jar or index fixture exists in the reference or the image, so the layout is
checked against this restatement and its published description only."""
import numpy as np
import pytest

from opensearch_amd import _lib, flatfiles as FF
from oracle import oracle as O

SID = bytes(range(16))


def test_dense_and_sparse_fields_round_trip(tmp_path):
    rng = np.random.default_rng(0)
    max_doc = 300_000
    dense = O.synth(0, max_doc, 8, 1, 3)
    # sparse: an ALL block (block 0), a DENSE block (block 1: 30k docs), a SPARSE block (block 2: 100
    # docs), an empty block (3) and a last SPARSE block (4)
    docs = np.concatenate([np.arange(0, 65536), 65536 + np.sort(rng.choice(65536, 30000, replace=False)),
                           131072 + np.sort(rng.choice(65536, 100, replace=False)),
                           262144 + np.sort(rng.choice(max_doc - 262144, 7, replace=False))]).astype(np.int32)
    sparse = O.synth(0, len(docs), 24, 2, 2)
    bytes_ = O.synth(0, 1000, 40, 3, 4)
    bdocs = np.sort(rng.choice(max_doc, 1000, replace=False)).astype(np.int32)
    vec, vemf = FF.write_segment(str(tmp_path), "_0", SID, max_doc,
                                 [(3, dense, 2, None), (7, sparse, 0, docs), (9, bytes_, 1, bdocs),
                                  (11, np.zeros((0, 4), np.float32), 1, None)], suffix="Lucene99_0")
    FF.check_data_file(vec, SID, "Lucene99_0")
    es = FF.read_meta(vemf, SID, "Lucene99_0")
    assert [(e.number, e.encoding, e.similarity, e.dim, e.size) for e in es] == \
        [(3, 0, 2, 8, max_doc), (7, 0, 0, 24, len(docs)), (9, 1, 1, 40, 1000), (11, 0, 1, 4, 0)]
    raw = open(vec, "rb").read()
    for e, rows in zip(es[:3], [dense, sparse, bytes_]):
        assert e.data_offset % (4 if e.encoding == 0 else 1) == 0
        got = np.frombuffer(raw, rows.dtype, count=rows.size, offset=e.data_offset).reshape(rows.shape)
        assert np.array_equal(got, rows)
    assert FF.ord_to_doc(vec, es[0], max_doc) is None
    assert np.array_equal(FF.ord_to_doc(vec, es[1], max_doc), docs)
    assert es[1].jump_table_entries == 5 and es[1].dense_rank_power == 9
    assert np.array_equal(FF.ord_to_doc(vec, es[2], max_doc), bdocs)
    assert len(FF.ord_to_doc(vec, es[3], max_doc)) == 0 and es[3].docs_with_field_offset == -2


def test_corruption_is_detected(tmp_path):
    vec, vemf = FF.write_segment(str(tmp_path), "_1", SID, 100, [(0, O.synth(0, 100, 4, 1, 3), 2, None)])
    data = bytearray(open(vemf, "rb").read())
    data[40] ^= 1
    open(vemf, "wb").write(bytes(data))
    with pytest.raises(FF.CorruptIndexError, match="checksum"):
        FF.read_meta(vemf, SID)
    with pytest.raises(FF.CorruptIndexError, match="segment id"):
        FF.check_data_file(vec, bytes(16))
    with pytest.raises(FF.CorruptIndexError, match="codec mismatch"):
        FF.read_meta(vec, SID)   # a data file is not a meta file


def test_headers_follow_codec_util(tmp_path):
    vec, vemf = FF.write_segment(str(tmp_path), "_2", SID, 10, [(0, np.ones((10, 4), np.float32), 1, None)], "s")
    raw = open(vemf, "rb").read()
    assert raw[:4] == bytes.fromhex("3fd76c17")                       # BE codec magic
    assert raw[4] == len(FF.META_CODEC) and raw[5:5 + raw[4]] == FF.META_CODEC.encode()
    assert raw[-16:-12] == bytes.fromhex("c02893e8")                  # BE footer magic = ~codec magic


@pytest.mark.skipif(__import__("torch").cuda.is_available(), reason="checks the no-device error path")
def test_stage_file_fails_loudly_without_gpu(tmp_path):
    import ctypes as C
    vec, vemf = FF.write_segment(str(tmp_path), "_3", SID, 10, [(0, np.ones((10, 4), np.float32), 1, None)])
    e = FF.read_meta(vemf, SID)[0]
    h = C.c_void_p()
    rc = _lib.lib().osk_seg_stage_file(0, vec.encode(), e.data_offset, e.size, e.dim, 0, 1, None, 10, C.byref(h))
    assert rc == _lib.OSK_ERR_NO_DEVICE
