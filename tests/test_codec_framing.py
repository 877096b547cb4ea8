"""flatfiles.py's CodecUtil framing pinned against Lucene-written bytes.

The files in tests/golden/lucene_codec/ were written by Lucene (extracted by
tests/golden/make_codec_fixtures.py from the reference's own backwards-compatibility test index
server/src/test/resources/indices/bwc/unsupported-2.4.5.zip).  Every Lucene file starts with the
CodecUtil index header (magic, codec name, version, 16-byte segment id, suffix) and ends with the
footer (footer magic, algorithm 0, CRC32 of everything before the checksum) — the framing of the
.vec / .vemf files `osk_seg_stage_file` reads (S/index/store/FsDirectoryFactory.java:98-110 maps them).
The .vemf field entries themselves stay unpinned: no vector segment exists in the reference.
"""
import struct
from pathlib import Path

import pytest

from opensearch_amd import flatfiles as F

GOLD = Path(__file__).resolve().parent / "golden" / "lucene_codec"
SEG_A1 = bytes.fromhex("328113086f23de19c93123a1ed5f4f16")
SEG_A0 = bytes.fromhex("328113086f23de19c93123a1ed5f4f15")
SEG_COMMIT = bytes.fromhex("328113086f23de19c93123a1ed5f4f18")
# file, codec name, version, segment id, suffix — as Lucene wrote them
CASES = [("_a1.si", "Lucene50SegmentInfo", 1, SEG_A1, ""),
         ("_a1.cfe", "Lucene50CompoundEntries", 0, SEG_A1, ""),
         ("_a0.fnm", "Lucene50FieldInfos", 1, SEG_A0, ""),
         ("segments_4t", "segments", 6, SEG_COMMIT, "4t")]


def _header_len(codec, suffix):
    return 4 + 1 + len(codec) + 4 + 16 + 1 + len(suffix)


@pytest.mark.parametrize("name,codec,version,seg_id,suffix", CASES)
def test_lucene_written_files_pass_the_header_and_footer_checks(name, codec, version, seg_id, suffix):
    data = (GOLD / name).read_bytes()
    i = F._In(data)
    assert F._check_header(i, codec, seg_id, suffix, 0, 10) == version
    assert i.p == _header_len(codec, suffix)
    F._check_footer(data)
    magic, algo, _ = struct.unpack(">IIQ", data[-16:])
    assert magic == F.FOOTER_MAGIC == 0xC02893E8 and algo == 0


@pytest.mark.parametrize("name,codec,version,seg_id,suffix", CASES)
def test_writer_reproduces_lucene_framing_byte_for_byte(name, codec, version, seg_id, suffix):
    data = (GOLD / name).read_bytes()
    body = data[_header_len(codec, suffix):-16]
    o = F._Out()
    F._write_header(o, codec, seg_id, suffix, version)
    o.raw(body)
    F._write_footer(o)
    assert bytes(o.b) == data


def test_corruptions_are_detected():
    data = (GOLD / "_a1.si").read_bytes()
    with pytest.raises(F.CorruptIndexError, match="checksum"):
        F._check_footer(data[:100] + bytes([data[100] ^ 1]) + data[101:])
    with pytest.raises(F.CorruptIndexError, match="segment id"):
        F._check_header(F._In(data), "Lucene50SegmentInfo", SEG_A0, "", 0, 10)
    with pytest.raises(F.CorruptIndexError, match="codec mismatch"):
        F._check_header(F._In(data), "Lucene99FlatVectorsFormatMeta", SEG_A1, "", 0, 10)
    with pytest.raises(F.CorruptIndexError, match="version"):
        F._check_header(F._In(data), "Lucene50SegmentInfo", SEG_A1, "", 2, 3)
    with pytest.raises(F.CorruptIndexError, match="footer"):
        F._check_footer(data[:-16] + bytes(16))
