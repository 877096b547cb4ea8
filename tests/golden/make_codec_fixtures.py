"""Extract the Lucene-written codec files that pin flatfiles.py's CodecUtil framing (run here, where
/root/reference exists; the extracted bytes are committed, the GPU box never reads the reference).

Source: /root/reference/server/src/test/resources/indices/bwc/unsupported-2.4.5.zip — an index that
OpenSearch's own backwards-compatibility tests hold (Lucene 5.5 codecs).  Lucene 10 writes the same
CodecUtil index header (magic 0x3fd76c17, codec name, version, 16-byte segment id, suffix) and footer
(magic 0xc02893e8, algorithm 0, CRC32) around every file, so these bytes pin the framing that
Lucene99FlatVectorsFormat's .vec/.vemf use.  The .vemf-specific fields stay unpinned: no vector
segment exists anywhere in the reference.
"""
import zipfile
from pathlib import Path

ZIP = "/root/reference/server/src/test/resources/indices/bwc/unsupported-2.4.5.zip"
BASE = "data/bwc_index_2.4.5/nodes/0/indices/index-2.4.5/0/index/"
FILES = ["_a1.si", "_a1.cfe", "_a0.fnm", "segments_4t"]

if __name__ == "__main__":
    out = Path(__file__).resolve().parent / "lucene_codec"
    out.mkdir(exist_ok=True)
    z = zipfile.ZipFile(ZIP)
    for f in FILES:
        (out / f).write_bytes(z.read(BASE + f))
        print("wrote", out / f)
