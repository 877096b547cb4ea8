"""Bridge between tests/golden/knn_golden.npz and the Java harness (LuceneGolden.java).

    python java/oracle/golden_io.py export /tmp/lg      # raw case files + manifest.txt
    bash   java/oracle/run.sh /tmp/lg                   # real Lucene writes <case>.lucene.bin
    python java/oracle/golden_io.py compare /tmp/lg     # Lucene vs the oracle's Panama-512 order

`compare` checks, per case (dense and sparse+filtered), that Lucene's docs equal the oracle's Panama-512
(o2) docs except swaps between near-ties and its scores are within 1e-5 relative (bit-identical for byte
vectors), then writes knn_golden_lucene.npz — the pinned fixture the tests would load.
"""
import sys
from pathlib import Path

import numpy as np

GOLD = Path(__file__).resolve().parents[2] / "tests" / "golden" / "knn_golden.npz"
K = 7


def cases(g):
    for key in g.files:
        if key.endswith("_rows"):
            yield key[:-5]


def export(out: Path):
    g = np.load(GOLD)
    out.mkdir(parents=True, exist_ok=True)
    lines = []
    for c in cases(g):
        enc, sim, dim = c.split("_")
        rows, qs, o2d = g[c + "_rows"], g[c + "_queries"], g[c + "_ord_to_doc"]
        for variant, od, acc in (("dense", np.arange(len(rows), dtype=np.int32), None),
                                 ("sparse_filtered", o2d, g[c + "_accept"])):
            name = f"{c}_{variant}"
            max_doc = int(od.max()) + 1
            words = acc if acc is not None else np.full((max_doc + 63) // 64, ~np.uint64(0), np.uint64)
            rows.tofile(out / f"{name}.rows")
            qs.tofile(out / f"{name}.queries")
            od.astype("<i4").tofile(out / f"{name}.ord_to_doc")
            words.astype("<u8").tofile(out / f"{name}.accept")
            lines.append(f"{name} {enc} {sim} {dim} {len(rows)} {len(qs)} {K}")
    (out / "manifest.txt").write_text("\n".join(lines) + "\n")


def compare(d: Path):
    g = np.load(GOLD)
    pinned = {}
    for line in (d / "manifest.txt").read_text().split("\n"):
        if not line:
            continue
        name, enc, sim, dim, n, nq, k = line.split()
        nq, k = int(nq), int(k)
        raw = np.fromfile(d / f"{name}.lucene.bin", np.uint8).reshape(nq, 4 + 8 * k)
        cnt = raw[:, :4].copy().view("<i4")[:, 0]
        pairs = raw[:, 4:].copy().view("<f4").reshape(nq, k, 2)
        sc = pairs[:, :, 0].copy()
        dc = pairs[:, :, 1].copy().view("<i4")
        if name.endswith("_sparse_filtered"):
            case, variant = name[: -len("_sparse_filtered")], "sparse_filtered"
        else:
            case, variant = name[: -len("_dense")], "dense"
        order = "o2" if enc == "f32" else "o0"
        want_s, want_d = g[f"{case}_{order}_{variant}_scores"], g[f"{case}_{order}_{variant}_docs"]
        for q in range(nq):
            c = int(cnt[q])
            assert c == int(g[f"{case}_{order}_{variant}_count"][q]), (name, q)
            if enc == "i8":
                assert np.array_equal(sc[q, :c].view(np.uint32), want_s[q, :c].view(np.uint32)), (name, q)
                assert np.array_equal(dc[q, :c], want_d[q, :c]), (name, q)
            else:
                assert np.allclose(sc[q, :c], want_s[q, :c], rtol=1e-5, atol=0), (name, q)
                assert sorted(dc[q, :c]) == sorted(want_d[q, :c]) or np.allclose(np.sort(sc[q, :c]),
                                                                                    np.sort(want_s[q, :c]), rtol=1e-6)
        pinned[f"{name}_scores"], pinned[f"{name}_docs"], pinned[f"{name}_count"] = sc, dc, cnt
    np.savez_compressed(GOLD.with_name("knn_golden_lucene.npz"), **pinned)
    print("pinned", len(pinned) // 3, "cases against lucene-core")


if __name__ == "__main__":
    {"export": export, "compare": compare}[sys.argv[1]](Path(sys.argv[2]))
