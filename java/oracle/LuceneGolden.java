// Re-derives tests/golden/knn_golden.npz with the real lucene-core 10.3.0 (SURVEY.md §8(c)): where a JDK
// and the jar exist, this turns the oracle's "parity unpinned" scoring into "pinned".  Not run in this
// image (no JDK).  Input: the raw little-endian case files that golden_io.py export writes; output, per
// case, <case>.lucene.bin = for every query: int32 count, then k × (float32 score, int32 doc).
// exactSearch is restated with Lucene's own pieces: VectorSimilarityFunction.compare (VectorUtil, Panama
// when run with --add-modules jdk.incubator.vector) and HitQueue (score desc, ties → lower doc).
import java.io.*;
import java.nio.*;
import java.nio.file.*;
import org.apache.lucene.index.VectorSimilarityFunction;
import org.apache.lucene.search.HitQueue;
import org.apache.lucene.search.ScoreDoc;

public final class LuceneGolden {
    static ByteBuffer read(Path p) throws IOException {
        return ByteBuffer.wrap(Files.readAllBytes(p)).order(ByteOrder.LITTLE_ENDIAN);
    }

    public static void main(String[] args) throws IOException {
        Path dir = Paths.get(args[0]);
        for (String line : Files.readAllLines(dir.resolve("manifest.txt"))) {
            // name enc sim dim n nq k   (enc: f32|i8; sim: VectorSimilarityFunction ordinal)
            String[] f = line.trim().split(" ");
            String name = f[0]; boolean f32 = f[1].equals("f32");
            VectorSimilarityFunction sim = VectorSimilarityFunction.values()[Integer.parseInt(f[2])];
            int dim = Integer.parseInt(f[3]), n = Integer.parseInt(f[4]), nq = Integer.parseInt(f[5]), k = Integer.parseInt(f[6]);
            ByteBuffer rows = read(dir.resolve(name + ".rows")), qs = read(dir.resolve(name + ".queries"));
            ByteBuffer o2d = read(dir.resolve(name + ".ord_to_doc")), acc = read(dir.resolve(name + ".accept"));
            ByteBuffer out = ByteBuffer.allocate(nq * (4 + 8 * k)).order(ByteOrder.LITTLE_ENDIAN);
            for (int q = 0; q < nq; q++) {
                HitQueue hq = new HitQueue(k, true);                  // sentinels: score −inf, doc MAX
                for (int ord = 0; ord < n; ord++) {
                    int doc = o2d.getInt(4 * ord);
                    if ((acc.getLong(8 * (doc >>> 6)) >>> (doc & 63) & 1L) == 0) continue;
                    float s;
                    if (f32) {
                        float[] a = new float[dim], b = new float[dim];
                        for (int i = 0; i < dim; i++) { a[i] = qs.getFloat(4 * (q * dim + i)); b[i] = rows.getFloat(4 * (ord * dim + i)); }
                        s = sim.compare(a, b);
                    } else {
                        byte[] a = new byte[dim], b = new byte[dim];
                        for (int i = 0; i < dim; i++) { a[i] = qs.get(q * dim + i); b[i] = rows.get(ord * dim + i); }
                        s = sim.compare(a, b);
                    }
                    ScoreDoc top = hq.top();
                    if (s > top.score) { top.score = s; top.doc = doc; hq.updateTop(); }   // strict >: ties keep the lower doc
                }
                // pop() yields the worst first (sentinels before hits): fill from the back, best lands at 0
                int cnt = 0; ScoreDoc[] res = new ScoreDoc[k];
                for (int i = k - 1; i >= 0; i--) { res[i] = hq.pop(); if (res[i].score != Float.NEGATIVE_INFINITY) cnt++; }
                out.putInt(cnt);
                for (int i = 0; i < k; i++) {
                    out.putFloat(i < cnt ? res[i].score : Float.NEGATIVE_INFINITY);
                    out.putInt(i < cnt ? res[i].doc : Integer.MAX_VALUE);
                }
            }
            Files.write(dir.resolve(name + ".lucene.bin"), out.array());
        }
    }
}
