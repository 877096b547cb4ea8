/*
 * [L] KnnVectorsReader for one segment, every vector field resident in HBM (osk_seg per field).  Storage stays
 * the stock flat reader; the constructor (= segment open, S/index/engine/InternalEngine.java:584-589) stages each
 * field's rows once with osk_seg_stage, search() runs osk_seg_search (exact top-k, Lucene's scores and tie
 * order), close() (the segment is merged away) drops the reader's reference — views over the segment keep it
 * alive until they are released (osk_seg_retain / osk_seg_release).
 */
package org.opensearch.knn.gpu;

import java.io.IOException;
import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.util.HashMap;
import java.util.Map;

import org.apache.lucene.codecs.KnnVectorsReader;
import org.apache.lucene.codecs.hnsw.FlatVectorsReader;
import org.apache.lucene.index.ByteVectorValues;
import org.apache.lucene.index.FieldInfo;
import org.apache.lucene.index.FloatVectorValues;
import org.apache.lucene.index.KnnVectorValues;
import org.apache.lucene.index.SegmentReadState;
import org.apache.lucene.index.VectorEncoding;
import org.apache.lucene.search.AcceptDocs;
import org.apache.lucene.search.DocIdSetIterator;
import org.apache.lucene.search.KnnCollector;
import org.apache.lucene.util.Bits;
import org.apache.lucene.util.FixedBitSet;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_BYTE;
import static java.lang.foreign.ValueLayout.JAVA_FLOAT;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

public final class GpuFlatVectorsReader extends KnnVectorsReader {
    private final FlatVectorsReader flat;            // Lucene99FlatVectorsReader: integrity, values, RAM
    private final Map<String, MemorySegment> segs = new HashMap<>();   // field → osk_seg*
    private final Map<String, VectorEncoding> encodings = new HashMap<>();
    private final int maxDoc;

    GpuFlatVectorsReader(SegmentReadState state, FlatVectorsReader flat, int device) throws IOException {
        this.flat = flat;
        this.maxDoc = state.segmentInfo.maxDoc();
        boolean ok = false;
        try {
            for (FieldInfo fi : state.fieldInfos) {
                if (fi.hasVectorValues()) stage(fi, device);
            }
            ok = true;
        } finally {
            if (!ok) close();
        }
    }

    private void stage(FieldInfo field, int device) throws IOException {
        boolean bytes = field.getVectorEncoding() == VectorEncoding.BYTE;
        KnnVectorValues values = bytes ? flat.getByteVectorValues(field.name) : flat.getFloatVectorValues(field.name);
        int dim = values.dimension(), n = values.size();
        try (Arena arena = Arena.ofConfined()) {
            // rows: the .vec slice read through the flat reader (osk_seg_stage_file stages it straight from the
            // mmapped file when the slice's offset is known, INTEGRATION.md §5b)
            MemorySegment rows = arena.allocate(bytes ? JAVA_BYTE : JAVA_FLOAT, Math.max(1L, (long) n * dim));
            for (int ord = 0; ord < n; ord++) {
                if (bytes) {
                    MemorySegment.copy(((ByteVectorValues) values).vectorValue(ord), 0, rows, JAVA_BYTE, (long) ord * dim, dim);
                } else {
                    MemorySegment.copy(((FloatVectorValues) values).vectorValue(ord), 0, rows, JAVA_FLOAT, (long) ord * dim * 4, dim);
                }
            }
            MemorySegment ordToDoc = MemorySegment.NULL;   // dense field: doc == ord
            if (n < maxDoc) {                              // sparse: ord → doc from the values' iterator
                ordToDoc = arena.allocate(JAVA_INT, Math.max(1, n));
                KnnVectorValues.DocIndexIterator it = values.iterator();
                for (int ord = 0; it.nextDoc() != DocIdSetIterator.NO_MORE_DOCS; ord++) {
                    ordToDoc.setAtIndex(JAVA_INT, ord, it.docID());
                }
            }
            MemorySegment out = arena.allocate(ADDRESS);
            OsKnn.check((int) OsKnn.SEG_STAGE.invokeExact(device, rows, (long) n, dim,
                bytes ? OsKnn.OSK_BYTE : OsKnn.OSK_FLOAT32, field.getVectorSimilarityFunction().ordinal(), ordToDoc,
                maxDoc, out));
            segs.put(field.name, out.get(ADDRESS, 0));
            encodings.put(field.name, field.getVectorEncoding());
        } catch (Throwable t) {
            throw OsKnn.wrap(t);
        }
    }

    /** The field's osk_seg* (GpuShardViews groups a shard's segments into one osk_view). */
    MemorySegment segment(String field) {
        MemorySegment s = segs.get(field);
        if (s == null) throw new IllegalArgumentException("field [" + field + "] has no vectors in this segment");
        return s;
    }

    int maxDoc() {
        return maxDoc;
    }

    /** [L] KnnVectorsReader.search(String, float[], KnnCollector, AcceptDocs) — the 4-arg Lucene 10.3 signature
     *  (S/index/engine/TranslogLeafReader.java:379-386). */
    @Override
    public void search(String field, float[] target, KnnCollector collector, AcceptDocs acceptDocs) throws IOException {
        if (encodings.get(field) != VectorEncoding.FLOAT32) {
            throw new IllegalArgumentException("field [" + field + "] is not a float vector field");
        }
        search(field, MemorySegment.ofArray(target), collector, acceptDocs);
    }

    /** [L] KnnVectorsReader.search(String, byte[], KnnCollector, AcceptDocs): exact int32 scores on the device. */
    @Override
    public void search(String field, byte[] target, KnnCollector collector, AcceptDocs acceptDocs) throws IOException {
        if (encodings.get(field) != VectorEncoding.BYTE) {
            throw new IllegalArgumentException("field [" + field + "] is not a byte vector field");
        }
        search(field, MemorySegment.ofArray(target), collector, acceptDocs);
    }

    private void search(String field, MemorySegment target, KnnCollector collector, AcceptDocs acceptDocs) throws IOException {
        int k = Math.min(collector.k(), 10000);   // OSK_MAX_K = index.max_result_window
        float[] scores = new float[k];
        int[] docs = new int[k];
        int[] count = new int[1];
        long[] visited = new long[1];
        long[] bits = acceptBits(acceptDocs, maxDoc);
        try {
            OsKnn.check((int) OsKnn.SEG_SEARCH.invokeExact(segment(field), target, 1, k,
                bits == null ? MemorySegment.NULL : MemorySegment.ofArray(bits),
                MemorySegment.ofArray(scores), MemorySegment.ofArray(docs),
                MemorySegment.ofArray(count), MemorySegment.ofArray(visited)));
        } catch (Throwable t) {
            throw OsKnn.wrap(t);
        }
        collector.incVisitedCount((int) Math.min(visited[0], Integer.MAX_VALUE));
        for (int i = 0; i < count[0]; i++) collector.collect(docs[i], scores[i]);   // best first
    }

    /** AcceptDocs (liveDocs ∩ filter) → ⌈maxDoc/64⌉ LSB-first words, the C-ABI's bitset.  A FixedBitSet (what
     *  BitsetFilterCache, S/index/cache/bitset/BitsetFilterCache.java:127-160, and liveDocs hold) passes its
     *  words through; anything else is materialised from its iterator.  null = every doc accepted. */
    static long[] acceptBits(AcceptDocs acceptDocs, int maxDoc) throws IOException {
        if (acceptDocs == null) return null;
        Bits b = acceptDocs.bits();
        if (b == null) return null;
        if (b instanceof FixedBitSet fbs) return fbs.getBits();
        FixedBitSet copy = new FixedBitSet(maxDoc);
        DocIdSetIterator it = acceptDocs.iterator();
        for (int d = it.nextDoc(); d != DocIdSetIterator.NO_MORE_DOCS; d = it.nextDoc()) copy.set(d);
        return copy.getBits();
    }

    /** HBM bytes the segment's fields hold (osk_seg_footprint): the rows and the prefilter copies. */
    public long hbmBytes() throws IOException {
        long total = 0;
        try (Arena a = Arena.ofConfined()) {
            MemorySegment b = a.allocate(JAVA_LONG);
            for (MemorySegment s : segs.values()) {
                OsKnn.check((int) OsKnn.SEG_FOOTPRINT.invokeExact(s, b));
                total += b.get(JAVA_LONG, 0);
            }
        } catch (Throwable t) {
            throw OsKnn.wrap(t);
        }
        return total;
    }

    @Override
    public void checkIntegrity() throws IOException {
        flat.checkIntegrity();
    }

    @Override
    public FloatVectorValues getFloatVectorValues(String field) throws IOException {
        return flat.getFloatVectorValues(field);
    }

    @Override
    public ByteVectorValues getByteVectorValues(String field) throws IOException {
        return flat.getByteVectorValues(field);
    }

    @Override
    public long ramBytesUsed() {
        return flat.ramBytesUsed();
    }

    @Override
    public void close() throws IOException {
        Throwable first = null;
        for (MemorySegment s : segs.values()) {
            try {
                OsKnn.check((int) OsKnn.SEG_RELEASE.invokeExact(s));
            } catch (Throwable t) {
                if (first == null) first = t;
            }
        }
        segs.clear();
        flat.close();
        if (first != null) throw OsKnn.wrap(first);
    }
}
