/*
 * The shared part of the plugin's k-NN queries' rewrite: ONE osk_view_search over every leaf of the shard
 * (its cached osk_view, GpuShardViews), each leaf's AcceptDocs = liveDocs ∩ filter pushed down as a bitset —
 * no per-leaf tasks and no CPU exactSearch branch for `cost ≤ k` leaves (Lucene's own query scores those on the
 * CPU, INTEGRATION.md §2).  Called once per shard by ContextIndexSearcher.rewrite
 * (S/search/internal/ContextIndexSearcher.java:203-218).
 */
package org.opensearch.knn.gpu;

import java.io.IOException;
import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.util.List;

import org.apache.lucene.index.IndexReader;
import org.apache.lucene.index.LeafReaderContext;
import org.apache.lucene.search.BooleanClause;
import org.apache.lucene.search.BooleanQuery;
import org.apache.lucene.search.DocIdSetIterator;
import org.apache.lucene.search.IndexSearcher;
import org.apache.lucene.search.MatchNoDocsQuery;
import org.apache.lucene.search.Query;
import org.apache.lucene.search.ScoreDoc;
import org.apache.lucene.search.ScoreMode;
import org.apache.lucene.search.Scorer;
import org.apache.lucene.search.Weight;
import org.apache.lucene.util.Bits;
import org.apache.lucene.util.FixedBitSet;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_BYTE;
import static java.lang.foreign.ValueLayout.JAVA_FLOAT;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

final class GpuKnnSupport {
    private GpuKnnSupport() {}

    /** The shard's rewritten query, or null when some leaf is not GPU-resident or k is above the library's
     *  OSK_MAX_K (take Lucene's route). */
    static Query rewrite(IndexSearcher searcher, String field, Object target, int k, Query filter) throws IOException {
        if (k < 1 || k > KnnQueryBuilder.MAX_K) return null;   // (osk_view_search refuses it: Lucene's per-leaf route)
        IndexReader reader = searcher.getIndexReader();
        GpuShardViews.Lease lease = GpuShardViews.forReader(reader, field);
        if (lease == null) return null;
        try {
            return search(searcher, reader, lease.view(), field, target, k, filter);
        } finally {
            GpuShardViews.done(lease);
        }
    }

    private static Query search(IndexSearcher searcher, IndexReader reader, MemorySegment view, String field,
                                Object target, int k, Query filter) throws IOException {
        List<LeafReaderContext> leaves = reader.leaves();
        Weight filterWeight = filter == null ? null : searcher.createWeight(searcher.rewrite(
            new BooleanQuery.Builder().add(filter, BooleanClause.Occur.FILTER).build()), ScoreMode.COMPLETE_NO_SCORES, 1f);
        try (Arena arena = Arena.ofConfined()) {
            MemorySegment accept = MemorySegment.NULL;
            boolean deletions = leaves.stream().anyMatch(c -> c.reader().getLiveDocs() != null);
            if (filterWeight != null || deletions) {
                int used = 0;
                accept = arena.allocate(ADDRESS, Math.max(1, leaves.size()));
                for (LeafReaderContext ctx : leaves) {   // the view's segments: the leaves with the field, in order
                    if (ctx.reader().getFieldInfos().fieldInfo(field) == null) continue;
                    FixedBitSet bits = acceptBits(ctx, filterWeight);
                    accept.setAtIndex(ADDRESS, used++, bits == null ? MemorySegment.NULL
                        : arena.allocateFrom(JAVA_LONG, bits.getBits()));
                }
            }
            MemorySegment q = target instanceof float[] f ? arena.allocateFrom(JAVA_FLOAT, f)
                                                          : arena.allocateFrom(JAVA_BYTE, (byte[]) target);
            MemorySegment sc = arena.allocate(JAVA_FLOAT, k), dc = arena.allocate(JAVA_INT, k),
                sh = arena.allocate(JAVA_INT, k), cnt = arena.allocate(JAVA_INT), tot = arena.allocate(JAVA_LONG),
                mx = arena.allocate(JAVA_FLOAT);
            OsKnn.check((int) OsKnn.VIEW_SEARCH.invokeExact(view, q, 1, k, 0, k, accept, sc, dc, sh, cnt, tot, mx));
            int n = cnt.get(JAVA_INT, 0);
            if (n == 0) return new MatchNoDocsQuery();
            ScoreDoc[] hits = new ScoreDoc[n];
            for (int i = 0; i < n; i++) hits[i] = new ScoreDoc(dc.getAtIndex(JAVA_INT, i), sc.getAtIndex(JAVA_FLOAT, i));
            return new GpuDocAndScoreQuery(reader.getContext().id(), hits);
        } catch (Throwable t) {
            throw OsKnn.wrap(t);
        }
    }

    /** The leaf's liveDocs ∩ filter as a bitset; null = every doc of the leaf accepted. */
    static FixedBitSet acceptBits(LeafReaderContext ctx, Weight filterWeight) throws IOException {
        Bits live = ctx.reader().getLiveDocs();
        if (filterWeight == null && live == null) return null;
        int maxDoc = ctx.reader().maxDoc();
        FixedBitSet bits = new FixedBitSet(maxDoc);
        if (filterWeight == null) {
            bits.set(0, maxDoc);
        } else {
            Scorer s = filterWeight.scorer(ctx);
            if (s != null) bits.or(s.iterator());
        }
        if (live != null) {
            for (int d = bits.nextSetBit(0); d != DocIdSetIterator.NO_MORE_DOCS;
                 d = d + 1 < maxDoc ? bits.nextSetBit(d + 1) : DocIdSetIterator.NO_MORE_DOCS) {
                if (!live.get(d)) bits.clear(d);
            }
        }
        return bits;
    }
}
