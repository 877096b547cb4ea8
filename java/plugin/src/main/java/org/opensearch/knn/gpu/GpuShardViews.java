/*
 * One osk_view per (point-in-time reader, field): the field's osk_seg of every leaf of the shard, with each
 * leaf's docBase, so a shard's whole top-k is ONE device call (osk_view_search) instead of one per leaf.  The view
 * retains its segments (a segment merged away under a live searcher stays valid, NRT refresh churn,
 * S/index/engine/InternalEngine.java:584-589) and is released by the reader's closed listener.
 */
package org.opensearch.knn.gpu;

import java.io.IOException;
import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.util.List;
import java.util.Map;
import java.util.concurrent.ConcurrentHashMap;

import org.apache.lucene.codecs.KnnVectorsReader;
import org.apache.lucene.codecs.perfield.PerFieldKnnVectorsFormat;
import org.apache.lucene.index.FilterLeafReader;
import org.apache.lucene.index.IndexReader;
import org.apache.lucene.index.LeafReader;
import org.apache.lucene.index.LeafReaderContext;
import org.apache.lucene.index.SegmentReader;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_INT;

final class GpuShardViews {
    private GpuShardViews() {}

    private record Key(Object readerKey, String field) {}

    private static final Map<Key, MemorySegment> VIEWS = new ConcurrentHashMap<>();

    /** The leaf's GPU reader for the field (the segment's per-field vectors reader), or null when the leaf's
     *  field is not on GpuFlatVectorsFormat (e.g. a segment written before the index turned the plugin on). */
    static GpuFlatVectorsReader readerOf(LeafReaderContext ctx, String field) {
        LeafReader r = FilterLeafReader.unwrap(ctx.reader());
        if (!(r instanceof SegmentReader sr)) return null;
        KnnVectorsReader vr = sr.getVectorReader();
        if (vr instanceof PerFieldKnnVectorsFormat.FieldsReader pf) vr = pf.getFieldReader(field);
        return vr instanceof GpuFlatVectorsReader g ? g : null;
    }

    /** A view handed to one search: {@code owned} when the reader has no cache helper (no closed listener to
     *  release a cached view), so the caller releases it after its call through {@link #done}. */
    record Lease(MemorySegment view, boolean owned) {}

    /** The shard's view over the field (created on first use, cached until the reader closes; a reader without a
     *  cache helper gets a view for this one call, never cached: nothing would release it); null when some leaf
     *  with the field is not GPU-resident (the caller then takes Lucene's per-leaf route). */
    static Lease forReader(IndexReader reader, String field) throws IOException {
        IndexReader.CacheHelper ch = reader.getReaderCacheHelper();
        if (ch == null) {
            MemorySegment v = create(reader.leaves(), field);
            return v == null ? null : new Lease(v, true);
        }
        Key key = new Key(ch.getKey(), field);
        MemorySegment v = VIEWS.get(key);
        if (v != null) return new Lease(v, false);
        synchronized (GpuShardViews.class) {
            v = VIEWS.get(key);
            if (v != null) return new Lease(v, false);
            v = create(reader.leaves(), field);
            if (v == null) return null;
            VIEWS.put(key, v);
            ch.addClosedListener(k -> release(new Key(k, field)));
            return new Lease(v, false);
        }
    }

    /** After the call: releases a view that was created for it alone. */
    static void done(Lease lease) {
        if (lease == null || !lease.owned()) return;
        try {
            OsKnn.check((int) OsKnn.VIEW_RELEASE.invokeExact(lease.view()));
        } catch (Throwable t) {
            throw OsKnn.wrap(t);
        }
    }

    private static MemorySegment create(List<LeafReaderContext> leaves, String field) throws IOException {
        try (Arena arena = Arena.ofConfined()) {
            int n = leaves.size();
            MemorySegment segs = arena.allocate(ADDRESS, Math.max(1, n));
            MemorySegment seg_shard = arena.allocate(JAVA_INT, Math.max(1, n));
            MemorySegment seg_base = arena.allocate(JAVA_INT, Math.max(1, n));
            int used = 0;
            for (LeafReaderContext ctx : leaves) {
                if (ctx.reader().getFieldInfos().fieldInfo(field) == null) continue;   // leaf without the field
                GpuFlatVectorsReader g = readerOf(ctx, field);
                if (g == null) return null;
                segs.setAtIndex(ADDRESS, used, g.segment(field));
                seg_shard.setAtIndex(JAVA_INT, used, 0);
                seg_base.setAtIndex(JAVA_INT, used, ctx.docBase);
                used++;
            }
            if (used == 0) return null;
            MemorySegment shardIndex = arena.allocateFrom(JAVA_INT, 0);
            MemorySegment out = arena.allocate(ADDRESS);
            OsKnn.check((int) OsKnn.VIEW_CREATE.invokeExact(segs, used, seg_shard, seg_base, 1, shardIndex, out));
            return out.get(ADDRESS, 0);
        } catch (Throwable t) {
            throw OsKnn.wrap(t);
        }
    }

    private static void release(Key key) {
        MemorySegment v = VIEWS.remove(key);
        if (v == null) return;
        try {
            OsKnn.check((int) OsKnn.VIEW_RELEASE.invokeExact(v));
        } catch (Throwable ignored) {
            // the view's segments stay referenced until the library is unloaded; nothing else to do on close
        }
    }
}
