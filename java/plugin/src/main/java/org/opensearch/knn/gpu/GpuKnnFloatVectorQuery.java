/*
 * KnnFloatVectorQuery whose rewrite is ONE osk_view_search over every leaf of the shard (GpuKnnSupport); a
 * shard with a leaf that is not GPU-resident falls back to Lucene's per-leaf route, whose exactSearch branch
 * (`cost ≤ k` leaves) is also sent to the device here.  Python mirror: opensearch_amd/lucene.py
 * GpuKnnFloatVectorQuery, tested against the oracle by tests/test_gpu_shard_query.py.
 */
package org.opensearch.knn.gpu;

import java.io.IOException;

import org.apache.lucene.index.LeafReaderContext;
import org.apache.lucene.index.QueryTimeout;
import org.apache.lucene.search.AcceptDocs;
import org.apache.lucene.search.DocIdSetIterator;
import org.apache.lucene.search.IndexSearcher;
import org.apache.lucene.search.KnnFloatVectorQuery;
import org.apache.lucene.search.Query;
import org.apache.lucene.search.ScoreDoc;
import org.apache.lucene.search.TopDocs;
import org.apache.lucene.search.TopKnnCollector;
import org.apache.lucene.util.FixedBitSet;

public final class GpuKnnFloatVectorQuery extends KnnFloatVectorQuery {
    private final String field;
    private final float[] target;
    private final int k;
    private final Query filter;

    public GpuKnnFloatVectorQuery(String field, float[] target, int k, Query filter) {
        super(field, target, k, filter);
        this.field = field;
        this.target = target;
        this.k = k;
        this.filter = filter;
    }

    @Override
    public Query rewrite(IndexSearcher searcher) throws IOException {
        Query q = GpuKnnSupport.rewrite(searcher, field, target, k, filter);
        return q != null ? q : super.rewrite(searcher);
    }

    /** [L] AbstractKnnVectorQuery.exactSearch — the per-leaf route's `cost ≤ k` branch, on the device. */
    @Override
    protected TopDocs exactSearch(LeafReaderContext ctx, DocIdSetIterator acceptIterator, QueryTimeout timeout)
            throws IOException {
        GpuFlatVectorsReader r = GpuShardViews.readerOf(ctx, field);
        if (r == null) return super.exactSearch(ctx, acceptIterator, timeout);
        FixedBitSet bits = new FixedBitSet(ctx.reader().maxDoc());
        bits.or(acceptIterator);
        TopKnnCollector c = new TopKnnCollector(k, Integer.MAX_VALUE);
        r.search(field, target, c, AcceptDocs.fromLiveDocs(bits, ctx.reader().maxDoc()));
        TopDocs td = c.topDocs();
        for (ScoreDoc sd : td.scoreDocs) sd.doc += ctx.docBase;
        return td;
    }
}
