/*
 * The rewritten k-NN query: a fixed set of (shard-level doc, score) hits, the role of Lucene's package-private
 * DocAndScoreQuery.  Its Weight yields, per leaf, the hits whose doc falls in [docBase, docBase + maxDoc), with
 * their scores (times the query boost).
 */
package org.opensearch.knn.gpu;

import java.io.IOException;
import java.util.Arrays;
import java.util.Objects;

import org.apache.lucene.index.LeafReaderContext;
import org.apache.lucene.search.DocIdSetIterator;
import org.apache.lucene.search.Explanation;
import org.apache.lucene.search.IndexSearcher;
import org.apache.lucene.search.Query;
import org.apache.lucene.search.QueryVisitor;
import org.apache.lucene.search.ScoreDoc;
import org.apache.lucene.search.ScoreMode;
import org.apache.lucene.search.Scorer;
import org.apache.lucene.search.ScorerSupplier;
import org.apache.lucene.search.Weight;

final class GpuDocAndScoreQuery extends Query {
    private final Object readerId;
    private final int[] docs;       // ascending
    private final float[] scores;

    GpuDocAndScoreQuery(Object readerId, ScoreDoc[] hits) {
        this.readerId = readerId;
        ScoreDoc[] sorted = hits.clone();
        Arrays.sort(sorted, (a, b) -> Integer.compare(a.doc, b.doc));
        docs = new int[sorted.length];
        scores = new float[sorted.length];
        for (int i = 0; i < sorted.length; i++) {
            docs[i] = sorted[i].doc;
            scores[i] = sorted[i].score;
        }
    }

    @Override
    public Weight createWeight(IndexSearcher searcher, ScoreMode scoreMode, float boost) {
        return new Weight(this) {
            @Override
            public ScorerSupplier scorerSupplier(LeafReaderContext ctx) {
                int lo = lowerBound(ctx.docBase), hi = lowerBound(ctx.docBase + ctx.reader().maxDoc());
                if (lo == hi) return null;
                final Scorer scorer = new Scorer() {
                    int i = lo - 1;
                    final DocIdSetIterator it = new DocIdSetIterator() {
                        @Override public int docID() {
                            return i < lo ? -1 : i >= hi ? NO_MORE_DOCS : docs[i] - ctx.docBase;
                        }
                        @Override public int nextDoc() {
                            i++;
                            return docID();
                        }
                        @Override public int advance(int target) {
                            int t = lowerBound(ctx.docBase + target);
                            i = Math.max(i + 1, Math.min(t, hi));
                            return docID();
                        }
                        @Override public long cost() {
                            return hi - lo;
                        }
                    };
                    @Override public int docID() { return it.docID(); }
                    @Override public DocIdSetIterator iterator() { return it; }
                    @Override public float getMaxScore(int upTo) {
                        float m = 0f;
                        for (int j = lo; j < hi; j++) m = Math.max(m, scores[j]);
                        return m * boost;
                    }
                    @Override public float score() { return scores[i] * boost; }
                };
                return new ScorerSupplier() {
                    @Override public Scorer get(long leadCost) { return scorer; }
                    @Override public long cost() { return hi - lo; }
                };
            }

            @Override
            public Explanation explain(LeafReaderContext ctx, int doc) {
                int j = Arrays.binarySearch(docs, ctx.docBase + doc);
                return j < 0 ? Explanation.noMatch("not a GPU k-NN hit")
                             : Explanation.match(scores[j] * boost, "GPU exact k-NN score");
            }

            @Override
            public boolean isCacheable(LeafReaderContext ctx) {
                return true;
            }
        };
    }

    private int lowerBound(int doc) {
        int j = Arrays.binarySearch(docs, doc);
        return j >= 0 ? j : -j - 1;
    }

    @Override
    public void visit(QueryVisitor visitor) {
        visitor.visitLeaf(this);
    }

    @Override
    public String toString(String field) {
        return "GpuDocAndScoreQuery[" + docs.length + " hits]";
    }

    @Override
    public boolean equals(Object o) {
        return sameClassAs(o) && readerId == ((GpuDocAndScoreQuery) o).readerId
            && Arrays.equals(docs, ((GpuDocAndScoreQuery) o).docs) && Arrays.equals(scores, ((GpuDocAndScoreQuery) o).scores);
    }

    @Override
    public int hashCode() {
        return Objects.hash(classHash(), System.identityHashCode(readerId), Arrays.hashCode(docs), Arrays.hashCode(scores));
    }
}
