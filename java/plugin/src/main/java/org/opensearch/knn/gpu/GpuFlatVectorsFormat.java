/*
 * [L] KnnVectorsFormat whose reader answers KnnVectorsReader.search on the GPU (libosknn).  Storage is the
 * stock Lucene99FlatVectorsFormat (.vec / .vemf): the writer IS the flat writer, so indices written with this
 * format stay readable by a node without the plugin (the flat format reads them), and the reader wraps the
 * flat reader for everything but search().  Registered for Lucene's SPI in
 * META-INF/services/org.apache.lucene.codecs.KnnVectorsFormat, which OpenSearch reloads for plugins
 * (S/plugins/PluginsService.java:828-836); the codec (GpuKnnCodec) hands it to knn_vector fields.
 */
package org.opensearch.knn.gpu;

import java.io.IOException;

import org.apache.lucene.codecs.KnnVectorsFormat;
import org.apache.lucene.codecs.KnnVectorsReader;
import org.apache.lucene.codecs.KnnVectorsWriter;
import org.apache.lucene.codecs.hnsw.FlatVectorScorerUtil;
import org.apache.lucene.codecs.hnsw.FlatVectorsFormat;
import org.apache.lucene.codecs.lucene99.Lucene99FlatVectorsFormat;
import org.apache.lucene.index.SegmentReadState;
import org.apache.lucene.index.SegmentWriteState;

public final class GpuFlatVectorsFormat extends KnnVectorsFormat {
    public static final String NAME = "GpuFlatVectorsFormat";
    /** The GPU the node's shards are staged on (one process per GPU), -Dosknn.device. */
    static final int DEVICE = Integer.getInteger("osknn.device", 0);
    static final int MAX_DIMS = 4096;   // OSK_MAX_DIM

    private final FlatVectorsFormat flat = new Lucene99FlatVectorsFormat(FlatVectorScorerUtil.getLucene99FlatVectorsScorer());

    /** The SPI constructor (Lucene instantiates formats by name when it opens a segment). */
    public GpuFlatVectorsFormat() {
        super(NAME);
    }

    @Override
    public KnnVectorsWriter fieldsWriter(SegmentWriteState state) throws IOException {
        return flat.fieldsWriter(state);
    }

    @Override
    public KnnVectorsReader fieldsReader(SegmentReadState state) throws IOException {
        return new GpuFlatVectorsReader(state, flat.fieldsReader(state), DEVICE);
    }

    @Override
    public int getMaxDimensions(String fieldName) {
        return MAX_DIMS;
    }

    @Override
    public String toString() {
        return NAME + "(flat=" + flat + ", device=" + DEVICE + ")";
    }
}
