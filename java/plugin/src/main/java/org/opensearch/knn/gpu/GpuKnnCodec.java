/*
 * The index's codec with the plugin: OpenSearch's per-field codec (S/index/codec/PerFieldMappingPostingFormatCodec
 * .java:62 — it must subclass the latest Lucene codec, Lucene103Codec) whose per-field vectors format is
 * GpuFlatVectorsFormat for knn_vector fields.  Every other format is OpenSearch's.
 */
package org.opensearch.knn.gpu;

import org.apache.logging.log4j.Logger;
import org.apache.lucene.codecs.KnnVectorsFormat;
import org.opensearch.index.codec.PerFieldMappingPostingFormatCodec;
import org.opensearch.index.mapper.MappedFieldType;
import org.opensearch.index.mapper.MapperService;

public final class GpuKnnCodec extends PerFieldMappingPostingFormatCodec {
    private static final KnnVectorsFormat GPU_FORMAT = new GpuFlatVectorsFormat();
    private final MapperService mapperService;

    public GpuKnnCodec(Mode compressionMode, MapperService mapperService, Logger logger) {
        super(compressionMode, mapperService, logger);
        this.mapperService = mapperService;
    }

    @Override
    public KnnVectorsFormat getKnnVectorsFormatForField(String field) {
        MappedFieldType ft = mapperService.fieldType(field);
        if (ft != null && ft.unwrap() instanceof KnnVectorFieldMapper.KnnVectorFieldType) return GPU_FORMAT;
        return super.getKnnVectorsFormatForField(field);
    }
}
