/*
 * CodecService of an index with index.knn.gpu = true (EnginePlugin.getCustomCodecServiceFactory,
 * S/plugins/EnginePlugin.java:87; CodecServiceFactory, S/index/codec/CodecServiceFactory.java:17-24, one per
 * index, S/index/engine/EngineConfigFactory.java:103-124): OpenSearch's codec names ("default", "lz4",
 * "best_compression", "zlib") map to GpuKnnCodec with the same compression mode; every other name is
 * OpenSearch's own.
 */
package org.opensearch.knn.gpu;

import java.util.Map;

import org.apache.lucene.codecs.Codec;
import org.apache.lucene.codecs.lucene103.Lucene103Codec;
import org.opensearch.index.codec.CodecService;
import org.opensearch.index.codec.CodecServiceConfig;

final class GpuCodecService extends CodecService {
    private final Map<String, Codec> gpu;

    GpuCodecService(CodecServiceConfig config) {
        super(config.getMapperService(), config.getIndexSettings(), config.getLogger());
        if (config.getMapperService() == null) {
            gpu = Map.of();
        } else {
            Codec fast = new GpuKnnCodec(Lucene103Codec.Mode.BEST_SPEED, config.getMapperService(), config.getLogger());
            Codec small = new GpuKnnCodec(Lucene103Codec.Mode.BEST_COMPRESSION, config.getMapperService(), config.getLogger());
            gpu = Map.of(DEFAULT_CODEC, fast, LZ4, fast, BEST_COMPRESSION_CODEC, small, ZLIB, small);
        }
    }

    @Override
    public Codec codec(String name) {
        Codec c = gpu.get(name);
        return c != null ? c : super.codec(name);
    }
}
