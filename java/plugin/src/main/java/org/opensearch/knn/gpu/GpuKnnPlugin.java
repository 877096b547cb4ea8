/*
 * The plugin: the `knn` query (SearchPlugin.getQueries, S/plugins/SearchPlugin.java:175), the `knn_vector`
 * field (MapperPlugin.getMappers, S/plugins/MapperPlugin.java:59), the codec of indices with index.knn.gpu = true
 * (EnginePlugin.getCustomCodecServiceFactory, S/plugins/EnginePlugin.java:87) and the setting itself.  The
 * vectors format is found by Lucene's SPI (META-INF/services/org.apache.lucene.codecs.KnnVectorsFormat,
 * reloaded for plugins at S/plugins/PluginsService.java:828-836), so segments written with it open on any
 * node with the plugin.
 */
package org.opensearch.knn.gpu;

import java.util.List;
import java.util.Map;
import java.util.Optional;

import org.opensearch.common.settings.Setting;
import org.opensearch.index.IndexSettings;
import org.opensearch.index.codec.CodecServiceFactory;
import org.opensearch.index.mapper.Mapper;
import org.opensearch.plugins.EnginePlugin;
import org.opensearch.plugins.MapperPlugin;
import org.opensearch.plugins.Plugin;
import org.opensearch.plugins.SearchPlugin;

public final class GpuKnnPlugin extends Plugin implements SearchPlugin, MapperPlugin, EnginePlugin {
    /** index.knn.gpu: knn_vector fields of the index use GpuFlatVectorsFormat (set at index creation). */
    public static final Setting<Boolean> INDEX_KNN_GPU = Setting.boolSetting(
        "index.knn.gpu", false, Setting.Property.IndexScope, Setting.Property.Final);

    @Override
    public List<Setting<?>> getSettings() {
        return List.of(INDEX_KNN_GPU);
    }

    /** S/plugins/SearchPlugin.java:175 — QuerySpec(name, Writeable.Reader, QueryParser), registered by
     *  SearchModule.registerQuery as a NamedWriteable and a NamedXContent parser. */
    @Override
    public List<QuerySpec<?>> getQueries() {
        return List.of(new QuerySpec<>(KnnQueryBuilder.NAME, KnnQueryBuilder::new, KnnQueryBuilder::fromXContent));
    }

    @Override
    public Map<String, Mapper.TypeParser> getMappers() {
        return Map.of(KnnVectorFieldMapper.CONTENT_TYPE, KnnVectorFieldMapper.PARSER);
    }

    @Override
    public Optional<CodecServiceFactory> getCustomCodecServiceFactory(IndexSettings indexSettings) {
        if (INDEX_KNN_GPU.get(indexSettings.getSettings()) == false) return Optional.empty();
        return Optional.of(GpuCodecService::new);
    }
}
