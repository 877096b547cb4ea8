/*
 * The `knn_vector` field (MapperPlugin.getMappers, S/plugins/MapperPlugin.java:59):
 *   {"type": "knn_vector", "dimension": 768, "data_type": "float" | "byte",
 *    "space_type": "l2" | "innerproduct" | "cosinesimil" | "dot_product", "method": {...}}
 * indexed as Lucene's KnnFloatVectorField / KnnByteVectorField with the space type's VectorSimilarityFunction;
 * the codec (GpuKnnCodec) gives the field GpuFlatVectorsFormat.  Python mirror and contract tests:
 * opensearch_amd/dsl.py, tests/test_dsl.py.
 */
package org.opensearch.knn.gpu;

import java.io.IOException;
import java.util.ArrayList;
import java.util.Collections;
import java.util.List;
import java.util.Map;

import org.apache.lucene.document.FieldType;
import org.apache.lucene.document.KnnByteVectorField;
import org.apache.lucene.document.KnnFloatVectorField;
import org.apache.lucene.index.VectorEncoding;
import org.apache.lucene.index.VectorSimilarityFunction;
import org.apache.lucene.search.FieldExistsQuery;
import org.apache.lucene.search.Query;
import org.opensearch.core.xcontent.XContentParser;
import org.opensearch.index.mapper.MappedFieldType;
import org.opensearch.index.mapper.ParametrizedFieldMapper;
import org.opensearch.index.mapper.ParseContext;
import org.opensearch.index.mapper.SourceValueFetcher;
import org.opensearch.index.mapper.TextSearchInfo;
import org.opensearch.index.mapper.ValueFetcher;
import org.opensearch.index.query.QueryShardContext;
import org.opensearch.index.query.QueryShardException;
import org.opensearch.search.lookup.SearchLookup;

public final class KnnVectorFieldMapper extends ParametrizedFieldMapper {
    public static final String CONTENT_TYPE = "knn_vector";

    static VectorSimilarityFunction similarity(String spaceType) {
        switch (spaceType) {
            case "l2": return VectorSimilarityFunction.EUCLIDEAN;
            case "innerproduct": return VectorSimilarityFunction.MAXIMUM_INNER_PRODUCT;
            case "cosinesimil": return VectorSimilarityFunction.COSINE;
            case "dot_product": return VectorSimilarityFunction.DOT_PRODUCT;
            default: throw new IllegalArgumentException("unknown space_type [" + spaceType + "]");
        }
    }

    private static KnnVectorFieldMapper toType(org.opensearch.index.mapper.FieldMapper in) {
        return (KnnVectorFieldMapper) in;
    }

    public static final class Builder extends ParametrizedFieldMapper.Builder {
        private final Parameter<Integer> dimension = Parameter.intParam("dimension", false, m -> toType(m).dimension, -1)
            .setValidator(d -> {
                if (d < 1 || d > GpuFlatVectorsFormat.MAX_DIMS)
                    throw new IllegalArgumentException("dimension must be in [1, " + GpuFlatVectorsFormat.MAX_DIMS + "], got " + d);
            });
        private final Parameter<String> dataType = Parameter.restrictedStringParam("data_type", false,
            m -> toType(m).dataType, "float", "byte");
        private final Parameter<String> spaceType = Parameter.restrictedStringParam("space_type", false,
            m -> toType(m).spaceType, "l2", "innerproduct", "cosinesimil", "dot_product");
        private final Parameter<Map<String, String>> meta = Parameter.metaParam();

        public Builder(String name) {
            super(name);
        }

        @Override
        protected List<Parameter<?>> getParameters() {
            return List.of(dimension, dataType, spaceType, meta);
        }

        @Override
        public KnnVectorFieldMapper build(BuilderContext context) {
            KnnVectorFieldType ft = new KnnVectorFieldType(buildFullName(context), dimension.getValue(),
                "byte".equals(dataType.getValue()) ? VectorEncoding.BYTE : VectorEncoding.FLOAT32,
                similarity(spaceType.getValue()), meta.getValue());
            return new KnnVectorFieldMapper(name, ft, multiFieldsBuilder.build(this, context), copyTo.build(), this);
        }
    }

    public static final TypeParser PARSER = new TypeParser((n, c) -> new Builder(n));

    /** The field type: its dimension, encoding and similarity decide the Lucene field and the query. */
    public static final class KnnVectorFieldType extends MappedFieldType {
        private final int dimension;
        private final VectorEncoding encoding;
        private final VectorSimilarityFunction similarity;

        public KnnVectorFieldType(String name, int dimension, VectorEncoding encoding, VectorSimilarityFunction similarity,
                                  Map<String, String> meta) {
            super(name, false, false, false, TextSearchInfo.NONE, meta);
            this.dimension = dimension;
            this.encoding = encoding;
            this.similarity = similarity;
        }

        public int dimension() {
            return dimension;
        }

        public boolean isByte() {
            return encoding == VectorEncoding.BYTE;
        }

        public VectorSimilarityFunction similarity() {
            return similarity;
        }

        /** A query vector as bytes for a byte field: every component an integer in [-128, 127]. */
        public byte[] toBytes(float[] v) {
            byte[] b = new byte[v.length];
            for (int i = 0; i < v.length; i++) {
                if (v[i] != Math.rint(v[i]) || v[i] < -128 || v[i] > 127)
                    throw new IllegalArgumentException("byte vector component [" + v[i] + "] is not an integer in [-128, 127]");
                b[i] = (byte) v[i];
            }
            return b;
        }

        @Override
        public String typeName() {
            return CONTENT_TYPE;
        }

        @Override
        public ValueFetcher valueFetcher(QueryShardContext context, SearchLookup searchLookup, String format) {
            return SourceValueFetcher.identity(name(), context, format);
        }

        @Override
        public Query existsQuery(QueryShardContext context) {
            return new FieldExistsQuery(name());
        }

        @Override
        public Query termQuery(Object value, QueryShardContext context) {
            throw new QueryShardException(context, "knn_vector field [" + name() + "] supports only the knn query");
        }
    }

    private final int dimension;
    private final String dataType, spaceType;

    private KnnVectorFieldMapper(String simpleName, KnnVectorFieldType ft, MultiFields multiFields, CopyTo copyTo, Builder b) {
        super(simpleName, ft, multiFields, copyTo);
        this.dimension = b.dimension.getValue();
        this.dataType = b.dataType.getValue();
        this.spaceType = b.spaceType.getValue();
    }

    @Override
    public KnnVectorFieldType fieldType() {
        return (KnnVectorFieldType) super.fieldType();
    }

    @Override
    protected void parseCreateField(ParseContext context) throws IOException {
        XContentParser parser = context.parser();
        List<Float> values = new ArrayList<>();
        if (parser.currentToken() != XContentParser.Token.START_ARRAY)
            throw new IllegalArgumentException("knn_vector field [" + name() + "] expects an array of numbers");
        for (XContentParser.Token t = parser.nextToken(); t != XContentParser.Token.END_ARRAY; t = parser.nextToken())
            values.add(parser.floatValue());
        if (values.size() != dimension)
            throw new IllegalArgumentException("vector of field [" + name() + "] has " + values.size() + " dims, the mapping "
                + dimension);
        KnnVectorFieldType ft = fieldType();
        float[] v = new float[values.size()];
        for (int i = 0; i < v.length; i++) v[i] = values.get(i);
        if (ft.isByte()) {
            context.doc().add(new KnnByteVectorField(ft.name(), ft.toBytes(v), ft.similarity()));
        } else {
            context.doc().add(new KnnFloatVectorField(ft.name(), v, ft.similarity()));
        }
    }

    @Override
    public ParametrizedFieldMapper.Builder getMergeBuilder() {
        return new Builder(simpleName()).init(this);
    }

    @Override
    protected String contentType() {
        return CONTENT_TYPE;
    }
}
