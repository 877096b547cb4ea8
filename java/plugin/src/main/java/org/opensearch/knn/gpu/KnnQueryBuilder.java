/*
 * The `knn` query: {"knn": {"<field>": {"vector": [...], "k": 10, "filter": <query>, "boost": 1, "_name": ...}}}.
 * Registered by GpuKnnPlugin.getQueries (S/plugins/SearchPlugin.java:175) as a NamedWriteable and a
 * NamedXContent parser (S/search/SearchModule.java:1191,1255-1258).  doToQuery returns the GPU query of the
 * field's encoding (one osk_view_search per shard, GpuKnnFloatVectorQuery).  Python mirror: dsl.py.
 */
package org.opensearch.knn.gpu;

import java.io.IOException;
import java.util.ArrayList;
import java.util.Arrays;
import java.util.List;
import java.util.Objects;

import org.apache.lucene.search.Query;
import org.opensearch.core.ParseField;
import org.opensearch.core.common.ParsingException;
import org.opensearch.core.common.io.stream.StreamInput;
import org.opensearch.core.common.io.stream.StreamOutput;
import org.opensearch.core.xcontent.XContentBuilder;
import org.opensearch.core.xcontent.XContentParser;
import org.opensearch.index.mapper.MappedFieldType;
import org.opensearch.index.query.AbstractQueryBuilder;
import org.opensearch.index.query.QueryBuilder;
import org.opensearch.index.query.QueryShardContext;
import org.opensearch.index.query.QueryShardException;

public final class KnnQueryBuilder extends AbstractQueryBuilder<KnnQueryBuilder> {
    public static final String NAME = "knn";
    static final ParseField VECTOR = new ParseField("vector");
    static final ParseField K = new ParseField("k");
    static final ParseField FILTER = new ParseField("filter");
    static final int MAX_K = 10000;   // index.max_result_window (S/index/IndexSettings.java:223-226) = OSK_MAX_K

    private final String field;
    private final float[] vector;
    private final int k;
    private final QueryBuilder filter;

    public KnnQueryBuilder(String field, float[] vector, int k, QueryBuilder filter) {
        if (field == null || field.isEmpty()) throw new IllegalArgumentException("[knn] requires a field");
        if (vector == null || vector.length == 0) throw new IllegalArgumentException("[knn] requires a vector");
        if (k < 1 || k > MAX_K) throw new IllegalArgumentException("[knn] k must be in [1, " + MAX_K + "], got " + k);
        this.field = field;
        this.vector = vector;
        this.k = k;
        this.filter = filter;
    }

    /** The Writeable.Reader. */
    public KnnQueryBuilder(StreamInput in) throws IOException {
        super(in);
        field = in.readString();
        vector = in.readFloatArray();
        k = in.readVInt();
        filter = in.readOptionalNamedWriteable(QueryBuilder.class);
    }

    @Override
    protected void doWriteTo(StreamOutput out) throws IOException {
        out.writeString(field);
        out.writeFloatArray(vector);
        out.writeVInt(k);
        out.writeOptionalNamedWriteable(filter);
    }

    public static KnnQueryBuilder fromXContent(XContentParser parser) throws IOException {
        String field = null, queryName = null;
        float[] vector = null;
        Integer k = null;
        QueryBuilder filter = null;
        float boost = DEFAULT_BOOST;
        XContentParser.Token token = parser.nextToken();
        if (token != XContentParser.Token.FIELD_NAME) throw new ParsingException(parser.getTokenLocation(), "[knn] expects a field");
        field = parser.currentName();
        if (parser.nextToken() != XContentParser.Token.START_OBJECT)
            throw new ParsingException(parser.getTokenLocation(), "[knn] expects an object for field [" + field + "]");
        String current = null;
        while ((token = parser.nextToken()) != XContentParser.Token.END_OBJECT) {
            if (token == XContentParser.Token.FIELD_NAME) {
                current = parser.currentName();
            } else if (VECTOR.match(current, parser.getDeprecationHandler())) {
                List<Float> v = new ArrayList<>();
                for (token = parser.nextToken(); token != XContentParser.Token.END_ARRAY; token = parser.nextToken())
                    v.add(parser.floatValue());
                vector = new float[v.size()];
                for (int i = 0; i < vector.length; i++) vector[i] = v.get(i);
            } else if (K.match(current, parser.getDeprecationHandler())) {
                k = parser.intValue();
            } else if (FILTER.match(current, parser.getDeprecationHandler())) {
                filter = parseInnerQueryBuilder(parser);
            } else if (BOOST_FIELD.match(current, parser.getDeprecationHandler())) {
                boost = parser.floatValue();
            } else if (NAME_FIELD.match(current, parser.getDeprecationHandler())) {
                queryName = parser.text();
            } else {
                throw new ParsingException(parser.getTokenLocation(), "[knn] unknown parameter [" + current + "]");
            }
        }
        if (parser.nextToken() != XContentParser.Token.END_OBJECT)
            throw new ParsingException(parser.getTokenLocation(), "[knn] supports exactly one field");
        if (k == null) throw new ParsingException(parser.getTokenLocation(), "[knn] requires k");
        KnnQueryBuilder b = new KnnQueryBuilder(field, vector, k, filter);
        b.boost(boost);
        b.queryName(queryName);
        return b;
    }

    @Override
    protected void doXContent(XContentBuilder builder, Params params) throws IOException {
        builder.startObject(NAME);
        builder.startObject(field);
        builder.array(VECTOR.getPreferredName(), vector);
        builder.field(K.getPreferredName(), k);
        if (filter != null) builder.field(FILTER.getPreferredName(), filter);
        printBoostAndQueryName(builder);
        builder.endObject();
        builder.endObject();
    }

    @Override
    protected Query doToQuery(QueryShardContext context) throws IOException {
        MappedFieldType mft = context.fieldMapper(field);
        if (mft == null || !(mft.unwrap() instanceof KnnVectorFieldMapper.KnnVectorFieldType ft))
            throw new QueryShardException(context, "[knn] field [" + field + "] is not a knn_vector field");
        if (vector.length != ft.dimension())
            throw new QueryShardException(context, "[knn] vector has " + vector.length + " dims, field [" + field + "] "
                + ft.dimension());
        Query f = filter == null ? null : filter.toQuery(context);
        return ft.isByte() ? new GpuKnnByteVectorQuery(field, ft.toBytes(vector), k, f)
                           : new GpuKnnFloatVectorQuery(field, vector, k, f);
    }

    @Override
    protected boolean doEquals(KnnQueryBuilder other) {
        return field.equals(other.field) && Arrays.equals(vector, other.vector) && k == other.k
            && Objects.equals(filter, other.filter);
    }

    @Override
    protected int doHashCode() {
        return Objects.hash(field, Arrays.hashCode(vector), k, filter);
    }

    @Override
    public String getWriteableName() {
        return NAME;
    }
}
