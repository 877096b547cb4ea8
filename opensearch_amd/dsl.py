"""The `knn_vector` field mapper and the `knn` query builder: the plugin-side DSL in front of the path.

The reference ships no vector DSL (core OpenSearch has no knn_vector mapper and no knn
query); a plugin contributes both through its SPI — `MapperPlugin.getMappers()` (S/plugins/
MapperPlugin.java:59, consumed at S/indices/IndicesModule.java:183) and `SearchPlugin.getQueries()`
(S/plugins/SearchPlugin.java:175, registered as a NamedWriteable + XContent parser at S/search/
SearchModule.java:1191,1255-1258).  Their shape is therefore ours; it follows the OpenSearch k-NN
plugin's public request format so existing requests keep working:

  mapping  {"type": "knn_vector", "dimension": 768, "data_type": "float" | "byte",
            "space_type": "l2" | "innerproduct" | "cosinesimil" | "dot_product",
            "method": {"name": "flat", "engine": "gpu"}}                     (method optional)
  query    {"knn": {"<field>": {"vector": [...], "k": 10, "filter": <query>}}}

`KnnQueryBuilder.do_to_query` ([L] AbstractQueryBuilder.doToQuery, S/index/query/AbstractQueryBuilder.java:
155) returns Lucene's own `KnnFloatVectorQuery` / `KnnByteVectorQuery` (opensearch_amd.lucene), whose
per-leaf search runs on the GPU reader.  The filter is any query over the shard's doc values that
this module parses (term / terms / range / bool / match_all), evaluated per leaf into the accept mask
([L] the filter Weight → AcceptDocs; OpenSearch caches such bitsets in BitsetFilterCache,
S/index/cache/bitset/BitsetFilterCache.java:127-160).  Contract tests mirror AbstractQueryTestCase
(testFromXContent :129, testToQuery :440, testSerialization :597) and MapperTestCase.
"""
from __future__ import annotations

import json
import struct
from dataclasses import dataclass, field
from typing import Any, Callable

import numpy as np

from .lucene import KnnByteVectorQuery, KnnFloatVectorQuery, VectorEncoding, VectorSimilarityFunction

MAX_RESULT_WINDOW = 10000          # index.max_result_window default, S/index/IndexSettings.java:223-226
MAX_DIMENSION = 4096               # libosknn's OSK_MAX_DIM

SPACE_TYPES = {
    "l2": VectorSimilarityFunction.EUCLIDEAN,
    "innerproduct": VectorSimilarityFunction.MAXIMUM_INNER_PRODUCT,
    "cosinesimil": VectorSimilarityFunction.COSINE,
    "dot_product": VectorSimilarityFunction.DOT_PRODUCT,
}
DATA_TYPES = {"float": VectorEncoding.FLOAT32, "byte": VectorEncoding.BYTE}


class MapperParsingException(ValueError):
    """S/index/mapper/MapperParsingException.java: a bad mapping."""


class ParsingException(ValueError):
    """S/core/common/ParsingException: a malformed query body."""


class QueryShardException(ValueError):
    """S/index/query/QueryShardException.java: a query that cannot run on this shard's mappings."""


# ------------------------------------------------------------------------------------------------
# mapper
# ------------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class KnnVectorFieldType:
    """The `knn_vector` MappedFieldType (S/index/mapper/MappedFieldType.java:84)."""
    name: str
    dimension: int
    encoding: VectorEncoding
    similarity: VectorSimilarityFunction
    space_type: str
    data_type: str
    method: dict = field(default_factory=dict, compare=False)

    def to_xcontent(self) -> dict:
        out = {"type": "knn_vector", "dimension": self.dimension, "data_type": self.data_type,
               "space_type": self.space_type}
        if self.method:
            out["method"] = dict(self.method)
        return out


def parse_knn_vector_mapping(name: str, node: dict) -> KnnVectorFieldType:
    """ParametrizedFieldMapper.Builder parse of a `knn_vector` field (S/index/mapper/
    ParametrizedFieldMapper.java:592-640): unknown parameters and bad values are rejected."""
    node = dict(node)
    if node.pop("type", None) != "knn_vector":
        raise MapperParsingException(f"field [{name}] is not of type [knn_vector]")
    if "dimension" not in node:
        raise MapperParsingException(f"Dimension value missing for vector: {name}")
    dim = node.pop("dimension")
    if not isinstance(dim, int) or isinstance(dim, bool) or not 1 <= dim <= MAX_DIMENSION:
        raise MapperParsingException(f"Dimension value must be an integer in [1, {MAX_DIMENSION}] for vector: {name}")
    data_type = node.pop("data_type", "float")
    if data_type not in DATA_TYPES:
        raise MapperParsingException(f"[data_type] must be one of {sorted(DATA_TYPES)} for vector: {name}")
    space = node.pop("space_type", "l2")
    if space not in SPACE_TYPES:
        raise MapperParsingException(f"[space_type] must be one of {sorted(SPACE_TYPES)} for vector: {name}")
    method = node.pop("method", {})
    if method and (method.get("name", "flat") != "flat" or method.get("engine", "gpu") != "gpu"):
        raise MapperParsingException(f"only exact search is served: method {{name: flat, engine: gpu}} ({name})")
    if node:
        raise MapperParsingException(f"unknown parameters {sorted(node)} for field [{name}]")
    return KnnVectorFieldType(name, dim, DATA_TYPES[data_type], SPACE_TYPES[space], space, data_type, method)


def parse_document_vector(ft: KnnVectorFieldType, value) -> np.ndarray:
    """A document's vector as the mapper indexes it (KnnFloatVectorField / KnnByteVectorField [L])."""
    arr = np.asarray(value, dtype=np.float64)
    if arr.ndim != 1 or len(arr) != ft.dimension:
        raise MapperParsingException(f"Vector dimension mismatch. Expected: {ft.dimension}, Given: {arr.size}")
    if not np.all(np.isfinite(arr)):
        raise MapperParsingException("KNN vector values cannot be NaN or Infinity")
    if ft.encoding == VectorEncoding.BYTE:
        if np.any(arr != np.round(arr)) or np.any(arr < -128) or np.any(arr > 127):
            raise MapperParsingException("[data_type] byte requires integers in [-128, 127]")
        return arr.astype(np.int8)
    return arr.astype(np.float32)


# ------------------------------------------------------------------------------------------------
# filter queries (evaluated per leaf over the shard's doc values)
# ------------------------------------------------------------------------------------------------
@dataclass
class QueryShardContext:
    """What a query needs from the shard: its mappings and per-leaf doc values
    (S/index/query/QueryShardContext.java:104; bitsetFilter :369)."""
    mappings: dict[str, Any]                                   # field → KnnVectorFieldType or "keyword"/"long"
    doc_values: Callable[[Any, str], np.ndarray] | None = None  # (leaf, field) → values per doc of the leaf

    def field_type(self, name: str):
        if name not in self.mappings:
            raise QueryShardException(f"failed to find field [{name}]")
        return self.mappings[name]


def _eval_filter(q: dict, ctx: QueryShardContext, leaf) -> np.ndarray:
    (kind, body), = q.items()
    n = leaf.max_doc
    if kind == "match_all":
        return np.ones(n, bool)
    if kind == "term":
        (f, v), = body.items()
        v = v["value"] if isinstance(v, dict) else v
        return ctx.doc_values(leaf, f) == v
    if kind == "terms":
        (f, vs), = body.items()
        return np.isin(ctx.doc_values(leaf, f), np.asarray(vs))
    if kind == "range":
        (f, b), = body.items()
        x = ctx.doc_values(leaf, f)
        m = np.ones(n, bool)
        for op, fn in (("gt", np.greater), ("gte", np.greater_equal), ("lt", np.less), ("lte", np.less_equal)):
            if op in b:
                m &= fn(x, b[op])
        return m
    if kind == "bool":
        m = np.ones(n, bool)
        for c in body.get("must", []) + body.get("filter", []):
            m &= _eval_filter(c, ctx, leaf)
        for c in body.get("must_not", []):
            m &= ~_eval_filter(c, ctx, leaf)
        should = body.get("should", [])
        if should:
            s = np.zeros(n, bool)
            for c in should:
                s |= _eval_filter(c, ctx, leaf)
            m &= s
        return m
    raise ParsingException(f"unknown filter query [{kind}]")


def _check_filter(q) -> None:
    if not isinstance(q, dict) or len(q) != 1:
        raise ParsingException("a filter is an object with exactly one query")
    (kind, body), = q.items()
    if kind == "bool":
        for clause in ("must", "filter", "must_not", "should"):
            for c in body.get(clause, []):
                _check_filter(c)
    elif kind not in ("match_all", "term", "terms", "range"):
        raise ParsingException(f"unknown filter query [{kind}]")


# ------------------------------------------------------------------------------------------------
# the knn query builder
# ------------------------------------------------------------------------------------------------
NAME = "knn"


@dataclass
class KnnQueryBuilder:
    """[L]-backed `knn` QueryBuilder (S/index/query/AbstractQueryBuilder.java:69)."""
    field_name: str
    vector: list
    k: int
    filter: dict | None = None
    boost: float = 1.0
    query_name: str | None = None

    def __post_init__(self):
        if not self.field_name:
            raise ValueError("[knn] requires a field name")
        if not isinstance(self.k, int) or isinstance(self.k, bool) or self.k < 1:
            raise ValueError("[knn] requires k > 0")
        if self.k > MAX_RESULT_WINDOW:
            raise ValueError(f"[knn] requires k <= {MAX_RESULT_WINDOW}")
        if not self.vector:
            raise ValueError("[knn] query vector is empty")
        if self.filter is not None:
            _check_filter(self.filter)

    # ---- XContent ------------------------------------------------------------------------------
    def to_xcontent(self) -> dict:
        inner = {"vector": list(self.vector), "k": self.k}
        if self.filter is not None:
            inner["filter"] = self.filter
        if self.boost != 1.0:
            inner["boost"] = self.boost
        if self.query_name is not None:
            inner["_name"] = self.query_name
        return {NAME: {self.field_name: inner}}

    @classmethod
    def from_xcontent(cls, body: dict | str) -> "KnnQueryBuilder":
        if isinstance(body, str):
            body = json.loads(body)
        if set(body) != {NAME}:
            raise ParsingException("expected a [knn] query")
        fields = body[NAME]
        if not isinstance(fields, dict) or len(fields) != 1:
            raise ParsingException("[knn] query expects exactly one field")
        (name, inner), = fields.items()
        if not isinstance(inner, dict):
            raise ParsingException("[knn] field body must be an object")
        unknown = set(inner) - {"vector", "k", "filter", "boost", "_name"}
        if unknown:
            raise ParsingException(f"[knn] unknown field(s) {sorted(unknown)}")
        if "vector" not in inner or "k" not in inner:
            raise ParsingException("[knn] requires [vector] and [k]")
        try:
            return cls(name, list(inner["vector"]), inner["k"], inner.get("filter"), float(inner.get("boost", 1.0)),
                       inner.get("_name"))
        except ValueError as e:
            raise ParsingException(str(e)) from e

    # ---- transport serialisation (NamedWriteable: writeTo / StreamInput ctor) -------------------
    def write_to(self) -> bytes:
        name = self.field_name.encode()
        filt = b"" if self.filter is None else json.dumps(self.filter, sort_keys=True).encode()
        qn = b"" if self.query_name is None else self.query_name.encode()
        vec = np.asarray(self.vector, np.float32)
        return (struct.pack(">I", len(name)) + name + struct.pack(">I", len(vec)) + vec.astype(">f4").tobytes()
                + struct.pack(">i", self.k) + struct.pack(">?", self.filter is not None)
                + struct.pack(">I", len(filt)) + filt + struct.pack(">f", self.boost)
                + struct.pack(">?", self.query_name is not None) + struct.pack(">I", len(qn)) + qn)

    @classmethod
    def read_from(cls, data: bytes) -> "KnnQueryBuilder":
        p = 0

        def take(n):
            nonlocal p
            v = data[p:p + n]
            p += n
            return v
        name = take(struct.unpack(">I", take(4))[0]).decode()
        n = struct.unpack(">I", take(4))[0]
        vec = np.frombuffer(take(4 * n), ">f4").astype(np.float32).tolist()
        k = struct.unpack(">i", take(4))[0]
        has_f = struct.unpack(">?", take(1))[0]
        filt = take(struct.unpack(">I", take(4))[0])
        boost = struct.unpack(">f", take(4))[0]
        has_qn = struct.unpack(">?", take(1))[0]
        qn = take(struct.unpack(">I", take(4))[0]).decode()
        return cls(name, vec, k, json.loads(filt) if has_f else None, boost, qn if has_qn else None)

    # ---- toQuery ---------------------------------------------------------------------------------
    def do_to_query(self, ctx: QueryShardContext):
        """[L] KnnFloatVectorQuery / KnnByteVectorQuery over the field, with the filter as per-leaf
        accept masks (AcceptDocs ∩ liveDocs is applied by the query's rewrite)."""
        ft = ctx.field_type(self.field_name)
        if not isinstance(ft, KnnVectorFieldType):
            raise QueryShardException(f"Field '{self.field_name}' is not knn_vector type.")
        target = parse_document_vector(ft, self.vector) if len(self.vector) == ft.dimension else None
        if target is None:
            raise QueryShardException(f"Query vector has invalid dimension: {len(self.vector)}. "
                                      f"Dimension should be: {ft.dimension}")
        filt = None
        if self.filter is not None:
            if ctx.doc_values is None:
                raise QueryShardException("[knn] filter needs the shard's doc values")
            filt = lambda leaf, q=self.filter: _eval_filter(q, ctx, leaf)   # noqa: E731
        cls = KnnByteVectorQuery if ft.encoding == VectorEncoding.BYTE else KnnFloatVectorQuery
        return cls(self.field_name, target, self.k, filt)


def parse_query(body: dict | str) -> KnnQueryBuilder:
    """SearchModule's registered parser for the `knn` NamedWriteable (S/search/SearchModule.java:1255-1258)."""
    return KnnQueryBuilder.from_xcontent(body)
