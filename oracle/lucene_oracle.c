/*
 * lucene_oracle.c — CPU restatement of the exact k-NN scoring path, used ONLY as a checker.
 *
 * TEST INFRASTRUCTURE.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only to check or to time the CPU baseline.  Nothing in opensearch_amd/
 * links, imports or calls it; the product path has no CPU fallback.
 *
 * What it restates (the reference snapshot is OpenSearch 3.3.0 on lucene-core 10.3.0; Lucene is an
 * un-vendored jar, gradle/libs.versions.toml:3, sha1 in server/licenses/lucene-core-10.3.0.jar.sha1,
 * so every [L] item is written from Lucene's published source, not from /root/reference):
 *   [L] VectorUtil.dotProduct / squareDistance / cosine (float[] and byte[]) in three summation
 *       orders: ORDER_DEVICE (the lane layout libosknn documents, DESIGN.md §Kernels — used for
 *       bit-exact checks), ORDER_SCALAR (DefaultVectorUtilSupport) and ORDER_PANAMA512
 *       (PanamaVectorUtilSupport with a 16-lane float species, 4 accumulators, reduceLanes modelled
 *       as a left-to-right lane sum).  Byte sums are exact int32, so the order is irrelevant there.
 *   [L] VectorSimilarityFunction.compare score transforms (EUCLIDEAN, DOT_PRODUCT, COSINE,
 *       MAXIMUM_INNER_PRODUCT) for float and byte vectors.
 *   [L] AbstractKnnVectorQuery.exactSearch: docs visited in ascending order, a HitQueue
 *       pre-populated with (−inf, Integer.MAX_VALUE) sentinels, replacement on a STRICTLY greater
 *       score (so equal scores keep the lower doc), sentinels dropped, result score desc / doc asc.
 *       Driven in the reference from S/search/internal/ContextIndexSearcher.java:203-218.
 *   [L] TopDocs.merge(start, size, shardHits) as SearchPhaseController.mergeTopDocs calls it
 *       (server/src/main/java/org/opensearch/action/search/SearchPhaseController.java:224-246,
 *       setShardIndex :248-253): score desc, shardIndex asc, doc asc; single shard with from == 0
 *       returned as is (:231-232); TopDocsStats (:839-901).
 *   The synthetic corpus generator of libosknn, restated independently.
 *
 * Pinning: the merge is pinned by the reference's own known-answer tests
 * (server/src/test/java/org/opensearch/action/search/SearchPhaseControllerTests.java:1347-1392,
 * FetchSearchPhaseTests.java:124-218; restated as fixtures in tests/golden/).  SCORING PARITY IS
 * UNPINNED: the reference holds no vector test, fixture or Lucene jar, and no JDK exists here
 * (SURVEY.md §8(c)).  The scoring formulas above are Lucene's published ones; DESIGN.md §Oracle.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORDER_DEVICE 0
#define ORDER_SCALAR 1
#define ORDER_PANAMA512 2
#define ORDER_SCALAR_NOFMA 3      /* Lucene's orders on a CPU without fast FMA (mul, then add) */
#define ORDER_PANAMA512_NOFMA 4

enum { SIM_EUCLIDEAN = 0, SIM_DOT_PRODUCT = 1, SIM_COSINE = 2, SIM_MIP = 3 };

/* ------------------------------------------------------------------------------------------ */
/* generator (restated)                                                                        */
/* ------------------------------------------------------------------------------------------ */
static uint64_t sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

static float gen_raw(int dist, uint64_t h) {
    if (dist == 0) return (float)(h >> 40) * 0x1p-24f;
    if (dist == 1) return ((float)(h >> 40) * 0x1p-24f) * 128.0f;
    uint32_t s = (uint32_t)(h & 0xFFFF) + (uint32_t)((h >> 16) & 0xFFFF) + (uint32_t)((h >> 32) & 0xFFFF) +
                 (uint32_t)(h >> 48);
    return ((float)s * 0x1p-16f - 2.0f) * 1.7320508f;
}

int orc_synth(void* out, int64_t row0, int64_t n, int dim, uint64_t seed, int dist) {
    const uint64_t mix = sm64(seed);
    for (int64_t r = 0; r < n; ++r) {
        const uint64_t g = (uint64_t)(row0 + r);
        if (dist == 4) {
            int8_t* o = (int8_t*)out + r * dim;
            for (int c = 0; c < dim; ++c) o[c] = (int8_t)(uint8_t)(sm64(mix + g * (uint64_t)dim + c) >> 56);
            continue;
        }
        float* o = (float*)out + r * dim;
        for (int c = 0; c < dim; ++c) o[c] = gen_raw(dist, sm64(mix + g * (uint64_t)dim + c));
        if (dist == 3) {
            float p[64];
            for (int l = 0; l < 64; ++l) {
                float a = 0.0f;
                for (int c = l; c < dim; c += 64) a = fmaf(o[c], o[c], a);
                p[l] = a;
            }
            for (int w = 32; w >= 1; w >>= 1)
                for (int i = 0; i < w; ++i) p[i] = p[i] + p[i + w];
            const float den = sqrtf(p[0]);
            for (int c = 0; c < dim; ++c) o[c] = o[c] / den;
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* float reductions                                                                            */
/* ------------------------------------------------------------------------------------------ */
/* lane layout of libosknn: units = ceil(dim/4) float4s; (L, V) by units */
static void lane_cfg(int units, int* L, int* V) {
    static const int lim[9] = {8, 16, 32, 64, 128, 192, 256, 512, 1 << 30};
    static const int LL[9] = {4, 8, 8, 16, 16, 16, 32, 64, 64};
    static const int VV[9] = {2, 2, 4, 4, 8, 12, 8, 8, 16};
    for (int i = 0; i < 9; ++i)
        if (units <= lim[i]) { *L = LL[i]; *V = VV[i]; return; }
}

static inline float elem(const float* v, int dim, int i) { return i < dim ? v[i] : 0.0f; }

/* kind 0: Σ a·b, kind 1: Σ (a−b)² — in the device lane layout.  Lane t keeps 4 fma chains over
 * units t, t+L, t+2L, …; chain e of lane t sees elements 4(t + jL) + e, j = 0..V−1, i.e. position
 * i = 4t + e of the j-th contiguous block of 4L elements — so the 4L chains are one contiguous fma
 * sweep per block (vectorisable, same arithmetic).  Then (x+y)+(z+w) per lane and an xor-butterfly
 * over the L lanes. */
static float device_sum(const float* a, const float* b, int dim, int kind) {
    int L, V;
    const int units = (dim + 3) / 4;
    lane_cfg(units, &L, &V);
    const int W = 4 * L;
    float acc[256];
    for (int i = 0; i < W; ++i) acc[i] = 0.0f;
    for (int j = 0; j < V; ++j) {
        const int base = j * W;
        if (base + W <= dim) {
            const float* x = a + base;
            const float* y = b + base;
            if (kind == 0)
                for (int i = 0; i < W; ++i) acc[i] = fmaf(x[i], y[i], acc[i]);
            else
                for (int i = 0; i < W; ++i) { const float d = x[i] - y[i]; acc[i] = fmaf(d, d, acc[i]); }
        } else {   /* the ragged tail block (zeros past dim, as the padded rows) */
            for (int i = 0; i < W; ++i) {
                const float x = elem(a, dim, base + i), y = elem(b, dim, base + i);
                if (kind == 0) acc[i] = fmaf(x, y, acc[i]);
                else { const float d = x - y; acc[i] = fmaf(d, d, acc[i]); }
            }
        }
    }
    float p[64];
    for (int t = 0; t < L; ++t) p[t] = (acc[4 * t] + acc[4 * t + 1]) + (acc[4 * t + 2] + acc[4 * t + 3]);
    for (int m = 1; m < L; m <<= 1) {
        float nx[64];
        for (int t = 0; t < L; ++t) nx[t] = p[t] + p[t ^ m];
        memcpy(p, nx, sizeof(float) * L);
    }
    return p[0];
}

/* [L] Lucene fuses the multiply-add only where the CPU has fast FMA (Constants.HAS_FAST_SCALAR_FMA /
 * HAS_FAST_VECTOR_FMA); elsewhere it is a rounded multiply then an add.  `fused` selects which
 * (ORDER_SCALAR / ORDER_PANAMA512 fuse, the *_NOFMA orders do not; -ffp-contract=off keeps a*b + c
 * two roundings). */
static inline float mac(float a, float b, float c, int fused) { return fused ? fmaf(a, b, c) : a * b + c; }

/* [L] DefaultVectorUtilSupport: 4 fma accumulators over a 4-aligned prefix when dim > 32, summed
 * ((a1+a2)+a3)+a4 and added to 0, then a scalar fma tail. */
static float scalar_sum(const float* a, const float* b, int dim, int kind, int fused) {
    float res = 0.0f;
    int i = 0;
    if (dim > 32) {
        float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        const int ub = dim & ~3;
        for (; i < ub; i += 4)
            for (int e = 0; e < 4; ++e) {
                if (kind == 0) acc[e] = mac(a[i + e], b[i + e], acc[e], fused);
                else { const float d = a[i + e] - b[i + e]; acc[e] = mac(d, d, acc[e], fused); }
            }
        res += ((acc[0] + acc[1]) + acc[2]) + acc[3];
    }
    for (; i < dim; ++i) {
        if (kind == 0) res = mac(a[i], b[i], res, fused);
        else { const float d = a[i] - b[i]; res = mac(d, d, res, fused); }
    }
    return res;
}

/* [L] PanamaVectorUtilSupport with FLOAT_SPECIES of 16 lanes (AVX-512): vector body when
 * dim > 2·16, unrolled by 4 accumulators, vector tail into acc1, lane-wise (acc1+acc2)+(acc3+acc4),
 * reduceLanes(ADD) (modelled left to right), scalar fma tail. */
static float panama_sum(const float* a, const float* b, int dim, int kind, int fused) {
    const int S = 16;
    float res = 0.0f;
    int i = 0;
    if (dim > 2 * S) {
        const int limit = dim - dim % S;
        float acc[4][16];
        memset(acc, 0, sizeof(acc));
        const int unrolled = limit - 3 * S;
        for (; i < unrolled; i += 4 * S)
            for (int u = 0; u < 4; ++u)
                for (int l = 0; l < S; ++l) {
                    const int ix = i + u * S + l;
                    if (kind == 0) acc[u][l] = mac(a[ix], b[ix], acc[u][l], fused);
                    else { const float d = a[ix] - b[ix]; acc[u][l] = mac(d, d, acc[u][l], fused); }
                }
        for (; i < limit; i += S)
            for (int l = 0; l < S; ++l) {
                const int ix = i + l;
                if (kind == 0) acc[0][l] = mac(a[ix], b[ix], acc[0][l], fused);
                else { const float d = a[ix] - b[ix]; acc[0][l] = mac(d, d, acc[0][l], fused); }
            }
        float r = 0.0f;
        for (int l = 0; l < S; ++l) r += (acc[0][l] + acc[1][l]) + (acc[2][l] + acc[3][l]);
        res += r;
    }
    for (; i < dim; ++i) {
        if (kind == 0) res = mac(a[i], b[i], res, fused);
        else { const float d = a[i] - b[i]; res = mac(d, d, res, fused); }
    }
    return res;
}

static float fsum(const float* a, const float* b, int dim, int kind, int order) {
    if (order == ORDER_SCALAR || order == ORDER_SCALAR_NOFMA) return scalar_sum(a, b, dim, kind, order == ORDER_SCALAR);
    if (order == ORDER_PANAMA512 || order == ORDER_PANAMA512_NOFMA)
        return panama_sum(a, b, dim, kind, order == ORDER_PANAMA512);
    return device_sum(a, b, dim, kind);
}

/* [L] cosine's three sums.  DEVICE: dot, |q|², |x|² each in the lane layout.  SCALAR
 * (DefaultVectorUtilSupport.cosine): 4 accumulators per sum over a 4-aligned prefix when dim > 32,
 * then a fused scalar tail.  PANAMA512 (PanamaVectorUtilSupport.cosineBody): 2 accumulators per
 * sum, vector tail into the first, lane-wise add, reduceLanes, scalar fma tail. */
static void cos_parts(const float* a, const float* b, int dim, int order, float* sum, float* n1,
                      float* n2) {
    if (order == ORDER_DEVICE) {
        *sum = device_sum(a, b, dim, 0);
        *n1 = device_sum(a, a, dim, 0);
        *n2 = device_sum(b, b, dim, 0);
        return;
    }
    float s = 0.0f, x = 0.0f, y = 0.0f;
    int i = 0;
    const int fused = order == ORDER_SCALAR || order == ORDER_PANAMA512;
    if (order == ORDER_SCALAR || order == ORDER_SCALAR_NOFMA) {
        if (dim > 32) {
            float as[4] = {0}, ax[4] = {0}, ay[4] = {0};
            const int ub = dim & ~3;
            for (; i < ub; i += 4)
                for (int e = 0; e < 4; ++e) {
                    as[e] = mac(a[i + e], b[i + e], as[e], fused);
                    ax[e] = mac(a[i + e], a[i + e], ax[e], fused);
                    ay[e] = mac(b[i + e], b[i + e], ay[e], fused);
                }
            s += ((as[0] + as[1]) + as[2]) + as[3];
            x += ((ax[0] + ax[1]) + ax[2]) + ax[3];
            y += ((ay[0] + ay[1]) + ay[2]) + ay[3];
        }
    } else {
        const int S = 16;
        if (dim > 2 * S) {
            const int limit = dim - dim % S;
            float vs[2][16], vx[2][16], vy[2][16];
            memset(vs, 0, sizeof(vs)); memset(vx, 0, sizeof(vx)); memset(vy, 0, sizeof(vy));
            const int unrolled = limit - S;
            for (; i < unrolled; i += 2 * S)
                for (int u = 0; u < 2; ++u)
                    for (int l = 0; l < S; ++l) {
                        const int ix = i + u * S + l;
                        vs[u][l] = mac(a[ix], b[ix], vs[u][l], fused);
                        vx[u][l] = mac(a[ix], a[ix], vx[u][l], fused);
                        vy[u][l] = mac(b[ix], b[ix], vy[u][l], fused);
                    }
            for (; i < limit; i += S)
                for (int l = 0; l < S; ++l) {
                    const int ix = i + l;
                    vs[0][l] = mac(a[ix], b[ix], vs[0][l], fused);
                    vx[0][l] = mac(a[ix], a[ix], vx[0][l], fused);
                    vy[0][l] = mac(b[ix], b[ix], vy[0][l], fused);
                }
            float rs = 0.0f, rx = 0.0f, ry = 0.0f;
            for (int l = 0; l < S; ++l) {
                rs += vs[0][l] + vs[1][l];
                rx += vx[0][l] + vx[1][l];
                ry += vy[0][l] + vy[1][l];
            }
            s = rs; x = rx; y = ry;
        }
    }
    for (; i < dim; ++i) {
        s = mac(a[i], b[i], s, fused);
        x = mac(a[i], a[i], x, fused);
        y = mac(b[i], b[i], y, fused);
    }
    *sum = s; *n1 = x; *n2 = y;
}

static float java_max0(float v) { return v >= 0.0f ? v : (v != v ? v : 0.0f); }
static float mip(float dot) { return dot < 0.0f ? 1.0f / (1.0f + -1.0f * dot) : dot + 1.0f; }

/* [L] VectorSimilarityFunction.compare(float[], float[]) */
float orc_score_f32(const float* q, const float* x, int dim, int sim, int order) {
    switch (sim) {
        case SIM_EUCLIDEAN: return 1.0f / (1.0f + fsum(q, x, dim, 1, order));
        case SIM_DOT_PRODUCT: return java_max0((1.0f + fsum(q, x, dim, 0, order)) / 2.0f);
        case SIM_COSINE: {
            float dot, n1, n2;
            cos_parts(q, x, dim, order, &dot, &n1, &n2);
            const float c = (float)((double)dot / sqrt((double)n1 * (double)n2));
            return java_max0((1.0f + c) / 2.0f);
        }
        default: return mip(fsum(q, x, dim, 0, order));
    }
}

/* [L] VectorSimilarityFunction.compare(byte[], byte[]) — exact int32 sums */
float orc_score_i8(const int8_t* q, const int8_t* x, int dim, int sim) {
    int32_t dot = 0, n1 = 0, n2 = 0, d2 = 0;
    for (int i = 0; i < dim; ++i) {
        dot += (int32_t)q[i] * x[i];
        n1 += (int32_t)q[i] * q[i];
        n2 += (int32_t)x[i] * x[i];
        const int32_t d = (int32_t)q[i] - x[i];
        d2 += d * d;
    }
    switch (sim) {
        case SIM_EUCLIDEAN: return 1.0f / (1.0f + (float)d2);
        case SIM_DOT_PRODUCT: return 0.5f + (float)dot / (float)(dim * (1 << 15));
        case SIM_COSINE: {
            const float c = (float)((double)dot / sqrt((double)n1 * (double)n2));
            return (1.0f + c) / 2.0f;
        }
        default: return mip((float)dot);
    }
}

/* ------------------------------------------------------------------------------------------ */
/* [L] HitQueue + exactSearch                                                                  */
/* ------------------------------------------------------------------------------------------ */
typedef struct { float score; int32_t doc; } Hit;

/* HitQueue.lessThan: equal scores → the higher doc is "less" */
static int less_than(Hit a, Hit b) { return a.score == b.score ? a.doc > b.doc : a.score < b.score; }

static void sift_down(Hit* h, int n, int i) {
    for (;;) {
        int l = 2 * i + 1, r = l + 1, m = i;
        if (l < n && less_than(h[l], h[m])) m = l;
        if (r < n && less_than(h[r], h[m])) m = r;
        if (m == i) return;
        Hit t = h[i]; h[i] = h[m]; h[m] = t;
        i = m;
    }
}

static int heap_finish(Hit* heap, int k, float* out_scores, int32_t* out_docs) {
    /* drop sentinels (score < 0 never happens for real hits: every score is >= 0) then pop */
    int n = k;
    Hit* tmp = (Hit*)malloc(sizeof(Hit) * (k > 0 ? k : 1));
    int cnt = 0;
    while (n > 0) {
        Hit top = heap[0];
        heap[0] = heap[n - 1];
        --n;
        sift_down(heap, n, 0);
        if (!(top.score < 0.0f)) tmp[cnt++] = top;
    }
    /* popped in ascending order → write from the end */
    for (int i = 0; i < cnt; ++i) {
        out_scores[i] = tmp[cnt - 1 - i].score;
        out_docs[i] = tmp[cnt - 1 - i].doc;
    }
    free(tmp);
    return cnt;
}

static int accepted(const uint64_t* bits, int32_t doc) {
    return bits == NULL || ((bits[doc >> 6] >> (doc & 63)) & 1ull);
}

/* rows: n × dim row-major; ord_to_doc NULL = dense; accept NULL = all. Returns hit count. */
int orc_exact_search_f32(const float* rows, int64_t n, int dim, const int32_t* ord_to_doc,
                         const uint64_t* accept, const float* q, int k, int sim, int order,
                         float* out_scores, int32_t* out_docs, int64_t* visited) {
    Hit* heap = (Hit*)malloc(sizeof(Hit) * k);
    for (int i = 0; i < k; ++i) { heap[i].score = -INFINITY; heap[i].doc = 0x7FFFFFFF; }
    int64_t vis = 0;
    for (int64_t o = 0; o < n; ++o) {
        const int32_t doc = ord_to_doc ? ord_to_doc[o] : (int32_t)o;
        if (!accepted(accept, doc)) continue;
        ++vis;
        const float s = orc_score_f32(q, rows + o * dim, dim, sim, order);
        if (s > heap[0].score) {
            heap[0].score = s;
            heap[0].doc = doc;
            sift_down(heap, k, 0);
        }
    }
    if (visited) *visited = vis;
    const int c = heap_finish(heap, k, out_scores, out_docs);
    free(heap);
    return c;
}

int orc_exact_search_i8(const int8_t* rows, int64_t n, int dim, const int32_t* ord_to_doc,
                        const uint64_t* accept, const int8_t* q, int k, int sim, float* out_scores,
                        int32_t* out_docs, int64_t* visited) {
    Hit* heap = (Hit*)malloc(sizeof(Hit) * k);
    for (int i = 0; i < k; ++i) { heap[i].score = -INFINITY; heap[i].doc = 0x7FFFFFFF; }
    int64_t vis = 0;
    for (int64_t o = 0; o < n; ++o) {
        const int32_t doc = ord_to_doc ? ord_to_doc[o] : (int32_t)o;
        if (!accepted(accept, doc)) continue;
        ++vis;
        const float s = orc_score_i8(q, rows + o * dim, dim, sim);
        if (s > heap[0].score) {
            heap[0].score = s;
            heap[0].doc = doc;
            sift_down(heap, k, 0);
        }
    }
    if (visited) *visited = vis;
    const int c = heap_finish(heap, k, out_scores, out_docs);
    free(heap);
    return c;
}

/* ------------------------------------------------------------------------------------------ */
/* [L] TopDocs.merge(start, size, shardHits) with shardIndex set + TopDocsStats               */
/* ------------------------------------------------------------------------------------------ */
typedef struct { float score; int32_t shard; int32_t doc; } SHit;

static int merge_cmp(const void* pa, const void* pb) {
    const SHit* a = (const SHit*)pa;
    const SHit* b = (const SHit*)pb;
    if (a->score != b->score) return a->score > b->score ? -1 : 1;
    if (a->shard != b->shard) return a->shard < b->shard ? -1 : 1;
    if (a->doc != b->doc) return a->doc < b->doc ? -1 : 1;
    return 0;
}

/* shard s: counts[s] hits at scores/docs + s*stride.  Each shard contributes min(count, from+size)
 * (what its top-docs collector returned).  Returns merged count. */
int orc_topdocs_merge(int n_shards, const int32_t* counts, const float* scores, const int32_t* docs,
                      int stride, const int32_t* shard_index, int from, int size, float* out_scores,
                      int32_t* out_docs, int32_t* out_shard, int64_t* total_hits, float* max_score) {
    int64_t tot = 0;
    for (int s = 0; s < n_shards; ++s) tot += counts[s];
    SHit* all = (SHit*)malloc(sizeof(SHit) * (tot > 0 ? tot : 1));
    int n = 0;
    float mx = -INFINITY;
    for (int s = 0; s < n_shards; ++s) {
        const int take = counts[s] < from + size ? counts[s] : from + size;
        if (counts[s] > 0 && scores[(int64_t)s * stride] > mx) mx = scores[(int64_t)s * stride];
        for (int i = 0; i < take; ++i) {
            all[n].score = scores[(int64_t)s * stride + i];
            all[n].shard = shard_index ? shard_index[s] : s;
            all[n].doc = docs[(int64_t)s * stride + i];
            ++n;
        }
    }
    qsort(all, n, sizeof(SHit), merge_cmp);
    int got = n - from;
    if (got < 0) got = 0;
    if (got > size) got = size;
    for (int r = 0; r < got; ++r) {
        out_scores[r] = all[from + r].score;
        out_docs[r] = all[from + r].doc;
        out_shard[r] = all[from + r].shard;
    }
    *total_hits = tot;
    *max_score = isinf(mx) ? NAN : mx;
    free(all);
    return got;
}

/* ------------------------------------------------------------------------------------------ */
/* CPU baseline driver: the Lucene-equivalent restatement over row slices on `nthreads` threads */
/* (one exact search per slice, like concurrent segment search slices —                        */
/* S/search/internal/MaxTargetSliceSupplier.java:28-77 — then the per-leaf TopDocs.merge).     */
/* ------------------------------------------------------------------------------------------ */
#include <pthread.h>

typedef struct {
    const float* rows; int64_t begin, end; int dim;
    const float* queries; int nq; int k; int sim; int order;
    float* scores; int32_t* docs; int32_t* counts;   /* [nq][k] for this slice */
} SliceJob;

static void* slice_run(void* arg) {
    SliceJob* j = (SliceJob*)arg;
    for (int q = 0; q < j->nq; ++q) {
        int c = orc_exact_search_f32(j->rows + j->begin * j->dim, j->end - j->begin, j->dim, NULL, NULL,
                                     j->queries + (int64_t)q * j->dim, j->k, j->sim, j->order,
                                     j->scores + (int64_t)q * j->k, j->docs + (int64_t)q * j->k, NULL);
        for (int i = 0; i < c; ++i) j->docs[(int64_t)q * j->k + i] += (int32_t)j->begin;
        j->counts[q] = c;
    }
    return NULL;
}

int orc_knn_batch_f32(const float* rows, int64_t n, int dim, const float* queries, int nq, int k,
                      int sim, int order, int nthreads, float* out_scores, int32_t* out_docs,
                      int32_t* out_counts) {
    if (nthreads < 1) nthreads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
    SliceJob* jobs = (SliceJob*)calloc(nthreads, sizeof(SliceJob));
    float* sc = (float*)malloc(sizeof(float) * (size_t)nthreads * nq * k);
    int32_t* dc = (int32_t*)malloc(sizeof(int32_t) * (size_t)nthreads * nq * k);
    int32_t* cc = (int32_t*)malloc(sizeof(int32_t) * (size_t)nthreads * nq);
    for (int t = 0; t < nthreads; ++t) {
        SliceJob* j = &jobs[t];
        j->rows = rows; j->dim = dim; j->queries = queries; j->nq = nq; j->k = k; j->sim = sim;
        j->order = order;
        j->begin = n * t / nthreads; j->end = n * (t + 1) / nthreads;
        j->scores = sc + (size_t)t * nq * k; j->docs = dc + (size_t)t * nq * k; j->counts = cc + (size_t)t * nq;
        pthread_create(&th[t], NULL, slice_run, j);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    /* per-leaf merge: score desc, doc asc (docs are distinct, shard index constant) */
    float* tmp_s = (float*)malloc(sizeof(float) * (size_t)nthreads * k);
    int32_t* tmp_d = (int32_t*)malloc(sizeof(int32_t) * (size_t)nthreads * k);
    int32_t* tmp_c = (int32_t*)malloc(sizeof(int32_t) * nthreads);
    int32_t* tmp_sh = (int32_t*)malloc(sizeof(int32_t) * k);
    int32_t* zero_idx = (int32_t*)calloc(nthreads, sizeof(int32_t));
    for (int q = 0; q < nq; ++q) {
        for (int t = 0; t < nthreads; ++t) {
            memcpy(tmp_s + (size_t)t * k, sc + ((size_t)t * nq + q) * k, sizeof(float) * k);
            memcpy(tmp_d + (size_t)t * k, dc + ((size_t)t * nq + q) * k, sizeof(int32_t) * k);
            tmp_c[t] = cc[(size_t)t * nq + q];
        }
        int64_t tot; float mx;
        out_counts[q] = orc_topdocs_merge(nthreads, tmp_c, tmp_s, tmp_d, k, zero_idx, 0, k,
                                          out_scores + (size_t)q * k, out_docs + (size_t)q * k, tmp_sh,
                                          &tot, &mx);
    }
    free(th); free(jobs); free(sc); free(dc); free(cc); free(tmp_s); free(tmp_d); free(tmp_c);
    free(tmp_sh); free(zero_idx);
    return 0;
}
