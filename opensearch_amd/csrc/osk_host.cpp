// osk_host.cpp — the host-only part of libosknn: error state, the synthetic generator's host
// twin, key decoding and the coordinator reduce over host arrays.  Nothing here touches a device,
// so these entry points also work (and are unit-tested) on a machine without a GPU.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "../../include/osknn.h"
#include "osk_common.h"

namespace osk {
static thread_local std::string t_err;
void set_error(const std::string& msg) { t_err = msg; }
void clear_error() { t_err.clear(); }
}  // namespace osk

using namespace osk;

extern "C" {

const char* osk_last_error(void) { return t_err.c_str(); }

int32_t osk_synth_host(void* out, int64_t row0, int64_t n_rows, int32_t dim, uint64_t seed,
                       int32_t dist) {
    try {
        if (!out || n_rows < 0 || dim < 1 || dist < 0 || dist > 4) {
            set_error("osk_synth_host: bad argument");
            return OSK_ERR_INVALID;
        }
        const uint64_t mix = splitmix64(seed);
        for (int64_t r = 0; r < n_rows; ++r) {
            const uint64_t grow = (uint64_t)(row0 + r);
            if (dist == DIST_INT8) {
                int8_t* o = static_cast<int8_t*>(out) + r * (int64_t)dim;
                for (int c = 0; c < dim; ++c) o[c] = synth_i8(synth_bits(mix, grow, dim, c));
                continue;
            }
            float* o = static_cast<float*>(out) + r * (int64_t)dim;
            for (int c = 0; c < dim; ++c) o[c] = synth_f32_raw(dist, synth_bits(mix, grow, dim, c));
            if (dist == DIST_NORMALISH_UNIT) {
                float part[64];
                for (int l = 0; l < 64; ++l) {
                    float acc = 0.0f;
                    for (int c = l; c < dim; c += 64) acc = std::fmaf(o[c], o[c], acc);
                    part[l] = acc;
                }
                const float den = std::sqrt(synth_row_norm2_lanes(part));
                for (int c = 0; c < dim; ++c) o[c] = o[c] / den;
            }
        }
        return OSK_OK;
    } catch (...) {
        set_error("osk_synth_host: exception");
        return OSK_ERR_INVALID;
    }
}

int32_t osk_decode_keys(const uint64_t* keys, int64_t n, float* scores, int32_t* docs) {
    if (!keys || n < 0 || !scores || !docs) {
        set_error("osk_decode_keys: bad argument");
        return OSK_ERR_INVALID;
    }
    for (int64_t i = 0; i < n; ++i) {
        if (keys[i] == 0) {
            scores[i] = -std::numeric_limits<float>::infinity();
            docs[i] = 0x7FFFFFFF;
        } else {
            scores[i] = key_score(keys[i]);
            docs[i] = key_doc(keys[i]);
        }
    }
    return OSK_OK;
}

// [L] TopDocs.merge(start=from, size, shardHits) as called from
// S/action/search/SearchPhaseController.java:224-246 with every ScoreDoc's shardIndex set
// (:248-253).  Order: score desc, then shardIndex asc, then doc asc ([L] TopDocs.DEFAULT_TIE_BREAKER).
// Each shard contributes its first min(count, from+size) hits — what the shard's top-docs collector
// returned (S/search/query/TopDocsCollectorContext.java:866 numDocs = min(from+size, …)).
// Stats follow TopDocsStats (:839-901): total = Σ shard hits, maxScore = max shard top score,
// NaN when there is none.
int32_t osk_topdocs_merge(int32_t n_shards, const int32_t* shard_counts, const float* shard_scores,
                          const int32_t* shard_docs, int32_t stride, const int32_t* shard_index,
                          const int32_t* hit_shard_index, int32_t from, int32_t size, float* out_scores, int32_t* out_docs,
                          int32_t* out_shard_index, int32_t* out_count, int64_t* out_total_hits,
                          float* out_max_score) {
    try {
        if (n_shards < 0 || (n_shards > 0 && (!shard_counts || !shard_scores || !shard_docs)) ||
            from < 0 || size < 0 || !out_count || !out_total_hits || !out_max_score ||
            (size > 0 && (!out_scores || !out_docs || !out_shard_index))) {
            set_error("osk_topdocs_merge: bad argument");
            return OSK_ERR_INVALID;
        }
        struct Hit {
            float score;
            int32_t shard;
            int32_t doc;
        };
        std::vector<Hit> hits;
        int64_t total = 0;
        float max_score = -std::numeric_limits<float>::infinity();
        const int64_t topn = (int64_t)from + size;
        for (int s = 0; s < n_shards; ++s) {
            const int c = shard_counts[s];
            if (c < 0 || c > stride) {
                set_error("osk_topdocs_merge: shard count out of range");
                return OSK_ERR_INVALID;
            }
            total += c;
            const int32_t si0 = shard_index ? shard_index[s] : s;
            if (c > 0 && !std::isnan(shard_scores[(int64_t)s * stride]))
                max_score = std::max(max_score, shard_scores[(int64_t)s * stride]);
            const int64_t take = std::min<int64_t>(c, topn);
            for (int64_t i = 0; i < take; ++i)
                hits.push_back(Hit{shard_scores[(int64_t)s * stride + i],
                                   hit_shard_index ? hit_shard_index[(int64_t)s * stride + i] : si0,
                                   shard_docs[(int64_t)s * stride + i]});
        }
        std::stable_sort(hits.begin(), hits.end(), [](const Hit& a, const Hit& b) {
            if (a.score != b.score) return a.score > b.score;
            if (a.shard != b.shard) return a.shard < b.shard;
            return a.doc < b.doc;
        });
        const int64_t got = std::max<int64_t>(0, std::min<int64_t>(size, (int64_t)hits.size() - from));
        for (int64_t r = 0; r < size; ++r) {
            if (r < got) {
                const Hit& h = hits[from + r];
                out_scores[r] = h.score;
                out_docs[r] = h.doc;
                out_shard_index[r] = h.shard;
            } else {
                out_scores[r] = -std::numeric_limits<float>::infinity();
                out_docs[r] = 0x7FFFFFFF;
                out_shard_index[r] = -1;
            }
        }
        *out_count = (int32_t)got;
        *out_total_hits = total;
        *out_max_score = std::isinf(max_score) ? std::numeric_limits<float>::quiet_NaN() : max_score;
        return OSK_OK;
    } catch (...) {
        set_error("osk_topdocs_merge: exception");
        return OSK_ERR_INVALID;
    }
}

}  // extern "C"
