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

// ------------------------------------------------------------------------------------------------
// Shard-result wire format: S/common/lucene/Lucene.java:407-447 (writeTopDocs, type 0 = plain
// TopDocs, what a k-NN DocAndScoreQuery's TopScoreDocCollector yields) and :314-357 (readTopDocs),
// with the StreamOutput / StreamInput encodings of libs/core/.../io/stream/StreamOutput.java
// (writeInt :247-254 big-endian, writeVInt :262-285, writeVLong :308-337, writeFloat :480-482 =
// writeInt(Float.floatToIntBits)) and StreamInput.java (readVInt :218-244, readVLong :267-319,
// readEnum :1280-1290).
// ------------------------------------------------------------------------------------------------
}  // extern "C"

namespace {

struct WireOut {
    uint8_t* p;
    int64_t cap, n = 0;
    void byte(uint8_t b) {
        if (p && n < cap) p[n] = b;
        ++n;
    }
    void i32(uint32_t v) {   // writeInt: big-endian
        byte((uint8_t)(v >> 24)); byte((uint8_t)(v >> 16)); byte((uint8_t)(v >> 8)); byte((uint8_t)v);
    }
    void vint(int32_t i) {   // writeVInt: 7-bit groups, low first; negatives take 5 bytes
        uint32_t u = (uint32_t)i;
        while (u & ~0x7Fu) { byte((uint8_t)((u & 0x7F) | 0x80)); u >>= 7; }
        byte((uint8_t)u);
    }
    void vlong(int64_t i) {
        uint64_t u = (uint64_t)i;
        while (u & ~0x7Full) { byte((uint8_t)((u & 0x7F) | 0x80)); u >>= 7; }
        byte((uint8_t)u);
    }
    void f32(float f) {      // Float.floatToIntBits: every NaN → 0x7fc00000
        uint32_t u;
        std::memcpy(&u, &f, 4);
        if (std::isnan(f)) u = 0x7fc00000u;
        i32(u);
    }
};

std::string hex32(uint32_t v) {   // Integer.toHexString
    char b[16];
    std::snprintf(b, sizeof b, "%x", v);
    return b;
}

struct WireIn {
    const uint8_t* p;
    int64_t len, pos = 0;
    std::string err;
    bool byte(int8_t& b) {
        if (pos >= len) { err = "EOF: tried to read past the end of the stream"; return false; }
        b = (int8_t)p[pos++];
        return true;
    }
    bool i32(uint32_t& v) {
        v = 0;
        for (int i = 0; i < 4; ++i) {
            int8_t b;
            if (!byte(b)) return false;
            v = (v << 8) | (uint8_t)b;
        }
        return true;
    }
    bool vint(int32_t& out) {   // StreamInput.readVInt: at most 5 bytes, the 5th without a continuation bit
        uint32_t i = 0;
        for (int sh = 0; sh < 28; sh += 7) {
            int8_t b;
            if (!byte(b)) return false;
            i |= (uint32_t)(b & 0x7F) << sh;
            if ((b & 0x80) == 0) { out = (int32_t)i; return true; }
        }
        int8_t b;
        if (!byte(b)) return false;
        if (b & 0x80) {
            err = "Invalid vInt ((" + hex32((uint32_t)(int32_t)b) + " & 0x7f) << 28) | " + hex32(i);
            return false;
        }
        out = (int32_t)(i | ((uint32_t)(b & 0x7F) << 28));
        return true;
    }
    bool vlong(int64_t& out) {  // StreamInput.readVLong: 9 groups of 7 bits, then a 0/1 sign byte
        uint64_t i = 0;
        for (int sh = 0; sh < 63; sh += 7) {
            int8_t b;
            if (!byte(b)) return false;
            i |= (uint64_t)(b & 0x7F) << sh;
            if ((b & 0x80) == 0) { out = (int64_t)i; return true; }
        }
        int8_t b;
        if (!byte(b)) return false;
        if (b != 0 && b != 1) {
            char h[32];
            std::snprintf(h, sizeof h, "%llx", (unsigned long long)i);
            err = "Invalid vlong (" + hex32((uint32_t)(int32_t)b) + " << 63) | " + h;
            return false;
        }
        out = (int64_t)(i | ((uint64_t)b << 63));
        return true;
    }
    bool f32(float& f) {
        uint32_t u;
        if (!i32(u)) return false;
        std::memcpy(&f, &u, 4);
        return true;
    }
};

}  // namespace

extern "C" {

int32_t osk_topdocs_write(int64_t total_hits, int32_t relation, float max_score, int32_t n,
                          const int32_t* docs, const float* scores, uint8_t* out, int64_t cap,
                          int64_t* out_len) {
    clear_error();
    if (!out_len || n < 0 || (n > 0 && (!docs || !scores)) || cap < 0 || (cap > 0 && !out)) {
        set_error("osk_topdocs_write: bad argument");
        return OSK_ERR_INVALID;
    }
    if (total_hits < 0) {   // StreamOutput.writeVLong :308-313
        set_error("Negative longs unsupported, use writeLong or writeZLong for negative numbers [" +
                  std::to_string(total_hits) + "]");
        return OSK_ERR_INVALID;
    }
    if (relation != 0 && relation != 1) {   // TotalHits.Relation {EQUAL_TO, GREATER_THAN_OR_EQUAL_TO}
        set_error("osk_topdocs_write: relation must be 0 (EQUAL_TO) or 1 (GREATER_THAN_OR_EQUAL_TO)");
        return OSK_ERR_INVALID;
    }
    WireOut w{out, cap};
    w.byte(0);                 // plain TopDocs
    w.vlong(total_hits);       // writeTotalHits (:402-405)
    w.vint(relation);          // writeEnum = writeVInt(ordinal)
    w.f32(max_score);
    w.vint(n);
    for (int32_t i = 0; i < n; ++i) {   // writeScoreDoc (:525-531)
        w.vint(docs[i]);
        w.f32(scores[i]);
    }
    *out_len = w.n;
    if (out && w.n > cap) {
        set_error("osk_topdocs_write: output buffer too small (need " + std::to_string(w.n) + " bytes)");
        return OSK_ERR_INVALID;
    }
    return OSK_OK;
}

int32_t osk_topdocs_read(const uint8_t* buf, int64_t len, int64_t* total_hits, int32_t* relation,
                         float* max_score, int32_t cap_hits, int32_t* n, int32_t* docs, float* scores,
                         int64_t* consumed) {
    clear_error();
    if ((!buf && len > 0) || len < 0 || !total_hits || !relation || !max_score || !n || cap_hits < 0 ||
        (cap_hits > 0 && (!docs || !scores))) {
        set_error("osk_topdocs_read: bad argument");
        return OSK_ERR_INVALID;
    }
    WireIn r{buf, len};
    int8_t type;
    int32_t rel, cnt;
    int64_t total;
    float mx;
    if (!r.byte(type)) { set_error(r.err); return OSK_ERR_INVALID; }
    if (type == 1 || type == 2) {   // TopFieldDocs / CollapseTopFieldDocs: never a k-NN shard result
        set_error("osk_topdocs_read: TopDocs type " + std::to_string(type) + " (field docs) is not produced by the k-NN path");
        return OSK_ERR_UNSUPPORTED;
    }
    if (type != 0) {
        set_error("Unknown type " + std::to_string(type));
        return OSK_ERR_INVALID;
    }
    if (!r.vlong(total) || !r.vint(rel) || (rel >= 0 && rel <= 1 && (!r.f32(mx) || !r.vint(cnt)))) {
        set_error(r.err);
        return OSK_ERR_INVALID;
    }
    if (rel < 0 || rel > 1) {
        set_error("Unknown Relation ordinal [" + std::to_string(rel) + "]");
        return OSK_ERR_INVALID;
    }
    if (cnt < 0) {
        set_error("Negative array size: " + std::to_string(cnt));
        return OSK_ERR_INVALID;
    }
    if (cnt > cap_hits) {
        set_error("osk_topdocs_read: " + std::to_string(cnt) + " hits exceed the output capacity " +
                  std::to_string(cap_hits));
        return OSK_ERR_INVALID;
    }
    for (int32_t i = 0; i < cnt; ++i) {
        if (!r.vint(docs[i]) || !r.f32(scores[i])) {
            set_error(r.err);
            return OSK_ERR_INVALID;
        }
    }
    *total_hits = total;
    *relation = rel;
    *max_score = mx;
    *n = cnt;
    if (consumed) *consumed = r.pos;
    return OSK_OK;
}

}  // extern "C"
