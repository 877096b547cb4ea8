// osk_common.h — definitions shared by the device kernels and the host side of libosknn.
//
// Everything here is arithmetic that must be identical on host and device:
//   * the hit key (score, doc) → uint64 encoding that orders hits exactly like Lucene's
//     exact search / TopKnnCollector (score desc, ties → lower doc);
//   * Lucene's VectorSimilarityFunction score transforms [L];
//   * the fixed per-dimension lane layout that defines the fp32 summation order;
//   * the counter-based synthetic corpus generator used by bench.py and the tests.
#pragma once
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define OSK_HD __host__ __device__ __forceinline__
#else
#define OSK_HD static inline
#endif

namespace osk {

// ---------------------------------------------------------------------------------------------
// Hit keys.  A hit is (float score, int32 doc).  Lucene keeps the top k of a leaf by score and,
// on equal score, the LOWER doc (exact search offers scores in doc order to a HitQueue with a
// strict '>' test; TopKnnCollector/NeighborQueue encode the node as ~node in the low bits).
// key = (sortable(score) << 32) | (0xFFFFFFFF - doc): a larger key is a better hit, so one
// unsigned 64-bit compare reproduces that total order.  Key 0 is the empty slot (no real hit
// can produce it: every Lucene similarity score is >= 0, whose sortable form is >= 2^31).
// ---------------------------------------------------------------------------------------------
OSK_HD uint32_t float_to_sortable(float s) {
    uint32_t u;
    __builtin_memcpy(&u, &s, 4);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
OSK_HD float sortable_to_float(uint32_t u) {
    uint32_t b = (u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u;
    float s;
    __builtin_memcpy(&s, &b, 4);
    return s;
}
// A NaN score is never a hit: [L] exactSearch collects a doc only when `score > topDoc.score` (the HitQueue
// starts full of −∞ sentinels), false for NaN — a COSINE zero vector (query or row) scores NaN and is visited but
// never collected.  Its key is the empty slot; the same holds for a NaN bound (COSINE: NaN exactly when the exact
// score is), so such a row is never a candidate either.
OSK_HD uint64_t make_key(float score, uint32_t doc) {
    if (score != score) return 0ull;
    return ((uint64_t)float_to_sortable(score) << 32) | (uint64_t)(0xFFFFFFFFu - doc);
}
OSK_HD float key_score(uint64_t key) { return sortable_to_float((uint32_t)(key >> 32)); }
OSK_HD int32_t key_doc(uint64_t key) { return (int32_t)(0xFFFFFFFFu - (uint32_t)key); }

// ---------------------------------------------------------------------------------------------
// [L] VectorSimilarityFunction.compare score transforms (lucene-core 10.3.0), written with the
// same float/double operations Java performs.  Similarity ordinals follow the Lucene enum.
//   EUCLIDEAN              1 / (1 + d²)                      (VectorUtil.normalizeDistanceToUnitInterval)
//   DOT_PRODUCT (float)    max((1 + dot) / 2, 0)             (VectorUtil.normalizeToUnitInterval)
//   COSINE (float)         max((1 + cos) / 2, 0), cos = (float)(dot / sqrt((double)|q|²·(double)|x|²))
//   MAXIMUM_INNER_PRODUCT  dot < 0 ? 1 / (1 + -1·dot) : dot + 1   (VectorUtil.scaleMaxInnerProductScore)
//   byte EUCLIDEAN         1 / (1f + (float)d²_int)
//   byte DOT_PRODUCT       0.5f + (float)dot_int / (float)(dim · 2^15)   (VectorUtil.dotProductScore)
//   byte COSINE            (1 + cos) / 2, cos from int sums as above (no max)
//   byte MAX_INNER_PRODUCT scaleMaxInnerProductScore((float)dot_int)
// ---------------------------------------------------------------------------------------------
enum { SIM_EUCLIDEAN = 0, SIM_DOT_PRODUCT = 1, SIM_COSINE = 2, SIM_MIP = 3 };
enum { ENC_FLOAT32 = 0, ENC_BYTE = 1 };

OSK_HD float java_max0(float v) { return v >= 0.0f ? v : (v != v ? v : 0.0f); }
OSK_HD float mip_scale(float dot) { return dot < 0.0f ? 1.0f / (1.0f + -1.0f * dot) : dot + 1.0f; }

OSK_HD float score_f32_l2(float d2) { return 1.0f / (1.0f + d2); }
OSK_HD float score_f32_dot(float dot) { return java_max0((1.0f + dot) / 2.0f); }
OSK_HD float cosine_from(double dot, float n1, float n2) {
    return (float)(dot / sqrt((double)n1 * (double)n2));
}
OSK_HD float score_f32_cos(float dot, float qn, float xn) {
    return java_max0((1.0f + cosine_from((double)dot, qn, xn)) / 2.0f);
}
OSK_HD float score_f32(int sim, float s, float qn, float xn) {
    switch (sim) {
        case SIM_EUCLIDEAN: return score_f32_l2(s);
        case SIM_DOT_PRODUCT: return score_f32_dot(s);
        case SIM_COSINE: return score_f32_cos(s, qn, xn);
        default: return mip_scale(s);
    }
}
// byte: `s` is Σab (DOT/COS/MIP); for EUCLIDEAN the caller passes d² = |q|² + |x|² - 2Σab (exact).
OSK_HD float score_i8(int sim, int32_t s, int32_t qn, int32_t xn, int dim) {
    switch (sim) {
        case SIM_EUCLIDEAN: return 1.0f / (1.0f + (float)s);
        case SIM_DOT_PRODUCT: return 0.5f + (float)s / (float)(dim * (1 << 15));
        case SIM_COSINE: {
            float c = (float)((double)s / sqrt((double)qn * (double)xn));
            return (1.0f + c) / 2.0f;
        }
        default: return mip_scale((float)s);
    }
}

// ---------------------------------------------------------------------------------------------
// Lane layout (defines the fp32 summation order).  A row of n4 float4s
// (dim rounded up to a multiple of 4, zero padded) is scored by L lanes of a wavefront; lane t
// reads float4s t, t+L, …, t+(V-1)L (zero past n4) and keeps 4 fmaf chains (x,y,z,w); the lane
// partial is (x+y)+(z+w); the L partials are summed by a pairwise tree (xor butterfly).
// The layout depends only on dim — never on batch size — so a (query, row) score is the same
// bits whichever kernel or batch computes it.  For byte vectors the unit is a 16-byte chunk and
// the sums are exact int32 (order irrelevant).
// ---------------------------------------------------------------------------------------------
struct LaneCfg { int L; int V; };
OSK_HD LaneCfg lane_cfg(int units) {   // units = float4s (f32) or 16-byte chunks (int8) per row
    if (units <= 8) return {4, 2};
    if (units <= 16) return {8, 2};
    if (units <= 32) return {8, 4};
    if (units <= 64) return {16, 4};
    if (units <= 128) return {16, 8};
    if (units <= 192) return {16, 12};
    if (units <= 256) return {32, 8};
    if (units <= 512) return {64, 8};
    return {64, 16};   // up to 1024 units (dim 4096 f32)
}

// ---------------------------------------------------------------------------------------------
// Synthetic corpus: a counter-based generator, identical on host and device (no libm
// transcendental; only IEEE add/mul/fma/div/sqrt, all correctly rounded on both sides).
// ---------------------------------------------------------------------------------------------
enum { DIST_UNIFORM01 = 0, DIST_UNIFORM01_X128 = 1, DIST_NORMALISH = 2, DIST_NORMALISH_UNIT = 3,
       DIST_INT8 = 4 };

OSK_HD uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
OSK_HD uint64_t synth_bits(uint64_t seed_mix, uint64_t row, int dim, int col) {
    return splitmix64(seed_mix + row * (uint64_t)dim + (uint64_t)col);
}
OSK_HD float synth_f32_raw(int dist, uint64_t h) {
    if (dist == DIST_UNIFORM01) return (float)(h >> 40) * 0x1p-24f;
    if (dist == DIST_UNIFORM01_X128) return ((float)(h >> 40) * 0x1p-24f) * 128.0f;
    uint32_t s = (uint32_t)(h & 0xFFFFu) + (uint32_t)((h >> 16) & 0xFFFFu) +
                 (uint32_t)((h >> 32) & 0xFFFFu) + (uint32_t)(h >> 48);
    return ((float)s * 0x1p-16f - 2.0f) * 1.7320508f;   // Irwin–Hall(4), unit variance
}
OSK_HD int8_t synth_i8(uint64_t h) { return (int8_t)(uint8_t)(h >> 56); }

// Row norm used by DIST_NORMALISH_UNIT: 64 lane partials (lane c: fmaf chain over columns
// c, c+64, …) summed by a pairwise tree; x = z / sqrt(norm2).
OSK_HD float synth_row_norm2_lanes(float* partial64) {
    for (int w = 32; w >= 1; w >>= 1)
        for (int i = 0; i < w; ++i) partial64[i] = partial64[i] + partial64[i + w];
    return partial64[0];
}

}  // namespace osk
