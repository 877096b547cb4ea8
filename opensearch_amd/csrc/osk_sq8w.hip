// osk_sq8w.hip — the certified int8 prefilter on MFMA for large batches: one corpus pass per 256 queries.
//
// sq8_mfma (osk_sq8.hip) takes 32 queries per launch, so a batch of B queries streams the int8 corpus
// B / 32 times: at 100M × 96 and B = 1024 that is 32 passes over 14 GB, 91 ms per batch.  A
// batched search is compute-light per byte — 96 int8 MACs per (row, query) — so the corpus is read once per
// 256 queries here:
//
//   * its own copy of each segment (launch_sq8w_build): int8 codes with ONE scale per 16-row group (the
//     group's max |x| / 127), in the MFMA-tiled layout (16-row blocks, 1 KiB slabs per 64 dims), and per
//     group the rows' bound terms with that scale plus the group's quick-test factor; KS = 2, 4, 8 or 12
//     slabs (≤ 128, 256, 512, 768 dims);
//   * persistent: one workgroup of 8 waves per CU takes every G-th (tile, quarter) of the tile order (tiles
//     interleaved over shards) as one continuous stream of steps (GPS groups of 16 rows) through an NS-deep
//     LDS-DMA ring (global_load_lds_dwordx4); a quarter is exactly one list of the settle
//     (sq8_settle_wide); one barrier per step;
//   * waves 0–3 load a step's int8 slabs (the tiled image is lane-linear: it IS the MFMA A operand), waves 4–7
//     its groups' bound terms; each wave owns 32 of the launch's 256 queries: B fragments in VGPRs for the
//     whole launch, 2 query blocks × KS v_mfma_i32_16x16x64_i8 per group, exact int32 dots;
//   * the quick test per group: every row of a group shares the scale s_g, so a lane's 4 rows pass the
//     per-row test I·s_g ≥ c iff their MAXIMUM dot does — one integer max, one convert and one fma per
//     (group, query block) and lane, then ONE wave vote per step (COSINE: the factor s_g / √(min |x|²)
//     bounds every row's s_g / √|x|²).  Only a step with a passing pair takes the slow path: per-row tests,
//     the precise bound in each passing pair's own lane and, above the floor, an append to its (quarter,
//     query) list by an LDS atomic; lists that would fill go through sq8_mfma's ordered insertion.  The
//     per-row test is relaxed to the quarter's row maxima (launch_wide_quarter_max) and is provably no
//     stricter than sq8_bounds' upper side (derivation at quick_consts);
//   * deferred insertions (main pass, when LDS allows: wide_qcap): the slow path only runs the per-row test
//     on the step's accumulators and appends each passing pair {int32 dot, row << 8 | query} to the wave's
//     LDS queue; the queue drains — precise bounds, floor check, list appends, 64 pairs per wave iteration —
//     at the quarter's end (or when full).  The step's barrier then waits for a short per-row test, not for
//     the slowest wave's bounds and atomics (C4 b256 9.0 → 7.5 ms, C3 b256 5.8 → 4.3 ms, profiles/r05d/);
//   * floors: pilot = 1 bounds each quarter's first step of rows (the best lower-bound key per query; their k-th
//     per (query, shard) floors the main pass); the main pass runs in two launches — 1/phase of the quarters
//     first, then the rest under floors raised to the k-th best list maximum of the first (launch_wide_floor;
//     the sq8_mfma pilot argument: k distinct rows score ≥ T, a row with ub < T cannot enter or tie into the
//     top k).
// Results are bit-identical to sq8_mfma's, the fp32 streaming scan's and the oracle's (tests/test_gpu_wide.py).
#include <hip/hip_ext.h>

#include <map>
#include <mutex>

#include "osk_device.h"
#include "osk_internal.h"
#include "osk_wave.h"

namespace osk {

// KS (64-dim slabs) of the wide kernel for a row of u8 16-byte int8 units: 2, 4, 8 or 12 (≤ 768 dims)
int sq8_wide_ks(int u8) { return u8 <= 8 ? 2 : u8 <= 16 ? 4 : u8 <= 32 ? 8 : 12; }
int sq8_wide_supported(int u8) { return u8 >= 1 && u8 <= 48 ? 1 : 0; }

// The wide kernel's copy of a segment (launch_sq8w_build), one wave per 16-row group: the group's scale
// s_g = max |x| over its rows / 127 (sq8_quantize's per-row formula over the group), codes
// q = clamp(rint(x / s_g), ±127) written in the MFMA-tiled layout (lane l of slab j: row l & 15, 16-B unit
// 4j + (l >> 4) — the lane-linear A operand), and the group's bound terms in the tiled struct-of-arrays layout
// of kAuxGroupF4 float4 (osk_internal.h): per row {s_g, s_g·|q| ↑, |x − s_g·q| ↑, |x|²} (sq8_quantize's terms,
// computed in double, ↑ = rounded up; COSINE stores each row's per-row quick-test factor s_g / √|x|² in place of
// s_g, which the kernel reads from the next-but-one slot), {max s|q|, max |δ|, max |x|², min |x|²}, {s_g, f_cos, zero-row flag, 0}
// and (COSINE) the rows' device-order |x|².  f_cos ≥ s_g / √|x|² of every row (rounded up, + 2^-20): the
// COSINE quick test's per-group factor; a group with a zero row (COSINE) sets the flag instead (its pairs
// always take the per-row test).  Rows past the last: zero codes and terms, not in the extrema.
__global__ __launch_bounds__(kBlock) void sq8w_build(const float4* __restrict__ X, int64_t n_rows, int units, int ks,
                                                     const float* __restrict__ xnorm, int cosine,
                                                     int4* __restrict__ codes, float4* __restrict__ auxt) {
    const int lane = threadIdx.x & 63, r = lane & 15, c = lane >> 4;
    const int64_t ng = (n_rows + 15) / 16;
    const int64_t wave_global = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) >> 6;
    for (int64_t g = wave_global; g < ng; g += n_waves) {
        const int64_t row = g * 16 + r;
        const bool valid = row < n_rows;
        const float4* xr = X + (valid ? row : 0) * (int64_t)units;
        float m = 0.0f;
        for (int j = 0; j < ks; ++j)
            for (int e = 0; e < 4; ++e) {
                const int f = (4 * j + c) * 4 + e;   // fp32 float4 unit
                if (valid && f < units) {
                    const float4 x = xr[f];
                    m = fmaxf(m, fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w))));
                }
            }
        for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
        const float sg = m / 127.0f;
        long long sq = 0;
        double se = 0.0, sx = 0.0;
        for (int j = 0; j < ks; ++j) {
            uint32_t w4[4];
            for (int e = 0; e < 4; ++e) {
                const int f = (4 * j + c) * 4 + e;
                uint32_t packed = 0u;
                if (valid && f < units) {
                    const float4 x = xr[f];
                    const float xs[4] = {x.x, x.y, x.z, x.w};
                    for (int t = 0; t < 4; ++t) {
                        int qi = 0;
                        if (sg > 0.0f) qi = (int)fminf(fmaxf(rintf(xs[t] / sg), -127.0f), 127.0f);
                        packed |= ((uint32_t)qi & 0xFFu) << (8 * t);
                        sq += (long long)(qi * qi);
                        const double rr = (double)xs[t] - (double)sg * (double)qi;   // exact in double
                        se += rr * rr;
                        sx += (double)xs[t] * (double)xs[t];
                    }
                }
                w4[e] = packed;
            }
            codes[(g * ks + j) * 64 + lane] = make_int4((int)w4[0], (int)w4[1], (int)w4[2], (int)w4[3]);
        }
        for (int o = 16; o <= 32; o <<= 1) {   // the row's 4 lanes (c = 0..3)
            sq += __shfl_xor(sq, o);
            se += __shfl_xor(se, o);
            sx += __shfl_xor(sx, o);
        }
        const float A = valid ? f32_round_up((double)sg * sqrt((double)sq) * (1.0 + 1e-12)) : 0.0f;
        const float B = valid ? f32_round_up(sqrt(se) * (1.0 + 1e-12)) : 0.0f;
        const float W = valid ? (float)sx : 0.0f;
        float mA = A, mB = B, mW = W, nW = valid ? W : __builtin_inff();
        for (int o = 1; o <= 8; o <<= 1) {
            mA = fmaxf(mA, __shfl_xor(mA, o));
            mB = fmaxf(mB, __shfl_xor(mB, o));
            mW = fmaxf(mW, __shfl_xor(mW, o));
            nW = fminf(nW, __shfl_xor(nW, o));
        }
        float* af = reinterpret_cast<float*>(auxt + g * kAuxGroupF4);
        if (c == 0) {
            // COSINE keeps each row's quick-test factor s_g / √|x|² here instead of s_g (which every valid row
            // shares: slot 17 holds it); round to nearest from double (a zero row: +∞, its pairs pass)
            af[r] = !valid ? 0.0f : !cosine ? sg : W > 0.0f ? (float)((double)sg / sqrt((double)W)) : __builtin_inff();
            af[16 + r] = A;
            af[32 + r] = B;
            af[48 + r] = W;
            af[72 + r] = (cosine && valid && xnorm) ? xnorm[row] : 0.0f;
        }
        if (lane == 0) {
            float fcos = 0.0f, zflag = 0.0f;
            if (cosine) {
                if (nW > 0.0f) fcos = f32_round_up((double)sg / sqrt((double)nW) * (1.0 + 0x1p-20));
                else zflag = 1.0f;
            }
            auxt[g * kAuxGroupF4 + 16] = make_float4(mA, mB, mW, nW);
            auxt[g * kAuxGroupF4 + 17] = make_float4(sg, fcos, zflag, 0.0f);
        }
    }
}

hipError_t launch_sq8w_build(const float4* rows, int64_t n_rows, int units, int u8, const float* xnorm, int cosine,
                             void* codes, float4* auxt, hipStream_t s) {
    if (n_rows <= 0) return hipMemsetAsync(auxt, 0, (size_t)kAuxGroupF4 * sizeof(float4), s);
    const int64_t ng = (n_rows + 15) / 16;
    const int64_t blocks = std::min<int64_t>(8192, (ng + 3) / 4);
    hipLaunchKernelGGL(sq8w_build, dim3((unsigned)blocks), dim3(kBlock), 0, s, rows, n_rows, units, sq8_wide_ks(u8),
                       xnorm, cosine, static_cast<int4*>(codes), auxt);
    return hipGetLastError();
}

// Per (tile, quarter): the maxima of its rows' bound terms over its 16-row groups (launch_wide_quarter_max).
// One workgroup per quarter, the quarter's geometry as sq8_wide's.
__global__ __launch_bounds__(kBlock) void wide_quarter_max(const TileDev* __restrict__ tiles,
                                                           const float4* const* __restrict__ auxt,
                                                           float4* __restrict__ out) {
    __shared__ float4 red[kBlock];
    const int j = blockIdx.x, tix = j >> 2, quarter = j & 3;
    const TileDev tile = tiles[tix];
    const int64_t trows = tile.row_end - tile.row_begin;
    const int64_t spw = ((trows + 4 * kMfmaScanR - 1) / (4 * kMfmaScanR)) * kMfmaScanR;
    const int64_t rb = min(tile.row_begin + quarter * spw, tile.row_end);
    const int64_t re = min(rb + spw, tile.row_end);
    const int64_t g0 = rb >> 4, g1 = (re + 15) >> 4;
    float4 m = make_float4(0.0f, 0.0f, 0.0f, __builtin_inff());
    for (int64_t g = g0 + threadIdx.x; g < g1; g += kBlock) {
        const float4 b = auxt[tile.seg][g * kAuxGroupF4 + 16];
        m = make_float4(fmaxf(m.x, b.x), fmaxf(m.y, b.y), fmaxf(m.z, b.z), fminf(m.w, b.w));
    }
    red[threadIdx.x] = m;
    __syncthreads();
    for (int o = kBlock / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            const float4 b = red[threadIdx.x + o];
            m = make_float4(fmaxf(m.x, b.x), fmaxf(m.y, b.y), fmaxf(m.z, b.z), fminf(m.w, b.w));
            red[threadIdx.x] = m;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) out[j] = m;
}

hipError_t launch_wide_quarter_max(const TileDev* tiles, int n_tiles, const float4* const* auxt, float4* out,
                                   hipStream_t s) {
    if (n_tiles < 1) return hipSuccess;
    hipLaunchKernelGGL(wide_quarter_max, dim3(4 * n_tiles), dim3(kBlock), 0, s, tiles, auxt, out);
    return hipGetLastError();
}

// The floors of launch_wide_floor (osk_internal.h): one workgroup per (shard, query), the k-th best of the
// shard's pilot keys (one per quarter: its first step's best lower-bound key) or of its lists' maxima, raised
// from a base floor.  A pilot key is one row's lower bound, and so is a list maximum (lists hold distinct
// rows): k quarters or lists with a value ≥ T are k distinct rows scoring ≥ T (the sq8_mfma pilot argument),
// so a row whose upper bound is below T cannot enter or tie into the shard's top k.
__global__ __launch_bounds__(kBlock) void wide_floor(const uint32_t* __restrict__ list_lbmax,
                                                     const uint64_t* __restrict__ pilot_keys, int n_lists,
                                                     const int32_t* __restrict__ shard_list_begin, int n_shards,
                                                     int k, const uint32_t* __restrict__ base,
                                                     uint32_t* __restrict__ floors) {
    __shared__ uint64_t lists[4 * 64];
    const int s = blockIdx.x, b = blockIdx.y;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const size_t o = (size_t)b * n_shards + s;
    uint32_t f = base ? base[o] : 0u;
    const int l0 = shard_list_begin[s], l1 = shard_list_begin[s + 1];
    uint64_t lk = 0ull, thr = 0ull;
    for (int i0 = l0 + wave * 64; i0 < l1; i0 += kBlock) {
        const int l = i0 + lane;
        uint64_t key = 0ull;
        if (pilot_keys) {
            key = l < l1 ? pilot_keys[(size_t)b * n_lists + l] : 0ull;   // (distinct: they carry the row)
        } else if (list_lbmax) {
            const uint32_t v = l < l1 ? list_lbmax[(size_t)b * n_lists + l] : 0u;
            key = v ? ((uint64_t)v << 32) | (uint32_t)(l + 1) : 0ull;
        }
        wave_offer(key, true, lk, thr, lane, k);
    }
    lists[wave * 64 + lane] = lane < k ? lk : 0ull;
    __syncthreads();
    if (wave != 0) return;
    block_fold(lists, lk, thr, lane, k);
    const uint64_t kth = readlane64(lk, k - 1);
    const uint32_t t = (uint32_t)(kth >> 32);
    if (kth && sortable_to_float(t) > 0.0f && t > f) f = t;
    if (threadIdx.x == 0) floors[o] = f;
}

hipError_t launch_wide_floor(const uint32_t* list_lbmax, const uint64_t* pilot_keys, int n_lists,
                             const int32_t* shard_list_begin, int n_shards, int nq, int k, const uint32_t* base,
                             uint32_t* floors, hipStream_t s) {
    if (n_shards < 1 || nq < 1 || k < 1 || k > 64) return hipErrorInvalidValue;
    hipLaunchKernelGGL(wide_floor, dim3(n_shards, nq), dim3(kBlock), 0, s, list_lbmax, pilot_keys, n_lists,
                       shard_list_begin, n_shards, k, base, floors);
    return hipGetLastError();
}

// The per-(step, query) constants of the quick test, from the step's row maxima bm = {max s·|q|, max |δ|,
// max |x|², min |x|²} (rows r of the step: a_r = s_x, w_r = |x|², y_r = s_x|q_x|, z_r = |δ_x|) and the
// query's terms (tq the list's quick threshold of sq8_quick, sb = s_b, inv its reciprocal (EUCLIDEAN: of 2s_b),
// QY/QZ/Q0 sq8_mfma's coefficients, zq = qc.z / s_b ≥ |q_b|, ig2m ≈ 1 / (1 − g2)).  In exact arithmetic
// sq8_mfma's quick test passes a pair when
//   DOT, MIP:   I·a_r·sb + E_r ≥ tq,            E_r = y_r·QY + z_r·QZ + w_r·QW + Q0
//   COSINE:     I·a_r·sb + E_r ≥ tq·√w_r
//   EUCLIDEAN:  2·I·a_r·sb ≥ w_r(1 − m) + Q0 − y_r·QY − z_r·QZ − tq / g2m
// and it is no stricter than sq8_bounds' upper side (sq8_mfma's derivation).  E_r and y_r·QY + z_r·QZ are
// at most their step maxima E, Em (every term ≥ 0), and √w_r ≥ √(min w), so each pass implies
//   DOT, MIP:   I·a_r ≥ (tq − E) / sb                               =: ca
//   COSINE:     I·(a_r / √w_r) ≥ (tq − E / √(min w)) / sb           =: ca
//   EUCLIDEAN:  I·a_r ≥ w_r·(1 − m)/(2sb) + (Q0 − Em − tq/g2m)/(2sb) =: w_r·ca + cb
// ca and cb are rounded DOWN by margins far above every float rounding here (the reciprocals and v_rsq are
// within 2 ulp): 2^-18 of the magnitudes entering each numerator, then 2^-16 of |c| + B, B ≥ |I·a_r|
// (Cauchy–Schwarz on the integer vectors: |I|·a_r ≤ y_r·|q_b|; COSINE ÷ √w_r).  The pair test
// fma(I, a, −c) is one rounding of an exact value, so it keeps its sign: every pair sq8_mfma's quick test
// passes, this one passes.  A zero query (sb = 0), a list that is not full (tq = ∓∞), a step with a zero
// row (COSINE) or a zero row itself (COSINE a/√w = NaN, taken as a pass) passes every pair.
template <int SIM>
__device__ __forceinline__ void quick_consts(float tq, float sb, float inv, float QY, float QZ, float Q0, float QW,
                                             float zq, float ig2m, float4 bm, float& ca, float& cb) {
    cb = 0.0f;
    if constexpr (SIM == SIM_EUCLIDEAN) {
        if (!(sb > 0.0f) || !(tq < __builtin_inff())) {
            ca = 0.0f;
            cb = -__builtin_inff();
            return;
        }
        const float Em = fmaf(bm.x, QY, bm.y * QZ);
        const float T = tq * ig2m;
        const float num = (Q0 - Em - T) - 0x1p-18f * (Q0 + Em + fabsf(T));
        ca = (1.0f - 0x1p-17f) * inv * (1.0f - 0x1p-20f);
        cb = num * inv;
        cb -= 0x1p-16f * (bm.z * ca + fabsf(cb) + bm.x * zq);
    } else {
        if (!(sb > 0.0f) || !(tq > -__builtin_inff())) {
            ca = -__builtin_inff();
            return;
        }
        float E = fmaf(bm.x, QY, fmaf(bm.y, QZ, fmaf(bm.z, QW, Q0)));
        float B = bm.x * zq;
        if constexpr (SIM == SIM_COSINE) {
            if (!(bm.w > 0.0f)) {
                ca = -__builtin_inff();
                return;
            }
            const float r = __builtin_amdgcn_rsqf(bm.w);
            E = E * r * (1.0f + 0x1p-20f);
            B = B * r;
        }
        const float num = (tq - E) - 0x1p-18f * (fabsf(tq) + E);
        const float c = num * inv;
        ca = c - 0x1p-16f * (fabsf(c) + B);
    }
}

// One quarter of a workgroup's share (persistent kernel), described once in LDS so that no global load of
// tile or segment metadata sits between the ring's LDS-DMAs (a compiler-inserted vmcnt(0) would drain it).
struct WideQuarter {
    const int4* xt;       // the wide copy's codes from the quarter's first 16-row group
    const float4* at;     // the wide copy's bound terms from its first group (kAuxGroupF4 float4 per group)
    uint32_t vrow0;       // view row of its first row
    int32_t nrows;        // (the pilot: its first step's rows at most)
    int32_t list;         // tile·4 + quarter: the settle's list, the pilot's slot
    int32_t shard;
    int32_t seg;
    int32_t pad[3];
    float4 bm;            // the quarter's row maxima {max s|q|, max |δ|, max |x|², min |x|²} (launch_wide_quarter_max)
};
static_assert(sizeof(WideQuarter) == 64, "one 64-B descriptor per quarter");

// Quarter j of the tile order (4 per wide tile): its rows, copy pointers and maxima.  The wide kernels read it
// from the view's table (launch_wide_quarter_table, built once with the tile table): computing it at launch
// took three dependent global loads (tile order → tile → the segment's pointers) in every workgroup's setup.
__device__ __forceinline__ WideQuarter wide_quarter_of(const TileDev* __restrict__ tiles,
                                                       const int32_t* __restrict__ tile_order, int j, int ks,
                                                       const int4* const* __restrict__ rows8t,
                                                       const float4* const* __restrict__ auxt,
                                                       const int64_t* __restrict__ seg_vrow,
                                                       const float4* __restrict__ quarter_bm) {
    const int tix = tile_order ? tile_order[j >> 2] : j >> 2, quarter = j & 3;
    const TileDev tile = tiles[tix];
    const int64_t trows = tile.row_end - tile.row_begin;
    const int64_t spw = ((trows + 4 * kMfmaScanR - 1) / (4 * kMfmaScanR)) * kMfmaScanR;
    const int64_t rb = min(tile.row_begin + quarter * spw, tile.row_end);
    const int64_t re = min(rb + spw, tile.row_end);
    WideQuarter d;
    d.xt = rows8t[tile.seg] + (rb >> 4) * (ks * 64);
    d.at = auxt[tile.seg] + (rb >> 4) * kAuxGroupF4;
    d.vrow0 = (uint32_t)(seg_vrow[tile.seg] + rb);
    d.nrows = (int32_t)(re - rb);
    d.list = tix * 4 + quarter;
    d.shard = tile.shard;
    d.seg = tile.seg;
    d.pad[0] = d.pad[1] = d.pad[2] = 0;
    d.bm = quarter_bm ? quarter_bm[d.list] : make_float4(0.f, 0.f, 0.f, 0.f);
    return d;
}
__global__ __launch_bounds__(kBlock) void wide_quarter_table(const TileDev* __restrict__ tiles,
                                                             const int32_t* __restrict__ tile_order, int n_q, int ks,
                                                             const int4* const* __restrict__ rows8t,
                                                             const float4* const* __restrict__ auxt,
                                                             const int64_t* __restrict__ seg_vrow,
                                                             const float4* __restrict__ quarter_bm,
                                                             WideQuarter* __restrict__ out) {
    const int j = blockIdx.x * kBlock + threadIdx.x;
    if (j < n_q) out[j] = wide_quarter_of(tiles, tile_order, j, ks, rows8t, auxt, seg_vrow, quarter_bm);
}
hipError_t launch_wide_quarter_table(const TileDev* tiles, const int32_t* tile_order, int n_q, int ks,
                                     const void* rows8t, const void* auxt, const int64_t* seg_vrow,
                                     const float4* quarter_bm, void* out, hipStream_t s) {
    if (n_q < 1) return hipSuccess;
    hipLaunchKernelGGL(wide_quarter_table, dim3((n_q + kBlock - 1) / kBlock), dim3(kBlock), 0, s, tiles, tile_order,
                       n_q, ks, static_cast<const int4* const*>(rows8t), static_cast<const float4* const*>(auxt),
                       seg_vrow, quarter_bm, static_cast<WideQuarter*>(out));
    return hipGetLastError();
}
// The parameters only the cold paths use (quarter-end flushes and drains, list overflows, the pilot's key
// stores), held in LDS: read from there they are not live across the step loop, whose hot values then keep
// their SGPRs instead of spilling to VGPR lanes.
struct WideCold {
    uint64_t* cand;
    uint32_t* cand_lb;
    uint32_t* list_lbmax;
    unsigned long long* visited;
    const float* qn_dev;
    uint64_t* pilot_keys;
    const uint32_t* floors;
    int q0, n_lists, q_count, n_quarters;
    float cos_slack, gam, g2;
};
constexpr int kWideMaxFloorShards = 16;   // per-(shard, query) floors held in LDS up to this many shards
constexpr int kWideThreads = kWideWaves * 64;
constexpr int kWideSorted = 1 << 20;      // s_cnt of a list the ordered insertion has sorted
constexpr int kWidePilotRows = 128;       // the pilot bounds each quarter's first 128 rows (1–4 steps)

// The ring's geometry per KS: GPS 16-row groups per step (one barrier per step), NS steps in the ring, the
// int8 slab DMAs per loader wave per step (waves 0–3: slab units w, w + 4, … of the step's GPS·KS) and the
// bound-term DMAs per aux wave (waves 4 … 4 + min(GPS, 4) − 1: groups w − 4, w, …).  LDS: KS = 2 → 4 steps of
// 8 groups (75 KB), 4 → 4 × 4 (71 KB), 8 → 4 × 2 (68 KB), 12 → 3 × 2 (76 KB), beside the lists (48 KB).
template <int KS>
struct WideGeom {
    static constexpr int GPS = KS <= 4 ? 16 / KS : 2;
    static constexpr int NS = KS <= 8 ? 4 : 3;
    static constexpr int LPW = GPS * KS / 4;
    static constexpr int APW = GPS >= 4 ? GPS / 4 : 1;
};

// Persistent: gridDim.x workgroups (one per CU), workgroup w takes quarters w, w + G, w + 2G, … of the
// tile order (tiles interleaved over shards), as ONE continuous stream of steps through the NS-deep LDS-DMA
// ring, so the ring never drains at a quarter boundary and the queries' B fragments, constants and floors
// are set up once per launch.  8 waves, two per SIMD; every wave scores its 32 queries against every group
// of a step.  Each wave flushes its queries' lists when its quarter ends.
template <int KS, int SIM>
__global__ __launch_bounds__(kWideThreads, 1) void sq8_wide(Sq8Params p) {
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    using Geo = WideGeom<KS>;
    constexpr int GPS = Geo::GPS, NS = Geo::NS, LPW = Geo::LPW, APW = Geo::APW;
    constexpr int QB = kWideQB;
    constexpr int AUXF4 = SIM == SIM_COSINE ? kAuxGroupF4 : 18;   // staged float4 of a group's bound terms
    constexpr int AUXB = AUXF4 * 16;          // a[16] y[16] z[16] w[16] {maxima} {s_g, f_cos, zero} (COSINE: xnorm[16])
    constexpr int GB = KS * 1024 + AUXB;      // one 16-row group in a slot
    constexpr int SLOT = GPS * GB;            // one step
    constexpr int sim = SIM;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int col = lane & 15, grp = lane >> 4;
    const bool dma_rows = wave < 4;                      // its int8 slabs (waves 0–3)…
    const bool dma_aux = !dma_rows && wave - 4 < GPS;    // …or bound terms (waves 4 … 4 + min(GPS, 4) − 1)
    const int u8 = p.units8, S = p.n_shards;
    const bool pilot = p.pilot != 0;
#ifdef OSK_TESTING
    // A/B timing only (results wrong): 1 skip the quick tests and lists, 2 skip the MFMAs, 8 no barrier between
    // steps, 16 no list / pilot-key stores, 32 quick tests without their insertions, 64 the ring alone
    const int ablate = p.ablate;
#else
    constexpr int ablate = 0;
#endif
    const int G = gridDim.x, n_quarters = 4 * p.n_tiles;
    const int qbeg = p.quarter_begin, n_range = (p.quarter_end > 0 ? p.quarter_end : n_quarters) - qbeg;
    const int n_mine = (int)blockIdx.x < n_range ? (n_range - 1 - (int)blockIdx.x) / G + 1 : 0;
    const bool floor_lds = S <= kWideMaxFloorShards;

    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ WideCold s_cold;
    if (tid == 0) s_cold = WideCold{p.cand, p.cand_lb, p.list_lbmax, p.visited, p.qn_dev, p.pilot_keys, p.floors, p.q0,
                                    p.n_lists, p.q_count, 4 * p.n_tiles, p.cos_slack, p.gam, p.g2};
    uint64_t* s_lk = reinterpret_cast<uint64_t*>(smem + NS * SLOT);      // [kWideQ][kKQ] upper-bound keys
    uint32_t* s_lp = reinterpret_cast<uint32_t*>(s_lk + kWideQ * kKQ);   // their lower bounds
    float4* s_qc = reinterpret_cast<float4*>(s_lp + kWideQ * kKQ);        // [kWideQ] query bound terms
    uint32_t* s_floor = reinterpret_cast<uint32_t*>(s_qc + kWideQ);       // [S][kWideQ] the pilot's floor scores
    int32_t* s_cnt = reinterpret_cast<int32_t*>(s_floor + (floor_lds ? S * kWideQ : 0));   // [kWideQ] list fill
    WideQuarter* s_quart = reinterpret_cast<WideQuarter*>(s_cnt + kWideQ);
    // the deferred insertions (p.wide_qcap > 0): per wave, qcap entries {int32 dot, row in quarter << 8 | query
    // in wave}, drained when the quarter ends (every wave at the same step) or when full
    // (EUCLIDEAN at KS = 2 keeps the immediate insertions: the queue's code spills there)
    const int qcap = (SIM == SIM_EUCLIDEAN && KS == 2) ? 0 : p.wide_qcap;
    uint2* s_q = reinterpret_cast<uint2*>(s_quart + n_mine) + (size_t)wave * qcap;
    for (int i = tid; i < kWideQ * kKQ; i += kWideThreads) {
        s_lk[i] = 0ull;
        s_lp[i] = 0u;
    }
    for (int i = tid; i < kWideQ; i += kWideThreads) s_cnt[i] = 0;
    for (int i = tid; i < kWideQ; i += kWideThreads) s_qc[i] = i < p.q_count ? p.qc[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    // the floor T of (query, shard) (launch_wide_floor; its score's sortable bits, 0 = none)
    auto floor_of = [&](int qi, int sh) -> uint32_t {
        return (pilot || !p.floors || qi >= p.q_count) ? 0u : p.floors[(size_t)qi * S + sh];
    };
    auto floor_of_cold = [&](int qi, int sh) -> uint32_t {   // (the same, in the step loop: from WideCold)
        const WideCold& c = s_cold;
        return (pilot || !c.floors || qi >= c.q_count) ? 0u : c.floors[(size_t)qi * S + sh];
    };
    if (floor_lds)
        for (int i = tid; i < S * kWideQ; i += kWideThreads) s_floor[i] = floor_of(i % kWideQ, i / kWideQ);
    for (int i = tid; i < n_mine; i += kWideThreads) {
        const int j = qbeg + (int)blockIdx.x + i * G;
        WideQuarter d = p.wide_qtable ? static_cast<const WideQuarter*>(p.wide_qtable)[j]
                                      : wide_quarter_of(p.tiles, p.tile_order, j, KS, p.rows8t, p.auxt, p.seg_vrow,
                                                        p.quarter_bm);
        if (pilot) d.nrows = min(d.nrows, p.pilot_rows > 0 ? p.pilot_rows : kWidePilotRows);   // its first rows
        s_quart[i] = d;
    }

    // this lane's queries: wq0 + qb·16 + col
    const int wq0 = wave * 16 * QB;
    i32x4 bfr[KS][QB];
    float sb[QB], inv[QB], QY[QB], QZ[QB], Q0[QB], zq[QB], tq[QB], qnd[QB];   // qnd: |q|² in device lane order (COSINE)
    uint64_t tkey[QB], qvm[QB];
    const float QW = __double2float_ru((double)p.gam * (1.0 + 0x1p-18));
    const float ig2m = 1.0f / (1.0f - p.g2);
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
        const int qi = wq0 + qb * 16 + col;
        const bool qv = qi < p.q_count;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int f = s * 4 + grp;
            const int4 v = (qv && f < u8) ? p.q8[(int64_t)qi * u8 + f] : make_int4(0, 0, 0, 0);
            bfr[s][qb] = i32x4{v.x, v.y, v.z, v.w};
        }
        const float4 qc = qv ? p.qc[qi] : make_float4(0.f, 0.f, 0.f, 0.f);
        sb[qb] = qc.x;
        inv[qb] = qc.x > 0.0f ? (SIM == SIM_EUCLIDEAN ? 0.5f : 1.0f) / qc.x : 0.0f;
        zq[qb] = qc.x > 0.0f ? qc.z / qc.x * (1.0f + 0x1p-20f) : 0.0f;
        if constexpr (SIM == SIM_EUCLIDEAN) {   // sq8_mfma's coefficients, exactly
            const double m = 0x1p-17;
            QY[qb] = __double2float_ru((2.0 + 2.0 * m) * (double)qc.y + 2.0 * m * (double)qc.z);
            QZ[qb] = __double2float_ru((2.0 + 2.0 * m) * (double)qc.z);
            Q0[qb] = __double2float_rd((double)qc.w * (1.0 - m));
        } else {
            const double r = 1.0 + 0x1p-18;
            QY[qb] = __double2float_ru(((double)qc.y + 0x1p-18 * (double)qc.z) * r);
            QZ[qb] = __double2float_ru((double)qc.z * r);
            Q0[qb] = __double2float_ru((double)p.gam * (double)qc.w * r);
        }
        qnd[qb] = (SIM == SIM_COSINE && qv) ? p.qn_dev[qi] : 0.0f;
        tkey[qb] = 0ull;
        tq[qb] = sq8_quick(sim, 0ull, 0.0f, 0.0f);
        qvm[qb] = __ballot(qv);
    }
    __syncthreads();   // lists zeroed; s_qc, the floors and the quarter descriptors written
    // Consume every register the prologue loaded from global memory before the first LDS-DMA: the compiler
    // cannot see the ring's DMAs, and a load still pending at the step loop's header makes it put a
    // vmcnt(0) inside the loop, which drains the whole ring each step.
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
#pragma unroll
        for (int s = 0; s < KS; ++s) asm volatile("" ::"v"(bfr[s][qb]));
        asm volatile("" ::"v"(qnd[qb]), "v"(inv[qb]));
    }

    // the workgroup's steps: its quarters' steps back to back (empty quarters take none)
    // (LDS values the whole wave reads alike: readfirstlane keeps the loop control in SGPRs)
    auto steps_of = [&](int q) {
        return __builtin_amdgcn_readfirstlane((s_quart[q].nrows + 16 * GPS - 1) / (16 * GPS));
    };
    int total = 0;
    for (int q = 0; q < n_mine; ++q) total += steps_of(q);
    total = __builtin_amdgcn_readfirstlane(total);
    const uint32_t ring_lds =
        __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(__attribute__((address_space(3))) char*)smem);
    // a group's dots: acc[qb] = the int8 dots of its 16 rows (4·grp + r) with query block qb (column col)
    auto group_dots = [&](const char* gb, i32x4 (&ac)[QB]) {
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) ac[qb] = i32x4{0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const i32x4 a = *reinterpret_cast<const i32x4*>(gb + s * 1024 + lane * 16);
#pragma unroll
            for (int qb = 0; qb < QB; ++qb) ac[qb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bfr[s][qb], ac[qb], 0, 0, 0);
        }
    };
    int iq = 0, ist = 0;   // the next step to issue: quarter iq of mine, its step ist
    while (iq < n_mine && steps_of(iq) == 0) ++iq;
    auto rfl_ptr = [](const void* ptr) {
        const uint64_t v = (uint64_t)ptr;
        return (const char*)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
                             (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v));
    };
    // the issuing quarter's descriptor, held in SGPRs while its steps are issued: a step reads no descriptor
    // from LDS (each such read is a round trip queued behind the other waves' fragment reads, and the DMAs'
    // asm clobbers memory, so it would be re-read between them)
    int i_nrows = 0, i_steps = 0;
    const int4* i_xt = nullptr;
    const float4* i_at = nullptr;
    auto load_iq = [&]() {
        if (iq >= n_mine) return;
        const WideQuarter& d = s_quart[iq];
        i_nrows = __builtin_amdgcn_readfirstlane(d.nrows);
        i_steps = __builtin_amdgcn_readfirstlane((i_nrows + 16 * GPS - 1) / (16 * GPS));
        i_xt = reinterpret_cast<const int4*>(rfl_ptr(d.xt));
        i_at = reinterpret_cast<const float4*>(rfl_ptr(d.at));
    };
    load_iq();
    // this wave's part of the step → slot; groups past the quarter load its first group (valid, skipped)
    auto issue = [&](int slot) {
        const int nrows = i_nrows;
        const int4* xt = i_xt;
        const float4* at = i_at;
        const uint32_t base = ring_lds + (uint32_t)(slot * SLOT);
        // a step inside the quarter (every step but possibly its last): one DMA statement per wave over
        // contiguous memory — the row waves' LPW consecutive 1 KiB units u = LPW·wave + j, the term waves' APW
        // consecutive groups — from one SGPR base with immediate offsets (no per-DMA address arithmetic)
        if ((LPW <= 4 || LPW == 6) && 16 * GPS * (ist + 1) <= nrows) {
            if (dma_rows) {
                const int u0 = LPW * wave;   // (KS ≥ 4: the units stay inside one group; KS = 2: 2 groups)
                constexpr int N0 = LPW <= 4 ? LPW : 4, N1 = LPW - N0;   // (6 units: 4 + 2, the offset field is 12-bit)
                uint32_t l0[N0], l1[N1 > 0 ? N1 : 1];
#pragma unroll
                for (int j = 0; j < LPW; ++j) {
                    const int u = u0 + j, g = u / KS, sl = u - g * KS;
                    (j < N0 ? l0[j] : l1[j - N0 < 0 ? 0 : j - N0]) = base + (uint32_t)(g * GB + sl * 1024);
                }
                const char* gb = reinterpret_cast<const char*>(xt) + ((size_t)(GPS * KS * ist + u0) << 10);
                glds16_run<N0, 1024>(gb, (uint32_t)lane * 16u, l0);
                if constexpr (N1 > 0) glds16_run<N1, 1024>(gb + N0 * 1024, (uint32_t)lane * 16u, l1);
            } else if (dma_aux && lane < AUXF4) {
                const int g0 = APW * (wave - 4);
                uint32_t l[APW];
#pragma unroll
                for (int h = 0; h < APW; ++h) l[h] = base + (uint32_t)((g0 + h) * GB + KS * 1024);
                glds16_run<APW, kAuxGroupF4 * 16>(at + (size_t)(GPS * ist + g0) * kAuxGroupF4, (uint32_t)lane * 16u, l);
            }
        } else if (dma_rows) {
#pragma unroll
            for (int j = 0; j < LPW; ++j) {
                const int u = wave + 4 * j, g = u / KS, s = u - g * KS;   // (wave-uniform)
                const int gi = GPS * ist + g;
                const int gv = 16 * gi < nrows ? gi : 0;
                glds16(xt + gv * (KS * 64) + s * 64 + lane, base + (uint32_t)(g * GB + s * 1024));
            }
        } else if (dma_aux && lane < AUXF4) {
#pragma unroll
            for (int h = 0; h < APW; ++h) {
                const int g = wave - 4 + 4 * h;
                const int gi = GPS * ist + g;
                const int gv = 16 * gi < nrows ? gi : 0;
                glds16(at + gv * kAuxGroupF4 + lane, base + (uint32_t)(g * GB + KS * 1024));
            }
        }
        if (++ist == i_steps) {
            ist = 0;
            do ++iq; while (iq < n_mine && steps_of(iq) == 0);
            load_iq();
        }
    };

    // the full bound terms {a, y, z, w} of the lane's 4 rows (4·grp + r) of a group (pilot and insertions)
    auto row_terms = [&](const char* ga, float4 (&ax)[4]) {
        // (COSINE: slot 0 holds the rows' quick-test factors; the scale s_g is the group's, in slot 17)
        float4 A;
        if constexpr (SIM == SIM_COSINE) {
            const float sg = *reinterpret_cast<const float*>(ga + 17 * 16);
            A = make_float4(sg, sg, sg, sg);
        } else {
            A = *reinterpret_cast<const float4*>(ga + grp * 16);
        }
        const float4 Y = *reinterpret_cast<const float4*>(ga + 64 + grp * 16);
        const float4 Z = *reinterpret_cast<const float4*>(ga + 128 + grp * 16);
        const float4 W = *reinterpret_cast<const float4*>(ga + 192 + grp * 16);
        ax[0] = make_float4(A.x, Y.x, Z.x, W.x);
        ax[1] = make_float4(A.y, Y.y, Z.y, W.y);
        ax[2] = make_float4(A.z, Y.z, Z.z, W.z);
        ax[3] = make_float4(A.w, Y.w, Z.w, W.w);
    };
    // the per-row quick test of the lane's 4 rows against one query: t_r = fma(I, a_r, −ca) (EUCLIDEAN
    // fma(I, a_r, −fma(w_r, ca, cb))), as packed pairs; pass = !(t_r < 0).  Rows past the quarter may pass
    // here (the insertion drops them).
    auto quick_t = [&](const i32x4& I, const float (&ar)[4], const float (&wr)[4], float c, float c2, f32x2& t01,
                       f32x2& t23) {
        const f32x2 I01 = {(float)I[0], (float)I[1]}, I23 = {(float)I[2], (float)I[3]};
        const f32x2 A01 = {ar[0], ar[1]}, A23 = {ar[2], ar[3]};
        if constexpr (SIM == SIM_EUCLIDEAN) {
            const f32x2 C = {c, c}, D = {c2, c2};
            t01 = __builtin_elementwise_fma(I01, A01, -__builtin_elementwise_fma(f32x2{wr[0], wr[1]}, C, D));
            t23 = __builtin_elementwise_fma(I23, A23, -__builtin_elementwise_fma(f32x2{wr[2], wr[3]}, C, D));
        } else {
            const f32x2 C = {-c, -c};
            t01 = __builtin_elementwise_fma(I01, A01, C);
            t23 = __builtin_elementwise_fma(I23, A23, C);
        }
    };
#ifdef OSK_TESTING
    uint32_t n_events = 0, n_pairs = 0, n_slow = 0;   // insertion events, quick-test passes, slow-path steps
    uint64_t cyc_wait = 0, cyc_loop = 0;   // wave 0's clocks: the step loop's waits, the whole loop
    uint64_t cyc_slow = 0, cyc_drain = 0;  // …the slow path's (deferred) enqueues, the quarter-end drains + flushes
#endif
    float ca[QB], cb[QB];   // the current quarter's quick-test constants
    // a quarter ends: its lists (this wave's queries, 4 per pass of 16 lanes) → the settle's arrays, zeroed
    auto flush = [&](const WideQuarter& d) {
        const WideCold& c = s_cold;
        const int q_end = min(wq0 + 16 * QB, c.q_count);
        for (int q0 = wq0; q0 < q_end; q0 += 4) {
            const int qg = q0 + (lane >> 4), e = lane & 15;
            const uint64_t lkb = s_lk[qg * kKQ + e];
            const uint32_t lpb = s_lp[qg * kKQ + e];
            uint32_t m = lkb ? lpb : 0u;
#pragma unroll
            for (int o = 8; o >= 1; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
            if (qg < q_end && !(ablate & 16)) {
                const size_t l = (size_t)(c.q0 + qg) * c.n_lists + d.list;
                c.cand[l * kKQ + e] = lkb;
                c.cand_lb[l * kKQ + e] = lpb;
                if (e == 0) c.list_lbmax[l] = m;
                s_lk[qg * kKQ + e] = 0ull;
                s_lp[qg * kKQ + e] = 0u;
                if (e == 0) s_cnt[qg] = 0;
            }
        }
        if (c.visited && c.q0 == 0 && tid == 0 && d.nrows > 0)
            atomicAdd(&c.visited[d.seg], (unsigned long long)d.nrows);
    };

    // empty quarters (tiles of a few rows) take no step, but the settle and the pilot merge read every
    // (query, quarter) slot: write them empty here (lists: zero keys; pilot: key 0)
    for (int q = 0; q < n_mine; ++q) {
        const WideQuarter& d = s_quart[q];
        if (d.nrows > 0) continue;
        if (pilot) {
#pragma unroll
            for (int qb = 0; qb < QB; ++qb) {
                const int qi = wq0 + qb * 16 + col;
                if (grp == 0 && qi < p.q_count) {
                    p.pilot_keys[(size_t)qi * n_quarters + d.list] = 0ull;
                    p.list_lbmax[(size_t)(p.q0 + qi) * p.n_lists + d.list] = 0u;   // (read as empty until written)
                }
            }
        } else {
            flush(d);   // (the LDS lists are all zero here)
        }
    }
    if (total > 0) {
        for (int st = 0; st < NS - 1 && st < total; ++st) issue(st);
        int s_issue = (NS - 1) % NS, s_read = 0;
        int pq = -1, pst = 0;   // the quarter of mine and its step the current step belongs to
        int p_nrows = 0, p_steps = 0;   // (its rows and steps, in SGPRs: see load_iq)
        const char* hslot = smem;
        int hst = 0, hgroups = 0, hq = 0;
        i32x4 acc[GPS][QB];
        uint64_t pbest[QB];   // the pilot: the current quarter's best lower-bound key per query so far
        float4 bm = make_float4(0.f, 0.f, 0.f, 0.f);
        int qn = 0;   // (wave-uniform) entries in this wave's deferred queue
        // The deferred insertions of quarter d, 64 at a time, one entry per lane: its row's bound terms from the
        // quarter's tiled terms in global memory (the ring slot is long gone), the precise bound, and above the
        // floor an append to its (quarter, query) list; lists that would fill take the ordered insertion, one
        // query at a time.  Same lists, same thresholds as the immediate path.
        auto drain = [&](const WideQuarter& d) {
            const int sh = d.shard;
            for (int i0 = 0; i0 < qn; i0 += 64) {
                const bool ok = i0 + lane < qn;
                const uint2 en = ok ? s_q[i0 + lane] : make_uint2(0u, 0u);
                const int qw = (int)(en.y & 255u), rowq = (int)(en.y >> 8);
                const int qi = wq0 + qw;
                const float* af = reinterpret_cast<const float*>(d.at + (rowq >> 4) * kAuxGroupF4);
                const int rr = rowq & 15;
                const float a_r = SIM == SIM_COSINE ? af[68] : af[rr];   // (COSINE: the group's s_g, slot 17)
                const float4 ax = ok ? make_float4(a_r, af[16 + rr], af[32 + rr], af[48 + rr]) : make_float4(0.f, 0.f, 0.f, 0.f);
                float xnd = 0.0f, qndq = 0.0f;
                if constexpr (SIM == SIM_COSINE) {
                    xnd = ok ? af[72 + rr] : 0.0f;
                    qndq = ok ? s_cold.qn_dev[qi] : 0.0f;
                }
                uint64_t key = 0ull;
                uint32_t lbs = 0u;
                bool ovf = false;
                if (ok) {
                    const float4 qcb = s_qc[qi];
                    float lo, hi;
                    sq8_bounds(sim, (float)(int32_t)en.x, ax, qcb, s_cold.gam, s_cold.g2, lo, hi);
                    const float ub = SIM == SIM_EUCLIDEAN ? score_f32_l2(lo) : score_f32(sim, hi, qndq, xnd);
                    const float lb = SIM == SIM_EUCLIDEAN ? score_f32_l2(hi) : score_f32(sim, lo, qndq, xnd);
                    const uint64_t kr = make_key(ub, d.vrow0 + (uint32_t)rowq);
                    const uint64_t tk = (uint64_t)(floor_lds ? s_floor[sh * kWideQ + qi] : floor_of_cold(qi, sh)) << 32;
                    if (kr > tk) {   // below the floor: cannot enter the top k
#ifdef OSK_TESTING
                        ++n_pairs;
#endif
                        const int pos = atomicAdd(&s_cnt[qi], 1);
                        if (pos < kKQ - 1) {
                            s_lk[qi * kKQ + pos] = kr;
                            s_lp[qi * kKQ + pos] = float_to_sortable(lb);
                        } else {
                            key = kr;
                            lbs = float_to_sortable(lb);
                            ovf = true;
                        }
                    }
                }
                uint64_t om = __ballot(ovf);
                while (om) {   // the overflowed queries, one at a time
                    const int Q = __builtin_amdgcn_readlane(qw, (int)__builtin_ctzll(om));
                    const int qo_g = wq0 + Q, o0 = qo_g * kKQ;
                    uint64_t lkb = lane < kKQ ? s_lk[o0 + lane] : 0ull;
                    uint32_t lpb = lane < kKQ ? s_lp[o0 + lane] : 0u;
                    if (s_cnt[qo_g] < kWideSorted) {   // first overflow: sort the appended rows (zeros last)
                        int rank = 0;
#pragma unroll 2
                        for (int j = 0; j < kKQ; ++j) {
                            const uint64_t kj = s_lk[o0 + j];
                            rank += (kj > lkb) || (kj == lkb && j < lane);
                        }
                        if (lane < kKQ) {
                            s_lk[o0 + rank] = lkb;
                            s_lp[o0 + rank] = lpb;
                        }
                        lkb = lane < kKQ ? s_lk[o0 + lane] : 0ull;
                        lpb = lane < kKQ ? s_lp[o0 + lane] : 0u;
                    }
                    uint64_t thrb = readlane64(lkb, kKQ - 1);
                    wave_offer2(key, lbs, ovf && qw == Q, lkb, lpb, thrb, lane, kKQ);
                    if (lane < kKQ) {
                        s_lk[o0 + lane] = lkb;
                        s_lp[o0 + lane] = lpb;
                    }
                    if (lane == 0) s_cnt[qo_g] = kWideSorted;
                    if (col == (Q & 15) && thrb) {   // full: its 16th key joins the floor under the threshold
#pragma unroll
                        for (int qb = 0; qb < QB; ++qb)
                            if (qb == (Q >> 4)) {
                                tq[qb] = sq8_quick(sim, thrb > tkey[qb] ? thrb : tkey[qb], sqrtf(qnd[qb]), s_cold.cos_slack);
                                quick_consts<SIM>(tq[qb], sb[qb], inv[qb], QY[qb], QZ[qb], Q0[qb], QW, zq[qb], ig2m, bm,
                                                  ca[qb], cb[qb]);
                            }
                    }
                    om = __ballot(ovf && qw != Q);
                    ovf = ovf && qw != Q;
                }
            }
            qn = 0;
        };
        // the step's quick tests and insertions
        auto quick_phase = [&]() __attribute__((always_inline)) {
            const WideQuarter& hd = s_quart[hq];
            // (1) the fast test: per group, the lane's largest dot over its 4 rows against a factor common to
            // the group's rows, ONE vote per step.  DOT / MIP: every row's factor is s_g, and fma(I, s_g, −c) is
            // monotone in I, so t = fma(max I, s_g, −c) < 0 iff every row fails the per-row test.  COSINE: the
            // per-row factor a_r·rsq(w_r) ≤ f_cos (2^-20 above s_g / √(min w), far beyond v_rsq's error), so with
            // c > 0 (a row can pass only with I > 0) t = fma(max I, f_cos, −c) < 0 implies every row fails; with
            // c ≤ 0 every pair takes the slow path, and so does a group with a zero row.  EUCLIDEAN: the per-row
            // test itself (its threshold is affine in each row's |x|²), reduced to one vote per step.
            float tf[GPS][QB];
            bool zg[GPS];
            uint32_t pbits[GPS];   // EUCLIDEAN: bit qb·4 + r = row r of the group passed for query block qb
            float sgs[GPS];        // DOT / MIP: the group's scale s_g (every valid row's per-row factor)
#pragma unroll
            for (int g = 0; g < GPS; ++g) {
                const char* ga = hslot + g * GB + KS * 1024;
                zg[g] = false;
                if constexpr (SIM == SIM_EUCLIDEAN) {
                    const float4 A4 = *reinterpret_cast<const float4*>(ga + grp * 16);
                    const float4 W4 = *reinterpret_cast<const float4*>(ga + 192 + grp * 16);
                    const float ar[4] = {A4.x, A4.y, A4.z, A4.w}, wr[4] = {W4.x, W4.y, W4.z, W4.w};
#pragma unroll
                    for (int qb = 0; qb < QB; ++qb) {
                        f32x2 t01, t23;
                        quick_t(acc[g][qb], ar, wr, ca[qb], cb[qb], t01, t23);
                        tf[g][qb] = fmaxf(fmaxf(t01.x, t01.y), fmaxf(t23.x, t23.y));
                        pbits[g] = (qb ? pbits[g] : 0u) | (uint32_t)!(t01.x < 0.0f) << (qb * 4) |
                                   (uint32_t)!(t01.y < 0.0f) << (qb * 4 + 1) | (uint32_t)!(t23.x < 0.0f) << (qb * 4 + 2) |
                                   (uint32_t)!(t23.y < 0.0f) << (qb * 4 + 3);
                    }
                } else {
                    const float4 gf = *reinterpret_cast<const float4*>(ga + 17 * 16);   // {s_g, f_cos, zero row, 0}
                    const float f = SIM == SIM_COSINE ? gf.y : gf.x;
                    sgs[g] = gf.x;
                    if constexpr (SIM == SIM_COSINE) zg[g] = gf.z != 0.0f;   // (wave-uniform: one LDS word)
#pragma unroll
                    for (int qb = 0; qb < QB; ++qb) {
                        const i32x4& I = acc[g][qb];
                        const int M = max(max(I[0], I[1]), max(I[2], I[3]));
                        const float c = (SIM == SIM_COSINE && !(ca[qb] > 0.0f)) ? -__builtin_inff() : ca[qb];
                        tf[g][qb] = fmaf((float)M, f, -c);
                    }
                }
            }
            float run = -__builtin_inff();
            bool zany = false;
#pragma unroll
            for (int g = 0; g < GPS; ++g) {
                zany = zany || zg[g];
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) run = fmaxf(run, tf[g][qb]);
            }
            if (!__ballot(!(run < 0.0f)) && !zany) return;
#ifdef OSK_TESTING
            ++n_slow;
            const uint64_t c_slow0 = clock64();
#endif
            if (!(SIM == SIM_EUCLIDEAN && KS == 2) && qcap > 0 && !(ablate & 32)) {
                // deferred mode: the passing pairs of each (group, query block) whose vote passed go to the wave's
                // queue — the per-row test on the step's accumulators (static indices), a ballot per row and an
                // LDS write per pair; bounds and list insertions wait for the quarter's end (drain)
#pragma unroll
                for (int g = 0; g < GPS; ++g) {
                    if (g >= hgroups) continue;   // (wave-uniform: the quarter's last step)
#pragma unroll
                    for (int qb = 0; qb < QB; ++qb) {
                        if (!(__ballot(!(tf[g][qb] < 0.0f) || zg[g]) & qvm[qb])) continue;
#ifdef OSK_TESTING
                        ++n_events;
#endif
                        const char* ga = hslot + g * GB + KS * 1024;
                        // the per-row factors: DOT / MIP the group's s_g (no LDS read), COSINE each row's
                        // s_g / √|x|² (slot 0; a zero row's +∞ makes its pairs pass)
                        float arg[4] = {sgs[g], sgs[g], sgs[g], sgs[g]};
                        const float wrg[4] = {0.0f, 0.0f, 0.0f, 0.0f};   // (EUCLIDEAN only)
                        if constexpr (SIM == SIM_COSINE) {
                            const float4 Ag = *reinterpret_cast<const float4*>(ga + grp * 16);
                            arg[0] = Ag.x, arg[1] = Ag.y, arg[2] = Ag.z, arg[3] = Ag.w;
                        }
                        const int r0 = 16 * (GPS * hst + g);
                        const int nr = min(16, p_nrows - r0);
                        bool pass[4];
                        if constexpr (SIM == SIM_EUCLIDEAN) {   // the fast test was the per-row test: its bits
#pragma unroll
                            for (int r = 0; r < 4; ++r) pass[r] = (pbits[g] >> (qb * 4 + r)) & 1u;
                        } else {
                            f32x2 t01, t23;
                            quick_t(acc[g][qb], arg, wrg, ca[qb], cb[qb], t01, t23);
                            pass[0] = !(t01.x < 0.0f), pass[1] = !(t01.y < 0.0f);
                            pass[2] = !(t23.x < 0.0f), pass[3] = !(t23.y < 0.0f);
                        }
                        const bool qv = (qvm[qb] >> lane) & 1ull;
                        bool pr[4];
                        uint64_t b[4];
                        int tot = 0;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            pr[r] = pass[r] && 4 * grp + r < nr && qv;
                            b[r] = __ballot(pr[r]);
                            tot += __popcll(b[r]);
                        }
                        if (qn + tot > qcap) drain(hd);   // (tot ≤ 256 ≤ qcap)
                        int base = qn;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(b[r] >> 32),
                                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)b[r], 0u));
                            if (pr[r])
                                s_q[base + below] = make_uint2((uint32_t)acc[g][qb][r],
                                                               (uint32_t)(r0 + 4 * grp + r) << 8 | (uint32_t)(qb * 16 + col));
                            base += __popcll(b[r]);
                        }
                        qn = base;
                    }
                }
#ifdef OSK_TESTING
                cyc_slow += clock64() - c_slow0;
#endif
                return;
            }
            // (2) the slow path: per group the wave's queries with a group that may pass (wave-uniform)
            uint32_t qmg[GPS];
#pragma unroll
            for (int g = 0; g < GPS; ++g) {
                uint32_t qm = 0u;
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) {
                    const uint64_t bl = __ballot(!(tf[g][qb] < 0.0f) || zg[g]) & qvm[qb];
                    qm |= (uint32_t)((bl | (bl >> 16) | (bl >> 32) | (bl >> 48)) & 0xFFFFull) << (16 * qb);
                }
                qmg[g] = g < hgroups ? qm : 0u;
            }
            uint32_t qany = 0u;
#pragma unroll
            for (int g = 0; g < GPS; ++g) qany |= qmg[g];
            if (!qany || (ablate & 32)) return;
            // group g's insertions, its dots in ac
            auto event_group = [&](int g, const i32x4 (&ac)[QB], uint32_t qmgg) __attribute__((always_inline)) {
#ifdef OSK_TESTING
                n_events += __popc(qmgg);
#endif
                const char* gb = hslot + g * GB;
                const char* ga = gb + KS * 1024;
                const float4 Ag = *reinterpret_cast<const float4*>(ga + grp * 16);
                const float4 Wg = *reinterpret_cast<const float4*>(ga + 192 + grp * 16);
                float arg[4] = {Ag.x, Ag.y, Ag.z, Ag.w};
                const float wrg[4] = {Wg.x, Wg.y, Wg.z, Wg.w};
                if constexpr (SIM == SIM_COSINE) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) arg[r] = arg[r] * __builtin_amdgcn_rsqf(wrg[r]);   // (0 · ∞ = NaN: passes)
                }
                const int r0 = 16 * (GPS * hst + g);   // rows of the quarter
                const int nr = min(16, p_nrows - r0);
                float4 ax[4];
                row_terms(ga, ax);
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) {
                    if (!((qmgg >> (16 * qb)) & 0xFFFFu)) continue;   // (wave-uniform)
                    // Every passing pair at once, in its own lane (row 4·grp + r, query col): its precise bound;
                    // above the floor it is appended to its (quarter, query) list by an LDS atomic while the list
                    // holds < kKQ − 1 rows (appended lists are unordered); the rest overflow to the ordered
                    // insertion below, which sorts the list once and keeps its best kKQ (a full list is sorted,
                    // its 16th key the threshold: the settle's contract).
                    f32x2 t01, t23;
                    quick_t(ac[qb], arg, wrg, ca[qb], cb[qb], t01, t23);
                    const float t[4] = {t01.x, t01.y, t23.x, t23.y};
                    const int qg = wq0 + qb * 16 + col;
                    const bool qv = (qvm[qb] >> lane) & 1ull;
                    uint64_t key[4];
                    uint32_t lbs[4];
                    bool ovf[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int rr = 4 * grp + r;
                        key[r] = 0ull;
                        lbs[r] = 0u;
                        ovf[r] = false;
                        if (!(t[r] < 0.0f) && rr < nr && qv) {
                            const float4 qcb = s_qc[qg];
                            float xnd = 0.0f;
                            if constexpr (SIM == SIM_COSINE) xnd = *reinterpret_cast<const float*>(ga + 288 + rr * 4);
                            float lo, hi;
                            sq8_bounds(sim, (float)ac[qb][r], ax[r], qcb, s_cold.gam, s_cold.g2, lo, hi);
                            const float ub = SIM == SIM_EUCLIDEAN ? score_f32_l2(lo) : score_f32(sim, hi, qnd[qb], xnd);
                            const float lb = SIM == SIM_EUCLIDEAN ? score_f32_l2(hi) : score_f32(sim, lo, qnd[qb], xnd);
                            const uint64_t kr = make_key(ub, hd.vrow0 + (uint32_t)(r0 + rr));
                            if (kr > tkey[qb]) {   // below the floor: cannot enter the top k
#ifdef OSK_TESTING
                                ++n_pairs;
#endif
                                const int pos = atomicAdd(&s_cnt[qg], 1);
                                if (pos < kKQ - 1) {
                                    s_lk[qg * kKQ + pos] = kr;
                                    s_lp[qg * kKQ + pos] = float_to_sortable(lb);
                                } else {
                                    key[r] = kr;
                                    lbs[r] = float_to_sortable(lb);
                                    ovf[r] = true;
                                }
                            }
                        }
                    }
                    uint64_t om = __ballot(ovf[0] || ovf[1] || ovf[2] || ovf[3]);
                    uint32_t qo = (uint32_t)((om | (om >> 16) | (om >> 32) | (om >> 48)) & 0xFFFFull);
                    while (qo) {   // the overflowed queries, one at a time (rare: the floor keeps lists short)
                        const int bc = __builtin_ctz(qo);
                        qo &= qo - 1u;
                        const int qo_g = wq0 + qb * 16 + bc;
                        const int o0 = qo_g * kKQ;
                        uint64_t lkb = lane < kKQ ? s_lk[o0 + lane] : 0ull;
                        uint32_t lpb = lane < kKQ ? s_lp[o0 + lane] : 0u;
                        if (s_cnt[qo_g] < kWideSorted) {   // first overflow: sort the appended rows (zeros last)
                            int rank = 0;
#pragma unroll 2
                            for (int j = 0; j < kKQ; ++j) {
                                const uint64_t kj = s_lk[o0 + j];
                                rank += (kj > lkb) || (kj == lkb && j < lane);
                            }
                            if (lane < kKQ) {
                                s_lk[o0 + rank] = lkb;
                                s_lp[o0 + rank] = lpb;
                            }
                            lkb = lane < kKQ ? s_lk[o0 + lane] : 0ull;
                            lpb = lane < kKQ ? s_lp[o0 + lane] : 0u;
                        }
                        uint64_t thrb = readlane64(lkb, kKQ - 1);
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            wave_offer2(key[r], lbs[r], ovf[r] && col == bc, lkb, lpb, thrb, lane, kKQ);
                        if (lane < kKQ) {
                            s_lk[o0 + lane] = lkb;
                            s_lp[o0 + lane] = lpb;
                        }
                        if (lane == 0) s_cnt[qo_g] = kWideSorted;   // sorted: later rows all take this path
                        if (col == bc && thrb) {   // full: its 16th key joins the floor under the threshold
                            tq[qb] = sq8_quick(sim, thrb > tkey[qb] ? thrb : tkey[qb], sqrtf(qnd[qb]), s_cold.cos_slack);
                            quick_consts<SIM>(tq[qb], sb[qb], inv[qb], QY[qb], QZ[qb], Q0[qb], QW, zq[qb], ig2m, bm,
                                              ca[qb], cb[qb]);
                        }
                    }
                }
            };
            if constexpr (GPS <= 2) {   // the step's accumulators are still here (static indices: unrolled)
#pragma unroll
                for (int g = 0; g < GPS; ++g)
                    if (g < hgroups && qmg[g]) event_group(g, acc[g], qmg[g]);
            } else {
#pragma unroll 1
                for (int g = 0; g < hgroups; ++g) {
                    uint32_t qmgg = 0u;   // (g is wave-uniform: selects, no indexed register access)
#pragma unroll
                    for (int gg = 0; gg < GPS; ++gg) qmgg = gg == g ? qmg[gg] : qmgg;
                    if (!qmgg) continue;
                    // group g's dots again, from its slot (no register array indexed by the runtime g: that
                    // would put the step's accumulators in scratch memory)
                    i32x4 ac[QB];
                    group_dots(hslot + g * GB, ac);
                    event_group(g, ac, qmgg);
                }
            }
        };
#ifdef OSK_TESTING
        const uint64_t c_loop0 = clock64();
#endif
        for (int i = 0; i < total; ++i) {
#ifdef OSK_TESTING
            const uint64_t c0 = clock64();
#endif
            // this wave's DMAs of step i have landed (steps i+1 … i+NS−2 may still be in flight); every wave's
            // have once all pass the barrier, which also retires every wave's reads of step i − 1's slot
            if (i + NS - 1 <= total) {
                if (dma_rows) vm_wait<(NS - 2) * LPW>();
                else if (dma_aux) vm_wait<(NS - 2) * APW>();
                else vm_wait<0>();
            } else {
                vm_wait<0>();
            }
            if (!(ablate & 8)) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#ifdef OSK_TESTING
            cyc_wait += clock64() - c0;
#endif
            if (i + NS - 1 < total) {
                issue(s_issue);
                s_issue = s_issue + 1 == NS ? 0 : s_issue + 1;
            }
            if (ablate & 64) continue;   // (A/B: the ring alone)
            if (pq < 0 || ++pst == p_steps) {   // a new quarter: flush the last one, take its floors
                if (pq >= 0 && !pilot) {
#ifdef OSK_TESTING
                    const uint64_t c_dr0 = clock64();
#endif
                    if (qn) drain(s_quart[pq]);
                    flush(s_quart[pq]);
#ifdef OSK_TESTING
                    cyc_drain += clock64() - c_dr0;
#endif
                }
                do ++pq; while (steps_of(pq) == 0);
                pst = 0;
                p_nrows = __builtin_amdgcn_readfirstlane(s_quart[pq].nrows);
                p_steps = __builtin_amdgcn_readfirstlane((p_nrows + 16 * GPS - 1) / (16 * GPS));
                const int sh = s_quart[pq].shard;
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) {
                    const int qi = wq0 + qb * 16 + col;
                    const uint32_t f = floor_lds ? s_floor[sh * kWideQ + qi] : floor_of_cold(qi, sh);
                    tkey[qb] = (uint64_t)f << 32;
                    tq[qb] = sq8_quick(sim, tkey[qb], sqrtf(qnd[qb]), s_cold.cos_slack);
                }
                // the quarter's row maxima → its quick-test constants (the quick test relaxes each pair's
                // error terms to the maxima of the rows it is taken over: here the quarter's)
                bm = s_quart[pq].bm;
#pragma unroll
                for (int qb = 0; qb < QB; ++qb)
                    quick_consts<SIM>(tq[qb], sb[qb], inv[qb], QY[qb], QZ[qb], Q0[qb], QW, zq[qb], ig2m, bm, ca[qb],
                                      cb[qb]);
            }
            hslot = smem + s_read * SLOT;
            s_read = s_read + 1 == NS ? 0 : s_read + 1;
            hq = pq;
            hst = pst;
            hgroups = __builtin_amdgcn_readfirstlane(min(GPS, ((p_nrows + 15) >> 4) - GPS * pst));   // (< GPS: the quarter's last step)
            if (pilot) {   // the quarter's first rows: per query the best lower-bound key → pilot_keys
                const WideQuarter& hd = s_quart[hq];
                if (pst == 0) {
#pragma unroll
                    for (int qb = 0; qb < QB; ++qb) pbest[qb] = 0ull;
                }
#pragma unroll 1
                for (int g = 0; g < hgroups; ++g) {
                    const char* gb = hslot + g * GB;
                    const char* ga = gb + KS * 1024;
                    const int r0 = 16 * (GPS * hst + g), nr = min(16, p_nrows - r0);
                    i32x4 pacc[QB];
                    group_dots(gb, pacc);
                    float4 ax[4];
                    row_terms(ga, ax);
#pragma unroll
                    for (int qb = 0; qb < QB; ++qb) {
                        const int qi = wq0 + qb * 16 + col;
                        const float4 qc = s_qc[qi];
                        // one precise bound per lane: of its 4 rows the one whose approximate score is best
                        // (any row's lower bound is a valid pilot key; the bound is ≈ 40 VALU, the pick 3 per row:
                        // DOT / MIP / COSINE I·a_r, EUCLIDEAN 2·I·a_r·s_q − |x|²)
                        // (the chosen row's operands carried along as selects: an index into ax[] put it in scratch)
                        int rb = 0, ib = pacc[qb][0];
                        float4 axb = ax[0];
                        float vb = -__builtin_inff();
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const float ia = (float)pacc[qb][r] * ax[r].x;
                            float v = SIM == SIM_EUCLIDEAN ? fmaf(2.0f * ia, qc.x, -ax[r].w) : ia;
                            if (!(4 * grp + r < nr)) v = -__builtin_inff();
                            const bool take = v > vb;
                            vb = take ? v : vb;
                            rb = take ? r : rb;
                            ib = take ? pacc[qb][r] : ib;
                            axb.x = take ? ax[r].x : axb.x;
                            axb.y = take ? ax[r].y : axb.y;
                            axb.z = take ? ax[r].z : axb.z;
                            axb.w = take ? ax[r].w : axb.w;
                        }
                        uint64_t best = 0ull;
                        {
                            const int rr = 4 * grp + rb;
                            float xnd = 0.0f;
                            if constexpr (SIM == SIM_COSINE) xnd = *reinterpret_cast<const float*>(ga + 288 + rr * 4);
                            float lo, hi;
                            sq8_bounds(sim, (float)ib, axb, qc, s_cold.gam, s_cold.g2, lo, hi);
                            const float lb = SIM == SIM_EUCLIDEAN ? score_f32_l2(hi) : score_f32(sim, lo, qnd[qb], xnd);
                            best = vb > -__builtin_inff() ? make_key(lb, hd.vrow0 + (uint32_t)(r0 + rr)) : 0ull;
                        }
#pragma unroll
                        for (int o = 16; o <= 32; o <<= 1) {
                            const uint64_t other = ((uint64_t)(uint32_t)__shfl_xor((int)(best >> 32), o) << 32) |
                                                   (uint32_t)__shfl_xor((int)(uint32_t)best, o);
                            best = other > best ? other : best;
                        }
                        pbest[qb] = best > pbest[qb] ? best : pbest[qb];
                    }
                }
                if (pst + 1 < p_steps) continue;   // (the quarter's last pilot step writes its keys)
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) {
                    const int qi = wq0 + qb * 16 + col;
                    if (grp == 0 && qi < s_cold.q_count && !(ablate & 16))
                        s_cold.pilot_keys[(size_t)qi * s_cold.n_quarters + hd.list] = pbest[qb];
                    // the two-pass main pass reads the second pass's list maxima as empty until it writes them
                    if (grp == 0 && qi < s_cold.q_count)
                        s_cold.list_lbmax[(size_t)(s_cold.q0 + qi) * s_cold.n_lists + hd.list] = 0u;
                }
                continue;
            }
            // read and multiply the step: every LDS read of a group's A fragments, then its KS·QB MFMAs as
            // straight-line code (≤ 256 dims: every group's reads first, one exposed LDS latency per step)
#pragma unroll
            for (int g = 0; g < GPS; ++g)
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) acc[g][qb] = i32x4{0, 0, 0, 0};
            if (ablate & 2) {
#pragma unroll
                for (int g = 0; g < GPS; ++g)
#pragma unroll
                    for (int s = 0; s < KS; ++s)
                        acc[g][0] ^= *reinterpret_cast<const i32x4*>(hslot + g * GB + s * 1024 + lane * 16);
            } else if constexpr (KS <= 4) {
                i32x4 a[GPS][KS];
#pragma unroll
                for (int g = 0; g < GPS; ++g)
#pragma unroll
                    for (int s = 0; s < KS; ++s) a[g][s] = *reinterpret_cast<const i32x4*>(hslot + g * GB + s * 1024 + lane * 16);
#pragma unroll
                for (int g = 0; g < GPS; ++g)
#pragma unroll
                    for (int s = 0; s < KS; ++s)
#pragma unroll
                        for (int qb = 0; qb < QB; ++qb)
                            acc[g][qb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[g][s], bfr[s][qb], acc[g][qb], 0, 0, 0);
            } else {
#pragma unroll
                for (int g = 0; g < GPS; ++g) group_dots(hslot + g * GB, acc[g]);
            }
            if (ablate & 1) {
                if (acc[0][0][0] + acc[GPS - 1][QB - 1][3] == 0x7FFFFFFF && bm.x == 1.0f) s_lp[tid] = 1u;
                continue;
            }
            quick_phase();
        }
        vm_wait<0>();
#ifdef OSK_TESTING
        cyc_loop += clock64() - c_loop0;
#endif
        if (pq >= 0 && !pilot) {
            if (qn) drain(s_quart[pq]);
            flush(s_quart[pq]);
        }
    }
#ifdef OSK_TESTING
    if (!pilot && p.counters) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) n_pairs += __shfl_xor(n_pairs, o);
        if (lane == 0) {
            atomicAdd(&p.counters[4], (unsigned long long)n_events);
            atomicAdd(&p.counters[5], (unsigned long long)n_pairs);
            atomicAdd(&p.counters[7], (unsigned long long)n_slow);
            if (wave == 0) {
                atomicAdd(&p.counters[6], (unsigned long long)cyc_wait);
                atomicAdd(&p.counters[8], (unsigned long long)cyc_loop);
                atomicAdd(&p.counters[9], (unsigned long long)cyc_slow);
                atomicAdd(&p.counters[10], (unsigned long long)cyc_drain);
            }
        }
    }
#endif
}

// ------------------------------------------------------------------------------------------------
// sq8_wide_rows — the wide prefilter for rows of ≤ 128 dims (KS = 2) with no step barrier.
//
// sq8_wide shares each LDS ring slot between its 8 waves (each wave owns 32 queries and reads every row of
// the step), so one barrier per 128-row step couples them: a step in which one wave takes the slow path holds
// all eight, and at C4 most steps hold one (18 % of wave-steps are slow; DESIGN.md §3g: barrier waits 29 %
// of wave 0's loop).  Here the roles are transposed: each wave owns ROWS — 16-row group g of a quarter goes
// to wave g mod 8 — and multiplies them against ALL 256 queries, whose B fragments it keeps in VGPRs for the
// launch (2 slabs × 16 query blocks × 4 = 128 VGPRs, which is why only KS = 2 takes this kernel).  A wave
// streams its own groups through its own LDS-DMA ring (kRowsNR groups deep: ≈ 68 KB in flight per CU, what
// HBM needs under load — a first version loaded 2 groups ahead into VGPRs, 34 KB per CU, and streamed at
// 3 TB/s) and reads them back as the A operand (the tiled copy is lane-linear: a 1 KiB slab IS the operand);
// it waits only on its own DMAs, never for another wave inside a quarter.
//   * the quick test per (group, query block) is sq8_wide's fast test (quick_consts: relaxed to the quarter's
//     row maxima), its per-(query, quarter) constants in an LDS table computed once per quarter;
//   * a passing (group, query block) runs the per-row test and appends each passing pair {int32 dot,
//     row << 8 | query} to the queue of the wave that OWNS the query (wave w owns queries 32w … 32w + 31:
//     their lists, floors and flush), one LDS atomic per block for the slots;
//   * at the quarter's end (two barriers per quarter, ≈ 1,000 groups at C4) each wave drains its queue —
//     precise bounds, floor, list appends or the ordered insertion, exactly sq8_wide's deferred drain — and
//     flushes its queries' lists for the settle.  A queue that fills drops its further entries and marks
//     their (quarter, query) lists for an exact re-scan by the settle (16th key above every threshold).
// Same lists, floors and settle contract as sq8_wide, so results are bit-identical (tests/test_gpu_wide.py).
// ------------------------------------------------------------------------------------------------
constexpr int kRowsNR = 6;      // groups in flight per wave: its LDS-DMA ring's slots
constexpr int kRowsQB = 4;      // query blocks per accumulator pass (4 passes of 4 over the 16 blocks)
constexpr int kRowsSlot = 2048 + 5 * 16;   // a ring slot: the group's 2 slabs, then 5 bound-term float4 (rows_issue)
constexpr int kRowsMaxFloorShards = 8;     // (per-(shard, query) floors in LDS up to this many shards)

// a pointer every lane of the wave holds alike (read from LDS), as SGPRs
__device__ __forceinline__ const char* rfl_ptr_c(const void* ptr) {
    const uint64_t v = (uint64_t)ptr;
    return (const char*)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v));
}

template <int SIM, bool PILOT>
__global__ __launch_bounds__(kWideThreads, 1) void sq8_wide_rows(Sq8Params p) {
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    constexpr int NQB = kWideQ / 16, NR = kRowsNR, PB = kRowsQB;
    static_assert(PB == 2 || PB == 4, "passes of 2 or 4 query blocks");
    constexpr int sim = SIM;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int col = lane & 15, grp = lane >> 4;
    const int u8 = p.units8, S = p.n_shards;
#ifdef OSK_TESTING
    // A/B timing only (results wrong): 1 skip each group's work (streaming alone), 2 the MFMAs replaced by XORs,
    // 4 skip the slow path, 8 MFMAs without the fast test (their results consumed by one max)
    const int ablate = p.ablate;
#else
    constexpr int ablate = 0;
#endif
    const int G = gridDim.x, n_quarters = 4 * p.n_tiles;
    const int qbeg = p.quarter_begin, n_range = (p.quarter_end > 0 ? p.quarter_end : n_quarters) - qbeg;
    const int n_mine = (int)blockIdx.x < n_range ? (n_range - 1 - (int)blockIdx.x) / G + 1 : 0;
    const bool floor_lds = S <= kRowsMaxFloorShards;
    // the deferred queues, qcap entries per owner wave (launch_sq8_wide_rows: what LDS leaves; tests less): one
    // sub-queue per (owner, producer) wave pair, sub = qcap / 16 entries each, which a producer appends to at
    // its own count (no atomics), and the other half a pool per owner for what a producer's sub-queue cannot
    // hold (one LDS atomic per overflowing event) — a heavy quarter for one producer no longer drops entries
    // while the owner's other sub-queues stand empty
    const int qcap = p.wide_qcap, sub = p.wide_qcap / (2 * kWideWaves), pool = p.wide_qcap - kWideWaves * sub;
    const bool claim_dyn = p.wide_claim != 0;
#ifdef OSK_TESTING
    const uint64_t t_start = clock64();
    uint64_t cyc_setup = 0, cyc_qend = 0, cyc_first = 0;
#endif

    // (the fixed-size arrays are static LDS: their addresses are constants, so the hot loop's LDS accesses take
    // immediate offsets instead of address registers; the rings, queues, quarter descriptors and floors are the
    // dynamic part)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ WideCold s_cold;
    __shared__ __attribute__((aligned(16))) float4 s_qc[kWideQ];   // query bound terms
    __shared__ __attribute__((aligned(16))) float s_ca[kWideQ];    // [16 col][16 qb] quick-test constants
    __shared__ __attribute__((aligned(16))) float s_cb[kWideQ];    // (EUCLIDEAN's second constant)
    __shared__ float s_qnd[kWideQ];                        // |q|² device order (COSINE)
    __shared__ int32_t s_cnt[kWideQ];                      // list fill
    __shared__ int32_t s_ovf[kWideQ];                      // queue overflowed this quarter
    __shared__ int32_t s_qn[kWideWaves * kWideWaves];      // [owner][producer] queue fill (published at quarter end)
    __shared__ int32_t s_qo[kWideWaves];                   // [owner] pool fill
    __shared__ int32_t s_next;                             // the quarter's next unclaimed group
    char* s_ring = smem;                                                                   // [8 waves][NR] slots
    // the lists [kWideQ][kKQ] keys + lower bounds (48 KB) overlay the rings: they live only in the quarter-end
    // drain and flush, when no DMA is in flight (a quarter's items are issued inside the quarter only)
    uint64_t* s_lk = reinterpret_cast<uint64_t*>(smem);
    uint32_t* s_lp = reinterpret_cast<uint32_t*>(s_lk + kWideQ * kKQ);
    WideQuarter* s_quart = reinterpret_cast<WideQuarter*>(smem + kWideWaves * NR * kRowsSlot);   // [n_mine]
    uint2* s_q = reinterpret_cast<uint2*>(s_quart + n_mine);                             // [8 owners][8 × sub + pool]
    uint32_t* s_floor = reinterpret_cast<uint32_t*>(s_q + kWideWaves * qcap);           // [S][kWideQ] (S ≤ 8)
    if (tid == 0) s_cold = WideCold{p.cand, p.cand_lb, p.list_lbmax, p.visited, p.qn_dev, p.pilot_keys, p.floors, p.q0,
                                    p.n_lists, p.q_count, 4 * p.n_tiles, p.cos_slack, p.gam, p.g2};
    for (int i = tid; i < kWideQ; i += kWideThreads) {
        s_cnt[i] = 0;
        s_ovf[i] = 0;
        s_qc[i] = i < p.q_count ? p.qc[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        s_qnd[i] = (SIM == SIM_COSINE && i < p.q_count) ? p.qn_dev[i] : 0.0f;
    }
    if (tid < kWideWaves * kWideWaves) s_qn[tid] = 0;
    if (tid < kWideWaves) s_qo[tid] = 0;
    if (floor_lds)
        for (int i = tid; i < S * kWideQ; i += kWideThreads) {
            const int qi = i % kWideQ;
            s_floor[i] = (!p.floors || qi >= p.q_count) ? 0u : p.floors[(size_t)qi * S + i / kWideQ];
        }
    for (int i = tid; i < n_mine; i += kWideThreads) {
        const int j = qbeg + (int)blockIdx.x + i * G;
        WideQuarter d = p.wide_qtable ? static_cast<const WideQuarter*>(p.wide_qtable)[j]
                                      : wide_quarter_of(p.tiles, p.tile_order, j, 2, p.rows8t, p.auxt, p.seg_vrow,
                                                        p.quarter_bm);
        if (PILOT) d.nrows = min(d.nrows, p.pilot_rows > 0 ? p.pilot_rows : kWidePilotRows);   // (its first rows)
        s_quart[i] = d;
    }
    // the pilot's per-query best key of the current quarter (the queues' LDS: the pilot has none)
    uint64_t* s_pk = reinterpret_cast<uint64_t*>(s_q);
    if (PILOT)
        for (int i = tid; i < kWideQ; i += kWideThreads) s_pk[i] = 0ull;
    // the launch's query fragments: query block qb, slab s (lane: query qb·16 + col, 16-B unit 4s + grp)
    i32x4 bfr[2][NQB];
#pragma unroll
    for (int qb = 0; qb < NQB; ++qb) {
        const int qi = qb * 16 + col;
        const bool qv = qi < p.q_count;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int f = s * 4 + grp;
            const int4 v = (qv && f < u8) ? p.q8[(int64_t)qi * u8 + f] : make_int4(0, 0, 0, 0);
            bfr[s][qb] = i32x4{v.x, v.y, v.z, v.w};
        }
    }
    const int wq0 = wave * 32;   // this wave owns queries wq0 … wq0 + 31 (their lists, queue and flush)
    auto floor_of = [&](int qi, int sh) -> uint32_t {
        const WideCold& c = s_cold;
        return floor_lds ? s_floor[sh * kWideQ + qi] : ((!c.floors || qi >= c.q_count) ? 0u : c.floors[(size_t)qi * S + sh]);
    };
    __syncthreads();   // lists zeroed; s_qc, s_qnd, the floors and the quarter descriptors written
#ifdef OSK_TESTING
    const uint64_t t_bar = clock64();
#endif
#pragma unroll
    for (int qb = 0; qb < NQB; ++qb)
#pragma unroll
        for (int s = 0; s < 2; ++s) asm volatile("" ::"v"(bfr[s][qb]));
#ifdef OSK_TESTING
    const uint64_t t_frag = clock64();
#endif

    // ---- the quarter-end work: drain this wave's queue into its queries' lists, then flush them ----
    auto drain_flush = [&](const WideQuarter& d) {
        const WideCold& c = s_cold;
        if constexpr (PILOT) {   // the quarter's best key per query → pilot_keys; its list maximum zeroed (the
                                 // two-pass main pass reads the second pass's lists as empty until it writes them)
            if (lane < 32) {
                const int qi = wq0 + lane;
                if (qi < c.q_count) {
                    c.pilot_keys[(size_t)qi * c.n_quarters + d.list] = s_pk[qi];
                    c.list_lbmax[(size_t)(c.q0 + qi) * c.n_lists + d.list] = 0u;
                }
                s_pk[qi] = 0ull;
            }
            return;
        }
        const int sh = d.shard;
        for (int i = lane; i < 32 * kKQ; i += 64) {   // this wave's queries' lists (ring memory: zero them first)
            s_lk[wq0 * kKQ + i] = 0ull;
            s_lp[wq0 * kKQ + i] = 0u;
        }
        // this owner's entries: producer p's sub-queue holds cnt[p] of them; entry e of the concatenation is found
        // by the producers' running offsets (8 scalar compares per lane)
        int off[kWideWaves + 1];
        off[0] = 0;
#pragma unroll
        for (int pw = 0; pw < kWideWaves; ++pw)
            off[pw + 1] = off[pw] + min(__builtin_amdgcn_readfirstlane(s_qn[wave * kWideWaves + pw]), sub);
        const int n_sub = off[kWideWaves];
        const int n = n_sub + min(__builtin_amdgcn_readfirstlane(s_qo[wave]), pool);   // (then the pool's)
        const uint2* q = s_q + (size_t)wave * qcap;
        for (int i0 = 0; i0 < n; i0 += 64) {
            const int e = i0 + lane;
            const bool ok = e < n;
            int pw = 0;
#pragma unroll
            for (int w = 1; w < kWideWaves; ++w) pw += e >= off[w];
            const int qx = e < n_sub ? pw * sub + (e - off[pw]) : kWideWaves * sub + (e - n_sub);
            const uint2 en = ok ? q[qx] : make_uint2(0u, 0u);
            const int qi = (int)(en.y & 255u), rowq = (int)(en.y >> 8);
            const float* af = reinterpret_cast<const float*>(d.at + (rowq >> 4) * kAuxGroupF4);
            const int rr = rowq & 15;
            uint64_t key = 0ull;
            uint32_t lbs = 0u;
            bool ovf = false;
            if (ok) {
                const float a_r = SIM == SIM_COSINE ? af[68] : af[rr];   // (COSINE: the group's s_g, slot 17)
                const float4 ax = make_float4(a_r, af[16 + rr], af[32 + rr], af[48 + rr]);
                const float xnd = SIM == SIM_COSINE ? af[72 + rr] : 0.0f;
                const float qndq = s_qnd[qi];
                float lo, hi;
                sq8_bounds(sim, (float)(int32_t)en.x, ax, s_qc[qi], c.gam, c.g2, lo, hi);
                const float ub = SIM == SIM_EUCLIDEAN ? score_f32_l2(lo) : score_f32(sim, hi, qndq, xnd);
                const float lb = SIM == SIM_EUCLIDEAN ? score_f32_l2(hi) : score_f32(sim, lo, qndq, xnd);
                const uint64_t kr = make_key(ub, d.vrow0 + (uint32_t)rowq);
                const uint64_t tk = (uint64_t)floor_of(qi, sh) << 32;
                if (kr > tk) {   // below the floor: cannot enter the top k
                    const int pos = atomicAdd(&s_cnt[qi], 1);
                    if (pos < kKQ - 1) {
                        s_lk[qi * kKQ + pos] = kr;
                        s_lp[qi * kKQ + pos] = float_to_sortable(lb);
                    } else {
                        key = kr;
                        lbs = float_to_sortable(lb);
                        ovf = true;
                    }
                }
            }
            uint64_t om = __ballot(ovf);
            while (om) {   // the overflowed queries, one at a time: sq8_wide's ordered insertion
                const int Q = __builtin_amdgcn_readlane(qi, (int)__builtin_ctzll(om));
                const int o0 = Q * kKQ;
                uint64_t lkb = lane < kKQ ? s_lk[o0 + lane] : 0ull;
                uint32_t lpb = lane < kKQ ? s_lp[o0 + lane] : 0u;
                if (s_cnt[Q] < kWideSorted) {   // first overflow: sort the appended rows (zeros last)
                    int rank = 0;
#pragma unroll 2
                    for (int j = 0; j < kKQ; ++j) {
                        const uint64_t kj = s_lk[o0 + j];
                        rank += (kj > lkb) || (kj == lkb && j < lane);
                    }
                    if (lane < kKQ) {
                        s_lk[o0 + rank] = lkb;
                        s_lp[o0 + rank] = lpb;
                    }
                    lkb = lane < kKQ ? s_lk[o0 + lane] : 0ull;
                    lpb = lane < kKQ ? s_lp[o0 + lane] : 0u;
                }
                uint64_t thrb = readlane64(lkb, kKQ - 1);
                wave_offer2(key, lbs, ovf && qi == Q, lkb, lpb, thrb, lane, kKQ);
                if (lane < kKQ) {
                    s_lk[o0 + lane] = lkb;
                    s_lp[o0 + lane] = lpb;
                }
                if (lane == 0) s_cnt[Q] = kWideSorted;
                om = __ballot(ovf && qi != Q);
                ovf = ovf && qi != Q;
            }
        }
        // flush: this wave's queries, 4 per pass of 16 lanes → the settle's arrays, zeroed.  A query whose queue
        // entries were dropped (s_ovf) gets a 16th key above every threshold: the settle re-scans the quarter
        // exactly for it (its list maximum at least score 0, so the settle does not skip the list)
        const int q_end = min(wq0 + 32, c.q_count);
        for (int q0 = wq0; q0 < q_end; q0 += 4) {
            const int qg = q0 + (lane >> 4), e = lane & 15;
            uint64_t lkb = s_lk[qg * kKQ + e];
            const uint32_t lpb = s_lp[qg * kKQ + e];
            const bool dropped = s_ovf[qg] != 0;
            if (dropped && e == kKQ - 1) lkb = 0xFFFFFFFF00000000ull;
            uint32_t m = (lkb && lkb != 0xFFFFFFFF00000000ull) ? lpb : 0u;
#pragma unroll
            for (int o = 8; o >= 1; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
            if (dropped) m = max(m, 0x80000000u);   // (sortable score 0: a lower bound of any row)
            if (qg < q_end) {
                const size_t l = (size_t)(c.q0 + qg) * c.n_lists + d.list;
                c.cand[l * kKQ + e] = lkb;
                c.cand_lb[l * kKQ + e] = lpb;
                if (e == 0) c.list_lbmax[l] = m;
                if (e == 0) {
                    s_cnt[qg] = 0;
                    s_ovf[qg] = 0;
                }
            }
        }
        if (lane < kWideWaves) s_qn[wave * kWideWaves + lane] = 0;
        if (lane == 0) s_qo[wave] = 0;
        if (c.visited && c.q0 == 0 && tid == 0 && d.nrows > 0)
            atomicAdd(&c.visited[d.seg], (unsigned long long)d.nrows);
    };
    // ---- a quarter starts: its quick-test constants for every query, each wave its own 32 (lanes 0..31) ----
    auto begin_quarter = [&](const WideQuarter& d) {
        if (tid == 0) s_next = 0;   // (read after the barrier that follows)
        if (!PILOT && lane < 32) {
            const int oq = wq0 + lane;
            float ca, cb = 0.0f;
            if (oq < s_cold.q_count) {
                const float4 qc = s_qc[oq];   // sq8_wide's per-query coefficients, exactly
                const float sb = qc.x;
                const float inv = qc.x > 0.0f ? (SIM == SIM_EUCLIDEAN ? 0.5f : 1.0f) / qc.x : 0.0f;
                const float zq = qc.x > 0.0f ? qc.z / qc.x * (1.0f + 0x1p-20f) : 0.0f;
                float QY, QZ, Q0;
                if constexpr (SIM == SIM_EUCLIDEAN) {
                    const double m = 0x1p-17;
                    QY = __double2float_ru((2.0 + 2.0 * m) * (double)qc.y + 2.0 * m * (double)qc.z);
                    QZ = __double2float_ru((2.0 + 2.0 * m) * (double)qc.z);
                    Q0 = __double2float_rd((double)qc.w * (1.0 - m));
                } else {
                    const double r = 1.0 + 0x1p-18;
                    QY = __double2float_ru(((double)qc.y + 0x1p-18 * (double)qc.z) * r);
                    QZ = __double2float_ru((double)qc.z * r);
                    Q0 = __double2float_ru((double)s_cold.gam * (double)qc.w * r);
                }
                const float QW = __double2float_ru((double)s_cold.gam * (1.0 + 0x1p-18));
                const float ig2m = 1.0f / (1.0f - s_cold.g2);
                const uint64_t tkey = (uint64_t)floor_of(oq, d.shard) << 32;
                const float tq = sq8_quick(sim, tkey, SIM == SIM_COSINE ? sqrtf(s_qnd[oq]) : 0.0f, s_cold.cos_slack);
                quick_consts<SIM>(tq, sb, inv, QY, QZ, Q0, QW, zq, ig2m, d.bm, ca, cb);
            } else if (SIM == SIM_EUCLIDEAN) {   // (no query: no pair passes)
                ca = 0.0f;
                cb = __builtin_inff();
            } else {
                ca = __builtin_inff();
            }
            s_ca[(oq & 15) * 16 + (oq >> 4)] = ca;
            if (SIM == SIM_EUCLIDEAN) s_cb[(oq & 15) * 16 + (oq >> 4)] = cb;
        }
    };
    // empty quarters take no group, but the settle and the floors read every (query, quarter) slot
    for (int q = 0; q < n_mine; ++q)
        if (__builtin_amdgcn_readfirstlane(s_quart[q].nrows) <= 0) drain_flush(s_quart[q]);   // (all empty here)

#ifdef OSK_TESTING
    uint32_t n_events = 0, n_pairs = 0, n_slow = 0;
#endif
    // ---- the wave's items: per nonempty quarter, its groups wave, wave + 8, … — issued kRowsNR ahead through the
    // wave's ring, never past the quarter's end (the lists overlay the rings in the quarter-end drain) ----
    auto groups_of = [&](int q) { return __builtin_amdgcn_readfirstlane((s_quart[q].nrows + 15) >> 4); };
    // this wave's ring: slot d at ring_base + d·kRowsSlot (LDS byte address for the DMAs, pointer for the reads)
    const uint32_t ring_lds = __builtin_amdgcn_readfirstlane(
        (uint32_t)(size_t)(__attribute__((address_space(3))) char*)smem + (uint32_t)(wave * NR * kRowsSlot));
    const char* ring = s_ring + wave * NR * kRowsSlot;
    const int4* c_xt = nullptr;
    const float4* c_at = nullptr;
    int c_ng = 0, c_nrows = 0;   // (the quarter's groups and rows, in SGPRs)
    uint32_t c_vrow0 = 0;        // (the pilot: the quarter's first view row)
    // group g's DMAs into slot d — the two 1 KiB slabs (lane-linear: the A operand), and 5 bound-term float4:
    // lanes 0–3 the rows' |x|² (EUCLIDEAN, slots 12–15) or per-row factors (COSINE, slots 0–3), lane 4 slot 17
    // {s_g, f_cos, zero-row flag, 0}: three DMA instructions
    auto issue = [&](int d, int g) {
        const int4* xg = c_xt + (size_t)g * 128;
        const float4* ag = c_at + (size_t)g * kAuxGroupF4;
        const uint32_t base = ring_lds + (uint32_t)(d * kRowsSlot);
        glds16(xg + lane, base);
        glds16(xg + 64 + lane, base + 1024u);
        if (lane < 5) glds16(ag + (lane == 4 ? 17 : (SIM == SIM_EUCLIDEAN ? 12 : 0) + lane), base + 2048u);
    };
    int q_cnt[kWideWaves];   // this wave's entries per owner in the current quarter (wave-uniform)
#pragma unroll
    for (int o = 0; o < kWideWaves; ++o) q_cnt[o] = 0;
    auto publish = [&]() {   // the counts → s_qn (before the quarter-end barrier), reset
#pragma unroll
        for (int o = 0; o < kWideWaves; ++o) {
            if (lane == 0) s_qn[o * kWideWaves + wave] = q_cnt[o];
            q_cnt[o] = 0;
        }
    };
    // ... and group g's work, its data in slot d
    auto process = [&](int d, int g) {
        if constexpr (PILOT) {
            // per query block: the lane's 4 rows' dots, its row with the best approximate score bounded
            // precisely (sq8_bounds, as the drain does), the best of the group's 16 rows per query (grp lanes)
            // → an LDS max per query over the quarter's groups
            const int r0 = 16 * g, nr = min(16, c_nrows - r0);
            const char* sl = ring + d * kRowsSlot;
            const i32x4 A0 = *reinterpret_cast<const i32x4*>(sl + lane * 16);
            const i32x4 A1 = *reinterpret_cast<const i32x4*>(sl + 1024 + lane * 16);
            const float4* ag = c_at + (size_t)g * kAuxGroupF4;   // (the group's full terms, from L2 / HBM)
            const float sg = *reinterpret_cast<const float*>(sl + 2048 + 64);
            const float4 ta = SIM == SIM_COSINE ? make_float4(sg, sg, sg, sg) : ag[grp];
            const float4 ty = ag[4 + grp], tz = ag[8 + grp], tw = ag[12 + grp];
            const float4 tx = SIM == SIM_COSINE ? ag[18 + grp] : make_float4(0.f, 0.f, 0.f, 0.f);
            const float fa[4] = {ta.x, ta.y, ta.z, ta.w}, fy[4] = {ty.x, ty.y, ty.z, ty.w};
            const float fz[4] = {tz.x, tz.y, tz.z, tz.w}, fw[4] = {tw.x, tw.y, tw.z, tw.w};
            const float fx[4] = {tx.x, tx.y, tx.z, tx.w};
#pragma unroll
            for (int h = 0; h < NQB / PB; ++h) {
                i32x4 acc[PB];
#pragma unroll
                for (int j = 0; j < PB; ++j)
                    acc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A0, bfr[0][h * PB + j], i32x4{0, 0, 0, 0}, 0, 0, 0);
#pragma unroll
                for (int j = 0; j < PB; ++j)
                    acc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A1, bfr[1][h * PB + j], acc[j], 0, 0, 0);
#pragma unroll
                for (int j = 0; j < PB; ++j) {
                    const int qi = (h * PB + j) * 16 + col;
                    const float4 qc = s_qc[qi];
                    int rb = 0, ib = acc[j][0];
                    float vb = -__builtin_inff(), ab = fa[0], yb = fy[0], zb = fz[0], wb = fw[0], xb = fx[0];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float ia = (float)acc[j][r] * fa[r];
                        float v = SIM == SIM_EUCLIDEAN ? fmaf(2.0f * ia, qc.x, -fw[r]) : ia;
                        if (!(4 * grp + r < nr)) v = -__builtin_inff();
                        const bool take = v > vb;
                        vb = take ? v : vb;
                        rb = take ? r : rb;
                        ib = take ? acc[j][r] : ib;
                        ab = take ? fa[r] : ab;
                        yb = take ? fy[r] : yb;
                        zb = take ? fz[r] : zb;
                        wb = take ? fw[r] : wb;
                        xb = take ? fx[r] : xb;
                    }
                    float lo, hi;
                    sq8_bounds(sim, (float)ib, make_float4(ab, yb, zb, wb), qc, s_cold.gam, s_cold.g2, lo, hi);
                    const float lb = SIM == SIM_EUCLIDEAN ? score_f32_l2(hi) : score_f32(sim, lo, s_qnd[qi], xb);
                    uint64_t key = (vb > -__builtin_inff() && qi < s_cold.q_count)
                                       ? make_key(lb, c_vrow0 + (uint32_t)(r0 + 4 * grp + rb)) : 0ull;
#pragma unroll
                    for (int o = 16; o <= 32; o <<= 1) {
                        const uint64_t other = ((uint64_t)(uint32_t)__shfl_xor((int)(key >> 32), o) << 32) |
                                               (uint32_t)__shfl_xor((int)(uint32_t)key, o);
                        key = other > key ? other : key;
                    }
                    if (grp == 0 && key) atomicMax(reinterpret_cast<unsigned long long*>(&s_pk[qi]),
                                                   (unsigned long long)key);
                }
            }
            return;
        }
        if (!(ablate & 1)) {
            const int r0 = 16 * g, nr = min(16, c_nrows - r0);
            // every LDS read of the item at once (one wait): the A operand, the group's terms, the query constants
            const char* sl = ring + d * kRowsSlot;
            const i32x4 A0 = *reinterpret_cast<const i32x4*>(sl + lane * 16);
            const i32x4 A1 = *reinterpret_cast<const i32x4*>(sl + 1024 + lane * 16);
            const float4 g17 = *reinterpret_cast<const float4*>(sl + 2048 + 64);   // {s_g, f_cos, zero-row flag, 0}
            const float4 xr4 = *reinterpret_cast<const float4*>(sl + 2048 + grp * 16);   // EUCLIDEAN |x|², COSINE factors
            // the pass's query constants (PB blocks: one ds_read_b128 / b64 each)
            auto consts = [&](int h, float (&cav)[PB], float (&cbv)[PB]) __attribute__((always_inline)) {
                if constexpr (PB == 4) {
                    const float4 cq = *reinterpret_cast<const float4*>(s_ca + col * 16 + h * PB);
                    cav[0] = cq.x, cav[1] = cq.y, cav[2] = cq.z, cav[3] = cq.w;
                    cbv[0] = cbv[1] = cbv[2] = cbv[3] = 0.0f;
                } else {
                    const float2 cq = *reinterpret_cast<const float2*>(s_ca + col * 16 + h * PB);
                    cav[0] = cq.x, cav[1] = cq.y;
                    cbv[0] = cbv[1] = 0.0f;
                }
                if constexpr (SIM == SIM_EUCLIDEAN) {
                    if constexpr (PB == 4) {
                        const float4 bq = *reinterpret_cast<const float4*>(s_cb + col * 16 + h * PB);
                        cbv[0] = bq.x, cbv[1] = bq.y, cbv[2] = bq.z, cbv[3] = bq.w;
                    } else {
                        const float2 bq = *reinterpret_cast<const float2*>(s_cb + col * 16 + h * PB);
                        cbv[0] = bq.x, cbv[1] = bq.y;
                    }
                }
            };
            // the group's factor: DOT / MIP / EUCLIDEAN s_g (every valid row's a_r: one scale per group), COSINE f_cos
            const float f = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(SIM == SIM_COSINE ? g17.y : g17.x)));
            bool zg = false;
            if constexpr (SIM == SIM_COSINE) zg = __builtin_amdgcn_readfirstlane(__float_as_int(g17.z)) != 0;
            // a pass of PB query blocks: their dots (2 chained MFMAs each)
            auto dots = [&](int h, i32x4 (&acc)[PB]) __attribute__((always_inline)) {
                if (!(ablate & 2)) {
#pragma unroll
                    for (int j = 0; j < PB; ++j)
                        acc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A0, bfr[0][h * PB + j], i32x4{0, 0, 0, 0}, 0, 0, 0);
#pragma unroll
                    for (int j = 0; j < PB; ++j)
                        acc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A1, bfr[1][h * PB + j], acc[j], 0, 0, 0);
                } else {
#pragma unroll
                    for (int j = 0; j < PB; ++j) acc[j] = (A0 ^ bfr[0][h * PB + j]) + (A1 ^ bfr[1][h * PB + j]);
                }
            };
            // the fast test: per block the lane's largest dot against the group's common factor (DOT / MIP:
            // s_g; COSINE: f_cos, a c ≤ 0 lets every pair through, as does a zero row) — sq8_wide's test.
            // EUCLIDEAN: the per-row test I_r·s_g ≥ w_r·ca + cb itself, t = max_r fma(I_r, s_g, −fma(w_r, ca, cb)) —
            // the score 2·x·q − |x|² is a small difference of large terms, and relaxing the lane's four rows to
            // (max I, min w) let every group through at C2 (uniform [0,1) coordinates: rows 4.000 slow passes of 4).
            // All 16 blocks first, ONE vote per group (no branch between the passes: the next pass's MFMAs overlap
            // this pass's tests); a passing pass recomputes its dots and tests in the slow path.
            auto tests = [&](const i32x4 (&acc)[PB], const float (&cav)[PB], const float (&cbv)[PB], float (&tf)[PB])
                __attribute__((always_inline)) {
#pragma unroll
                for (int j = 0; j < PB; ++j) {
                    const i32x4& I = acc[j];
                    if constexpr (SIM == SIM_EUCLIDEAN) {
                        tf[j] = fmaxf(fmaxf(fmaf((float)I[0], f, -fmaf(xr4.x, cav[j], cbv[j])),
                                            fmaf((float)I[1], f, -fmaf(xr4.y, cav[j], cbv[j]))),
                                      fmaxf(fmaf((float)I[2], f, -fmaf(xr4.z, cav[j], cbv[j])),
                                            fmaf((float)I[3], f, -fmaf(xr4.w, cav[j], cbv[j]))));
                    } else {
                        const int M = max(max(I[0], I[1]), max(I[2], I[3]));
                        float c = cav[j];
                        if constexpr (SIM == SIM_COSINE) c = !(cav[j] > 0.0f) ? -__builtin_inff() : cav[j];
                        tf[j] = fmaf((float)M, f, -c);
                    }
                }
            };
            float hm[NQB / PB];   // per pass, the lane's largest test value
#pragma unroll
            for (int h = 0; h < NQB / PB; ++h) {
                i32x4 acc[PB];
                float cav[PB], cbv[PB], tf[PB];
                dots(h, acc);
                if (ablate & 8) {   // (A/B: the MFMAs alone)
                    int m = acc[0][0];
#pragma unroll
                    for (int j = 1; j < PB; ++j) m = max(m, acc[j][j & 3]);
                    hm[h] = (float)m;
                    continue;
                }
                consts(h, cav, cbv);
                tests(acc, cav, cbv, tf);
                float m = tf[0];
#pragma unroll
                for (int j = 1; j < PB; ++j) m = fmaxf(m, tf[j]);
                hm[h] = m;
            }
            float run = hm[0];
#pragma unroll
            for (int h = 1; h < NQB / PB; ++h) run = fmaxf(run, hm[h]);
            if (ablate & 12) {
                if (run == 1.2345f) s_ovf[0] = 1;   // (keeps the work)
            } else if (__ballot(!(run < 0.0f)) || zg) {
                // the slow path: per passing block the per-row test, then the passing pairs → the owner's queue
                const float4 arow = SIM == SIM_COSINE ? xr4 : make_float4(f, f, f, f);   // the rows' factors
#pragma unroll
                for (int h = 0; h < NQB / PB; ++h) {
                    if (!__ballot(!(hm[h] < 0.0f)) && !zg) continue;
#ifdef OSK_TESTING
                    ++n_slow;
#endif
                    i32x4 acc[PB];
                    float cav[PB], cbv[PB], tf[PB];
                    consts(h, cav, cbv);
                    dots(h, acc);
                    tests(acc, cav, cbv, tf);
#pragma unroll
                    for (int j = 0; j < PB; ++j) {
                        const int qb = h * PB + j;
                        if (!__ballot(!(tf[j] < 0.0f) || zg)) continue;   // (invalid queries never pass: their c)
#ifdef OSK_TESTING
                        ++n_events;
#endif
                        // the lane's column and row group, opaque here: else the compiler hoists the (block, row)
                        // combinations of the enqueue's words and tests out of the loop as 64 per-lane constants,
                        // and at EUCLIDEAN (whose tests hold one more constant per query) spilled them to scratch —
                        // each reload a vmcnt(0), which drains the wave's DMA ring
                        int ocol = col, ogrp = grp;
                        __asm__ volatile("" : "+v"(ocol), "+v"(ogrp));
                        const int qi = qb * 16 + ocol;
                        const bool qv = qi < s_cold.q_count;
                        bool pass[4];
                        if constexpr (SIM == SIM_EUCLIDEAN) {   // the per-row test: t_r = fma(I, s_g, −fma(w_r, ca, cb))
                            const float wr[4] = {xr4.x, xr4.y, xr4.z, xr4.w};
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                pass[r] = !(fmaf((float)acc[j][r], f, -fmaf(wr[r], cav[j], cbv[j])) < 0.0f);
                        } else {
                            const float ar[4] = {arow.x, arow.y, arow.z, arow.w};
#pragma unroll
                            for (int r = 0; r < 4; ++r) pass[r] = !(fmaf((float)acc[j][r], ar[r], -cav[j]) < 0.0f);
                        }
                        bool pr[4];
                        uint64_t b[4];
                        int tot = 0;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            pr[r] = pass[r] && 4 * ogrp + r < nr && qv;
                            b[r] = __ballot(pr[r]);
                            tot += __popcll(b[r]);
                        }
                        if (!tot) continue;
                        const int owner = qb >> 1;   // (queries qb·16 … qb·16 + 15 belong to wave qb / 2)
                        const int own0 = q_cnt[owner];   // (this wave's sub-queue of the owner: no other writer)
                        int base = own0;
                        q_cnt[owner] += tot;
                        uint2* oq_ = s_q + (size_t)owner * qcap + (size_t)wave * sub;
                        // what the sub-queue cannot hold goes to the owner's pool, in the event's order
                        const int n_over = tot - min(tot, max(0, sub - own0));
                        int pbase = 0;
                        if (n_over) {
                            if (lane == 0) pbase = atomicAdd(&s_qo[owner], n_over);
                            pbase = __builtin_amdgcn_readfirstlane(pbase);
                        }
                        const int ovf0 = max(own0, sub);   // (the slot of the event's first pool entry)
                        uint2* pq_ = s_q + (size_t)owner * qcap + (size_t)kWideWaves * sub;
                        bool dropped = false;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(b[r] >> 32),
                                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)b[r], 0u));
                            const int slot = base + below;
                            if (pr[r]) {
                                const uint2 en = make_uint2((uint32_t)acc[j][r], (uint32_t)(r0 + 4 * ogrp + r) << 8 | (uint32_t)qi);
                                const int ps = pbase + (slot - ovf0);
                                if (slot < sub)
                                    oq_[slot] = en;
                                else if (ps < pool)
                                    pq_[ps] = en;
                                else
                                    dropped = true;
                            }
                            base += __popcll(b[r]);
                        }
                        if (dropped) s_ovf[qi] = 1;
#ifdef OSK_TESTING
                        if (lane == 0) n_pairs += tot;
#endif
                    }
                }
            }
        }
    };
    int cur = -1;
#ifdef OSK_TESTING
    cyc_setup = clock64() - t_start;
#endif
    for (int q = 0; q < n_mine; ++q) {
        if (groups_of(q) == 0) continue;   // (flushed above)
#ifdef OSK_TESTING
        const uint64_t t_q0 = clock64();
#endif
        // the quarter changes: the last one's drain + flush, this one's constants (two barriers; between them no
        // wave has a DMA in flight, so the lists may overlay the rings)
        if (cur >= 0) {
            publish();
            __syncthreads();
            drain_flush(s_quart[cur]);
        }
        begin_quarter(s_quart[q]);
        __syncthreads();
#ifdef OSK_TESTING
        cyc_qend += clock64() - t_q0;
#endif
        cur = q;
        c_nrows = __builtin_amdgcn_readfirstlane(s_quart[q].nrows);
        if (PILOT) c_vrow0 = __builtin_amdgcn_readfirstlane(s_quart[q].vrow0);
        c_ng = (c_nrows + 15) >> 4;
        c_xt = reinterpret_cast<const int4*>(rfl_ptr_c(s_quart[q].xt));
        c_at = reinterpret_cast<const float4*>(rfl_ptr_c(s_quart[q].at));
        // this wave's groups: claimed one at a time from the quarter's counter as a ring slot frees (p.wide_claim;
        // 0: the fixed interleave wave + 8i), so the 8 waves reach the quarter's end together whatever their
        // slow paths cost — a wave's claims increase, so the first claim past the quarter ends its work
        int n_claim = 0;
        auto claim = [&]() -> int {
            int g;
            if (claim_dyn) {
                g = 0;
                if (lane == 0) g = atomicAdd(&s_next, 1);
                g = __builtin_amdgcn_readfirstlane(g);
            } else {
                g = wave + kWideWaves * n_claim;
            }
            ++n_claim;
            return g;
        };
        int gs[NR];
        int issued = 0, done_items = 0;
#pragma unroll
        for (int d = 0; d < NR; ++d) {
            gs[d] = claim();
            if (gs[d] < c_ng) {
                issue(d, gs[d]);
                ++issued;
            }
        }
        bool more = issued > 0;
        while (more) {
#pragma unroll
            for (int d = 0; d < NR; ++d) {
                if (more) {
                    if (gs[d] >= c_ng) {
                        more = false;   // (claims increase: every later slot is past the quarter too)
                    } else {
                        // slot d's three DMAs have landed (the NR − 1 younger items' may not; at the quarter's
                        // tail fewer are younger: wait for all)
#ifdef OSK_TESTING
                        const uint64_t t_w0 = clock64();
#endif
                        if (issued - done_items - 1 >= NR - 1) vm_wait<(NR - 1) * 3>();
                        else vm_wait<0>();
#ifdef OSK_TESTING
                        if (done_items == 0) cyc_first += clock64() - t_w0;
#endif
                        process(d, gs[d]);
                        ++done_items;
                        gs[d] = claim();
                        if (gs[d] < c_ng) {
                            issue(d, gs[d]);
                            ++issued;
                        }
                    }
                }
            }
        }
    }
    vm_wait<0>();   // (no DMA is in flight past a quarter; kept: nothing may land after the workgroup retires)
    // the last quarter's drain and flush
#ifdef OSK_TESTING
    const uint64_t t_e0 = clock64();
#endif
    publish();
    __syncthreads();
    if (cur >= 0) drain_flush(s_quart[cur]);
#ifdef OSK_TESTING
    cyc_qend += clock64() - t_e0;
    if (!PILOT && p.counters && tid == 0) {
        atomicAdd(&p.counters[16], (unsigned long long)(clock64() - t_start));
        atomicAdd(&p.counters[17], (unsigned long long)cyc_setup);
        atomicAdd(&p.counters[18], (unsigned long long)cyc_qend);
        atomicAdd(&p.counters[19], (unsigned long long)cyc_first);
        atomicAdd(&p.counters[20], (unsigned long long)(t_bar - t_start));   // setup: to the first barrier
        atomicAdd(&p.counters[21], (unsigned long long)(t_frag - t_bar));    // then the fragments' arrival
    }
    if (p.counters) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) n_pairs += __shfl_xor(n_pairs, o);
        if (lane == 0) {
            atomicAdd(&p.counters[4], (unsigned long long)n_events);
            atomicAdd(&p.counters[5], (unsigned long long)n_pairs);
            atomicAdd(&p.counters[7], (unsigned long long)n_slow);
        }
    }
#endif
}

using WideFn = void (*)(Sq8Params);
#define OSK_WIDE_SIMS(KS) {sq8_wide<KS, 0>, sq8_wide<KS, 1>, sq8_wide<KS, 2>, sq8_wide<KS, 3>}
static const WideFn kWide[4][4] = {OSK_WIDE_SIMS(2), OSK_WIDE_SIMS(4), OSK_WIDE_SIMS(8), OSK_WIDE_SIMS(12)};
static_assert(sizeof(WideCold) <= 128, "WideCold: 128 B of static LDS reserved");

template <int KS>
static size_t wide_ring_bytes(int sim) {
    using Geo = WideGeom<KS>;
    return (size_t)Geo::NS * Geo::GPS * (KS * 1024 + (sim == SIM_COSINE ? kAuxGroupF4 : 18) * 16);
}
static size_t sq8_wide_lds(int ks, int sim, int n_shards, int n_mine) {
    const size_t ring = ks == 2 ? wide_ring_bytes<2>(sim) : ks == 4 ? wide_ring_bytes<4>(sim)
                      : ks == 8 ? wide_ring_bytes<8>(sim) : wide_ring_bytes<12>(sim);
    return ring + (size_t)kWideQ * kKQ * 12 + (size_t)kWideQ * 16 + (size_t)kWideQ * 4 +
           (n_shards <= kWideMaxFloorShards ? (size_t)n_shards * kWideQ * 4 : 0) + (size_t)n_mine * sizeof(WideQuarter);
}

using RowsFn = void (*)(Sq8Params);
static const RowsFn kWideRows[2][4] = {{sq8_wide_rows<0, false>, sq8_wide_rows<1, false>, sq8_wide_rows<2, false>,
                                        sq8_wide_rows<3, false>},
                                       {sq8_wide_rows<0, true>, sq8_wide_rows<1, true>, sq8_wide_rows<2, true>,
                                        sq8_wide_rows<3, true>}};
// dynamic LDS: the rings, the quarter descriptors and the floors (+ the queues, sized from what is left); the rest
// is static, kRowsStatic bytes
static size_t sq8_wide_rows_lds(int n_shards, int n_mine) {
    return (size_t)kWideWaves * kRowsNR * kRowsSlot + (size_t)n_mine * sizeof(WideQuarter) +
           (n_shards <= kRowsMaxFloorShards ? (size_t)n_shards * kWideQ * 4 : 0);
}
// the kernel's static LDS as compiled (hipFuncGetAttributes, once per kernel): a hand-kept estimate fell 160 B
// short when the queue counts grew to [8][8], so EUCLIDEAN's dynamic LDS (sized to fill the 160 KB) took the
// launch past the CU's LDS and the GPU faulted (round 6; found by tests/test_gpu_wide.py)
static size_t kernel_static_lds(const void* fn) {
    static std::mutex mu;
    static std::map<const void*, size_t> cache;
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(fn);
    if (it != cache.end()) return it->second;
    hipFuncAttributes a{};
    const size_t v = hipFuncGetAttributes(&a, fn) == hipSuccess ? a.sharedSizeBytes : (size_t)16 * 1024;   // (else: generous)
    cache[fn] = v;
    return v;
}
static_assert(kWideWaves * kRowsNR * kRowsSlot >= kWideQ * kKQ * 12, "the lists overlay the rings");
static constexpr int kRowsMinQcap = 128;   // deferred entries per owner wave at least (else more workgroups)
bool sq8_wide_rows_supported(int u8) { return sq8_wide_supported(u8) && sq8_wide_ks(u8) == 2; }

hipError_t launch_sq8_wide_rows(const Sq8Params& p, hipStream_t s, hipEvent_t ev_start, hipEvent_t ev_stop) {
    if (!sq8_wide_rows_supported(p.units8) || p.q_count < 1 || p.q_count > kWideQ || p.accept || p.gtiles ||
        p.sim < 0 || p.sim > 3 || !p.rows8t || !p.auxt || p.n_lists != 4 * p.n_tiles || p.k < 1 || p.k > kKQ ||
        p.n_shards < 1 || p.wide_grid < 1 || (p.pilot && !p.pilot_keys) || (!p.pilot && !p.quarter_bm))
        return hipErrorInvalidValue;
    const int nq4 = (p.quarter_end > 0 ? p.quarter_end : 4 * p.n_tiles) - p.quarter_begin;
    if (p.quarter_begin < 0 || nq4 < 1 || p.quarter_begin + nq4 > 4 * p.n_tiles || (p.quarter_begin && p.pilot))
        return hipErrorInvalidValue;
    int grid = std::min(p.wide_grid, std::max(1, nq4));
    const auto fn = kWideRows[p.pilot ? 1 : 0][p.sim];
    const size_t cap = 160 * 1024 - kernel_static_lds(reinterpret_cast<const void*>(fn));
    while (sq8_wide_rows_lds(p.n_shards, (nq4 + grid - 1) / grid) + (size_t)kWideWaves * kRowsMinQcap * sizeof(uint2) >
           cap)
        grid *= 2;
    size_t lds = sq8_wide_rows_lds(p.n_shards, (nq4 + grid - 1) / grid);
    // the queues: what LDS leaves, ≤ 1024 entries per owner wave (multiples of 64); tests ask for fewer
    Sq8Params q = p;
    const int room = (int)std::min<size_t>(1024, (cap - lds) / (kWideWaves * sizeof(uint2)) / 64 * 64);
    q.wide_qcap = p.wide_qcap > 0 ? std::min(p.wide_qcap, room) : room;
    lds += (size_t)kWideWaves * q.wide_qcap * sizeof(uint2);
    if (lds > cap) return hipErrorInvalidValue;   // (never: the grid doubling above)
    if (ev_start || ev_stop)
        hipExtLaunchKernelGGL(fn, dim3(grid), dim3(kWideThreads), lds, s, ev_start, ev_stop, 0, q);
    else
        hipLaunchKernelGGL(fn, dim3(grid), dim3(kWideThreads), lds, s, q);
    return hipGetLastError();
}

hipError_t launch_sq8_wide(const Sq8Params& p, hipStream_t s, hipEvent_t ev_start, hipEvent_t ev_stop) {
    if (!sq8_wide_supported(p.units8) || p.q_count < 1 || p.q_count > kWideQ || p.accept || p.gtiles ||
        p.sim < 0 || p.sim > 3 || !p.rows8t || !p.auxt || p.n_lists != 4 * p.n_tiles || p.k < 1 || p.k > kKQ ||
        p.n_shards < 1 || p.wide_grid < 1 || (p.pilot && !p.pilot_keys) || (!p.pilot && !p.quarter_bm))
        return hipErrorInvalidValue;
    const int ks = sq8_wide_ks(p.units8);
    const auto fn = kWide[ks == 2 ? 0 : ks == 4 ? 1 : ks == 8 ? 2 : 3][p.sim];
    const int nq4 = (p.quarter_end > 0 ? p.quarter_end : 4 * p.n_tiles) - p.quarter_begin;
    if (p.quarter_begin < 0 || nq4 < 1 || p.quarter_begin + nq4 > 4 * p.n_tiles || (p.quarter_begin && p.pilot))
        return hipErrorInvalidValue;
    int grid = std::min(p.wide_grid, std::max(1, nq4));
    // more workgroups (rounds of the chip) when one CU's share of quarter descriptors does not fit
    const size_t lcap = 160 * 1024 - kernel_static_lds(reinterpret_cast<const void*>(fn));
    while (sq8_wide_lds(ks, p.sim, p.n_shards, (nq4 + grid - 1) / grid) > lcap) grid *= 2;
    size_t lds = sq8_wide_lds(ks, p.sim, p.n_shards, (nq4 + grid - 1) / grid);
    // the deferred-insertion queues in what LDS is left: ≥ 256 entries per wave (one (group, query block) adds at
    // most 64 lanes × 4 rows), else the immediate insertions (and always for the pilot)
    Sq8Params q = p;
    const int room = (int)((lcap - lds) / (kWideWaves * sizeof(uint2))) / 64 * 64;
    q.wide_qcap = (!p.pilot && p.wide_defer && room >= 256) ? std::min(room, 512) : 0;
    lds += (size_t)kWideWaves * q.wide_qcap * sizeof(uint2);
    if (ev_start || ev_stop)
        hipExtLaunchKernelGGL(fn, dim3(grid), dim3(kWideThreads), lds, s, ev_start, ev_stop, 0, q);
    else
        hipLaunchKernelGGL(fn, dim3(grid), dim3(kWideThreads), lds, s, q);
    return hipGetLastError();
}

#ifdef OSK_TESTING
// glds16_run's destination contract, kept as a GPU test (tests/test_gpu_wide.py::test_glds16_run_destinations;
// round 5 built the one-statement DMAs on the wrong reading of the immediate offset and faulted a box): for
// N = 1, 2, 4 DMAs at both strides the kernel uses (1 KiB slabs, kAuxGroupF4 bound-term groups), each DMA k
// reads gbase + lane·16 + k·GS and must land at ldsk[k] + lane·16 — the destinations here are out of order and
// not GS apart — with every other LDS byte untouched.  One 64-lane workgroup; out: 6 images of the 16 KiB LDS.
// (Every destination is ≥ k·GS above the LDS base: glds16_run's precondition.  The first version of this probe
// put them in reverse order from offset 512, so M0 = ldsk[k] − k·GS went below 0 for three of its DMAs, and
// exactly those three (192 words) did not land: M0 does not wrap.)
template <int N, int GS>
__device__ void glds_probe_case(const int4* src, int4* lds, int4* out) {
    for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = make_int4(-1, -1, -1, -1);
    __syncthreads();
    const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(__attribute__((address_space(3))) char*)lds);
    uint32_t ldsk[N];
#pragma unroll
    for (int k = 0; k < N; ++k) ldsk[k] = base + (uint32_t)(3072 + (N - 1 - k) * 2048 + 512);
    glds16_run<N, GS>(src, (uint32_t)threadIdx.x * 16u, ldsk);
    vm_wait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    for (int i = threadIdx.x; i < 1024; i += 64) out[i] = lds[i];
    __syncthreads();
}
__global__ __launch_bounds__(64) void glds_probe(const int4* src, int4* out) {
    __shared__ __attribute__((aligned(16))) int4 lds[1024];
    glds_probe_case<1, 1024>(src, lds, out);
    glds_probe_case<2, 1024>(src, lds, out + 1024);
    glds_probe_case<4, 1024>(src, lds, out + 2048);
    glds_probe_case<1, kAuxGroupF4 * 16>(src, lds, out + 3072);
    glds_probe_case<2, kAuxGroupF4 * 16>(src, lds, out + 4096);
    glds_probe_case<4, kAuxGroupF4 * 16>(src, lds, out + 5120);
}
hipError_t launch_glds_probe(const int4* src, int4* out, hipStream_t s) {
    hipLaunchKernelGGL(glds_probe, dim3(1), dim3(64), 0, s, src, out);
    return hipGetLastError();
}
#endif

}  // namespace osk
