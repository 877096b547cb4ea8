// osk_sq8w.hip — the certified int8 prefilter on MFMA for large batches: one corpus pass per 256 queries.
//
// sq8_mfma (osk_sq8.hip) takes 32 queries per launch, so a batch of B queries streams the int8 corpus
// B / 32 times: at 100M × 96 and B = 1024 that is 32 passes over 14 GB, 91 ms per batch.  A
// batched search is compute-light per byte — 96 int8 MACs per (row, query) — so the corpus is read once per
// 256 queries here (C4 b1024: 38.7 ms):
//
//   * persistent: one workgroup of 8 waves per CU takes every G-th (tile, quarter) of the tile order (tiles
//     interleaved over shards) as one continuous stream of 128-row steps through a 4-deep LDS-DMA ring
//     (global_load_lds_dwordx4); a quarter is exactly the row range of one scan-wave list of the settle
//     (list = tile·4 + quarter), so the settle and the per-shard merge are sq8_mfma's;
//   * a step is 8 groups of 16 rows: waves 0–3 load the groups' int8 slabs (chunk-major tiled copy: the
//     lane-linear image is the MFMA A operand), waves 4–7 their bound terms (launch_sq8_aux_tile: struct of
//     arrays, a lane's 4 rows in one ds_read_b128); one barrier per step;
//   * each wave owns 32 of the launch's 256 queries: B fragments in VGPRs for the whole launch, 2 query
//     blocks × KS v_mfma_i32_16x16x64_i8 per group, exact int32 dots;
//   * the quick test per (row, query) is one fma and a compare (packed pairs): the bound's error terms are
//     relaxed to the quarter's row maxima (launch_wide_quarter_max), so what stays per pair is I·s_x against a
//     per-(quarter, query) threshold (EUCLIDEAN: a per-row affine function of |x|²) — provably no stricter
//     than sq8_bounds' upper side (derivation at quick_consts).  A passing pair takes the precise bound in
//     its own lane and, above the floor, is appended to its (quarter, query) list by an LDS atomic; lists
//     that would fill go through sq8_mfma's ordered insertion (sorted once, best kKQ kept);
//   * floors: pilot = 1 bounds each quarter's first step of rows (the best lower-bound key per query; their k-th
//     per (query, shard) floors the main pass); the main pass runs in two launches — 1/phase of the quarters
//     first, then the rest under floors raised to the k-th best list maximum of the first (launch_wide_floor;
//     the sq8_mfma pilot argument: k distinct rows score ≥ T, a row with ub < T cannot enter or tie into the
//     top k).  C4 b256: 3.7M → 0.97M insertions per search.
// Results are bit-identical to sq8_mfma's, the fp32 streaming scan's and the oracle's (tests/test_gpu_wide.py).
#include <hip/hip_ext.h>

#include "osk_device.h"
#include "osk_internal.h"
#include "osk_wave.h"

namespace osk {

int sq8_wide_supported(int u8) { return u8 >= 1 && u8 <= 16 ? 1 : 0; }   // KS = 2 (≤ 128 dims) or 4 (≤ 256)

// The wide kernel's bound terms per 16-row group (osk_internal.h, launch_sq8_aux_tile): one thread per float4.
__global__ __launch_bounds__(kBlock) void sq8_aux_tile(const float4* __restrict__ aux, const float* __restrict__ xnorm,
                                                       int64_t n_rows, float4* __restrict__ out) {
    const int64_t ng = (n_rows + 15) / 16, total = ng * kAuxGroupF4;
    for (int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x; t < total; t += (int64_t)gridDim.x * kBlock) {
        const int64_t g = t / kAuxGroupF4, r0 = g * 16;
        const int slot = (int)(t - g * kAuxGroupF4);
        float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
        if (slot < 16 || slot >= 18) {   // component slot / 4 of rows 4·(slot % 4) … + 3 (slots 18–21: xnorm)
            const int c = slot >> 2, rb = (slot & 3) * 4;   // (slot 18 → rows 8…: re-based below)
            const int rbase = slot >= 18 ? (slot - 18) * 4 : rb;
            float v[4];
            for (int i = 0; i < 4; ++i) {
                const int64_t r = r0 + rbase + i;
                if (slot >= 18) {
                    v[i] = (xnorm && r < n_rows) ? xnorm[r] : 0.0f;
                } else {
                    const float4 a = r < n_rows ? aux[r] : make_float4(0.f, 0.f, 0.f, 0.f);
                    v[i] = c == 0 ? a.x : c == 1 ? a.y : c == 2 ? a.z : a.w;
                }
            }
            o = make_float4(v[0], v[1], v[2], v[3]);
        } else {
            float y = 0.0f, z = 0.0f, w = 0.0f, wmin = __builtin_inff(), amax = 0.0f, amin = __builtin_inff();
            for (int i = 0; i < 16 && r0 + i < n_rows; ++i) {
                const float4 a = aux[r0 + i];
                y = fmaxf(y, a.y);
                z = fmaxf(z, a.z);
                w = fmaxf(w, a.w);
                wmin = fminf(wmin, a.w);
                amax = fmaxf(amax, a.x);
                amin = fminf(amin, a.x);
            }
            o = slot == 16 ? make_float4(y, z, w, wmin) : make_float4(amax, amin, 0.0f, 0.0f);
        }
        out[t] = o;
    }
}

hipError_t launch_sq8_aux_tile(const float4* aux, const float* xnorm, int64_t n_rows, float4* out, hipStream_t s) {
    if (n_rows <= 0) return hipMemsetAsync(out, 0, (size_t)kAuxGroupF4 * sizeof(float4), s);
    const int64_t total = (n_rows + 15) / 16 * kAuxGroupF4;
    const int64_t blocks = std::min<int64_t>(8192, (total + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(sq8_aux_tile, dim3((unsigned)blocks), dim3(kBlock), 0, s, aux, xnorm, n_rows, out);
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
    const int4* xt;       // the tiled int8 rows from the quarter's first 16-row group
    const float4* at;     // the tiled bound terms from its first group (kAuxGroupF4 float4 per group)
    uint32_t vrow0;       // view row of its first row
    int32_t nrows;        // (the pilot: its first step's rows at most)
    int32_t list;         // tile·4 + quarter: the settle's list, the pilot's slot
    int32_t shard;
    int32_t seg;
    int32_t pad[3];
    float4 bm;            // the quarter's row maxima {max s|q|, max |δ|, max |x|², min |x|²} (launch_wide_quarter_max)
};
constexpr int kWideMaxFloorShards = 16;   // per-(shard, query) floors held in LDS up to this many shards
constexpr int kWideThreads = kWideWaves * 64;
constexpr int kWideSorted = 1 << 20;      // s_cnt of a list the ordered insertion has sorted

// Persistent: gridDim.x workgroups (one per CU), workgroup w takes quarters w, w + G, w + 2G, … of the
// tile order (tiles interleaved over shards), as ONE continuous stream of 64-row steps through an NS-deep
// LDS-DMA ring, so the ring never drains at a quarter boundary and the queries' B fragments, constants and
// floors are set up once per launch.  8 waves, two per SIMD (one's MFMAs overlap the other's quick tests
// and LDS latency): waves 0–3 load group w's KS int8 slabs of a step, waves 4–7 group w − 4's bound terms;
// every wave scores its 32 queries against all 4 groups.  Each wave flushes its queries' lists when its
// quarter ends.
template <int KS, int HT, int SIM, int NS>
__global__ __launch_bounds__(kWideThreads, 1) void sq8_wide(Sq8Params p) {
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    constexpr int QB = kWideQB;
    constexpr int AUXF4 = SIM == SIM_COSINE ? kAuxGroupF4 : 18;   // staged float4 of a group's bound terms
    constexpr int AUXB = AUXF4 * 16;          // a[16] y[16] z[16] w[16] {maxima} {a range} (COSINE: xnorm[16])
    constexpr int GB = KS * 1024 + AUXB;      // one 16-row group in a slot
    constexpr int GPS = KS == 2 ? 8 : 4;      // 16-row groups per step (one barrier per step)
    constexpr int PP = 0;                     // 1: waves 4–7 run a step's quick tests one step late (ping-pong;
                                              // measured no faster), the ring then holds one more step
    constexpr int SLOT = GPS * GB;            // one step
    constexpr int sim = SIM;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int col = lane & 15, grp = lane >> 4;
    const int gm = wave & 3;            // the groups of a step this wave loads: gm, gm + 4, …
    const bool dma_rows = wave < 4;     // its int8 slabs (waves 0–3) or its bound terms (waves 4–7)
    const int u8 = p.units8, S = p.n_shards;
    const bool pilot = p.pilot != 0;
#ifdef OSK_TESTING
    // A/B timing only (results wrong): 1 skip the quick tests and lists, 2 skip the MFMAs, 8 no barrier between steps, 16 no list / pilot-key stores, 32 quick tests without
    // their insertions, 64 the ring alone (no step processing)
    const int ablate = p.ablate;
#else
    constexpr int ablate = 0;
#endif
    const int G = gridDim.x, n_quarters = 4 * p.n_tiles;
    const int qbeg = p.quarter_begin, n_range = (p.quarter_end > 0 ? p.quarter_end : n_quarters) - qbeg;
    const int n_mine = (int)blockIdx.x < n_range ? (n_range - 1 - (int)blockIdx.x) / G + 1 : 0;
    const bool floor_lds = S <= kWideMaxFloorShards;

    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint64_t* s_lk = reinterpret_cast<uint64_t*>(smem + NS * SLOT);      // [kWideQ][kKQ] upper-bound keys
    uint32_t* s_lp = reinterpret_cast<uint32_t*>(s_lk + kWideQ * kKQ);   // their lower bounds
    float4* s_qc = reinterpret_cast<float4*>(s_lp + kWideQ * kKQ);        // [kWideQ] query bound terms
    uint32_t* s_floor = reinterpret_cast<uint32_t*>(s_qc + kWideQ);       // [S][kWideQ] the pilot's floor scores
    int32_t* s_cnt = reinterpret_cast<int32_t*>(s_floor + (floor_lds ? S * kWideQ : 0));   // [kWideQ] list fill
    WideQuarter* s_quart = reinterpret_cast<WideQuarter*>(s_cnt + kWideQ);
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
    if (floor_lds)
        for (int i = tid; i < S * kWideQ; i += kWideThreads) s_floor[i] = floor_of(i % kWideQ, i / kWideQ);
    for (int i = tid; i < n_mine; i += kWideThreads) {
        const int j = qbeg + (int)blockIdx.x + i * G;
        const int tix = p.tile_order ? p.tile_order[j >> 2] : j >> 2, quarter = j & 3;
        const TileDev tile = p.tiles[tix];
        const int64_t trows = tile.row_end - tile.row_begin;
        const int64_t spw = ((trows + 4 * kMfmaScanR - 1) / (4 * kMfmaScanR)) * kMfmaScanR;
        const int64_t rb = min(tile.row_begin + quarter * spw, tile.row_end);
        const int64_t re = min(rb + spw, tile.row_end);
        WideQuarter d;
        d.xt = p.rows8t[tile.seg] + (rb >> 4) * (KS * 64);
        d.at = p.auxt[tile.seg] + (rb >> 4) * kAuxGroupF4;
        d.vrow0 = (uint32_t)(p.seg_vrow[tile.seg] + rb);
        d.nrows = (int32_t)(pilot ? min<int64_t>(16 * GPS, re - rb) : re - rb);   // the pilot: one step
        d.list = tix * 4 + quarter;
        d.shard = tile.shard;
        d.seg = tile.seg;
        d.bm = p.quarter_bm ? p.quarter_bm[d.list] : make_float4(0.f, 0.f, 0.f, 0.f);
        s_quart[i] = d;
    }

    // this lane's queries: wq0 + qb·16 + col
    const int wq0 = wave * 16 * QB;
    // the dims' K-steps: nf full 64-dim slabs, then (ht) a 32-dim tail, the first two chunks of slab nf (a
    // slab with ≤ 2 of its 4 chunks in use; v_mfma_i32_16x16x32_i8: half the MFMA cycles, LDS reads and
    // HBM bytes of that slab)
    constexpr bool ht = HT != 0;
    constexpr int nf = KS - HT;   // (dims short of the last slab compute zeros there: exact)
    i32x4 bfr[KS][QB];
    long bfh[QB];   // the tail's B fragment: 8 B (chunk (grp >> 1) of slab nf, half grp & 1)
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
        {
            const int f = nf * 4 + (grp >> 1);
            const int4 v = (ht && qv && f < u8) ? p.q8[(int64_t)qi * u8 + f] : make_int4(0, 0, 0, 0);
            bfh[qb] = (grp & 1) ? (long)(((uint64_t)(uint32_t)v.w << 32) | (uint32_t)v.z)
                                : (long)(((uint64_t)(uint32_t)v.y << 32) | (uint32_t)v.x);
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
        asm volatile("" ::"v"(bfh[qb]));
        asm volatile("" ::"v"(qnd[qb]), "v"(inv[qb]));
    }

    // the workgroup's steps: its quarters' 64-row steps back to back (empty quarters take none)
    auto steps_of = [&](int q) { return (s_quart[q].nrows + 16 * GPS - 1) / (16 * GPS); };
    int total = 0;
    for (int q = 0; q < n_mine; ++q) total += steps_of(q);
    const uint32_t ring_lds =
        __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(__attribute__((address_space(3))) char*)smem);
    // a lane's tail fragment in its slab image (chunk-major: row lane & 15, 8 B at dims 8·(lane >> 4))
    const uint32_t tail_off = (uint32_t)((lane >> 5) * 256 + (lane & 15) * 16 + ((lane >> 4) & 1) * 8);
    // a group's dots: acc[qb] = the int8 dots of its 16 rows (4·grp + r) with query block qb (column col)
    auto group_dots = [&](const char* gb, i32x4 (&ac)[QB]) {
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) ac[qb] = i32x4{0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            if (s < nf) {
                const i32x4 a = *reinterpret_cast<const i32x4*>(gb + s * 1024 + lane * 16);
#pragma unroll
                for (int qb = 0; qb < QB; ++qb)
                    ac[qb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bfr[s][qb], ac[qb], 0, 0, 0);
            }
        }
        if (ht) {   // (own accumulators, added after: no K=64 → K=32 MFMA accumulator chain)
            const long ah = *reinterpret_cast<const long*>(gb + nf * 1024 + tail_off);
#pragma unroll
            for (int qb = 0; qb < QB; ++qb)
                ac[qb] += __builtin_amdgcn_mfma_i32_16x16x32_i8(ah, bfh[qb], i32x4{0, 0, 0, 0}, 0, 0, 0);
        }
    };
    int iq = 0, ist = 0;   // the next step to issue: quarter iq of mine, its step ist
    while (iq < n_mine && steps_of(iq) == 0) ++iq;
    // this wave's part of the step → slot; groups past the quarter load its first group (valid, skipped)
    auto issue = [&](int slot) {
        const WideQuarter& d = s_quart[iq];
#pragma unroll
        for (int h = 0; h < GPS / 4; ++h) {
            const int gi = GPS * ist + gm + 4 * h;
            const int gv = 16 * gi < d.nrows ? gi : 0;
            const uint32_t dst = ring_lds + (uint32_t)(slot * SLOT + (gm + 4 * h) * GB);
            if (dma_rows) {
                const int4* src = d.xt + gv * (KS * 64);
#pragma unroll
                for (int s = 0; s < KS; ++s)
                    if (s < nf) glds16(src + s * 64 + lane, dst + s * 1024);   // (the slab image is lane-linear)
                if (ht && lane < 32) glds16(src + nf * 64 + lane, dst + nf * 1024);
            } else if (lane < AUXF4) {
                glds16(d.at + gv * kAuxGroupF4 + lane, dst + KS * 1024);
            }
        }
        if (++ist == steps_of(iq)) {
            ist = 0;
            do ++iq; while (iq < n_mine && steps_of(iq) == 0);
        }
    };

    // the full bound terms {a, y, z, w} of the lane's 4 rows (4·grp + r) of a group (pilot and insertions)
    auto row_terms = [&](const char* ga, float4 (&ax)[4]) {
        const float4 A = *reinterpret_cast<const float4*>(ga + grp * 16);
        const float4 Y = *reinterpret_cast<const float4*>(ga + 64 + grp * 16);
        const float4 Z = *reinterpret_cast<const float4*>(ga + 128 + grp * 16);
        const float4 W = *reinterpret_cast<const float4*>(ga + 192 + grp * 16);
        ax[0] = make_float4(A.x, Y.x, Z.x, W.x);
        ax[1] = make_float4(A.y, Y.y, Z.y, W.y);
        ax[2] = make_float4(A.z, Y.z, Z.z, W.z);
        ax[3] = make_float4(A.w, Y.w, Z.w, W.w);
    };
    // the quick test of the lane's 4 rows against one query: t_r = fma(I, a_r, −ca) (EUCLIDEAN
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
    uint32_t n_events = 0, n_pairs = 0;   // insertion events (wave-uniform) and quick-test passes (per lane)
    uint64_t cyc_wait = 0, cyc_loop = 0;   // wave 0's clocks: the step loop's waits, the whole loop
#endif
    float ca[QB], cb[QB];   // the held step's quick-test constants
    // a quarter ends: its lists (this wave's queries, 4 per pass of 16 lanes) → the settle's arrays, zeroed
    auto flush = [&](const WideQuarter& d) {
        const int q_end = min(wq0 + 16 * QB, p.q_count);
        for (int q0 = wq0; q0 < q_end; q0 += 4) {
            const int qg = q0 + (lane >> 4), e = lane & 15;
            const uint64_t lkb = s_lk[qg * kKQ + e];
            const uint32_t lpb = s_lp[qg * kKQ + e];
            uint32_t m = lkb ? lpb : 0u;
#pragma unroll
            for (int o = 8; o >= 1; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
            if (qg < q_end && !(ablate & 16)) {
                const size_t l = (size_t)(p.q0 + qg) * p.n_lists + d.list;
                p.cand[l * kKQ + e] = lkb;
                p.cand_lb[l * kKQ + e] = lpb;
                if (e == 0) p.list_lbmax[l] = m;
                s_lk[qg * kKQ + e] = 0ull;
                s_lp[qg * kKQ + e] = 0u;
                if (e == 0) s_cnt[qg] = 0;
            }
        }
        if (p.visited && p.q0 == 0 && tid == 0 && d.nrows > 0)
            atomicAdd(&p.visited[d.seg], (unsigned long long)d.nrows);
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
        // Two waves per SIMD in ping-pong: waves 0–3 read and multiply step i, then run its quick tests;
        // waves 4–7 first run step i − 1's quick tests (held in registers), then read and multiply step i.
        // So one wave's MFMAs and LDS reads overlap the other's quick tests and insertions, and the ring keeps
        // one more slot (step i − 1) readable: the DMA at step i targets step i − 2's slot.
        const bool late = PP && wave >= 4;
        for (int st = 0; st < NS - 1 - PP && st < total; ++st) issue(st);
        int s_issue = (NS - 1 - PP) % NS, s_read = 0;
        int pq = -1, pst = 0;   // the quarter of mine and its step that the next read starts from / reaches
        // the held step (read and multiplied, quick tests pending)
        bool held = false;
        const char* hslot = smem;
        int hst = 0, hgroups = 0, hq = 0;
        i32x4 acc[GPS][QB];
        float4 bm = make_float4(0.f, 0.f, 0.f, 0.f);
        // the held step's quick tests and insertions
        auto quick_phase = [&]() __attribute__((always_inline)) {
            const WideQuarter& hd = s_quart[hq];
            float4 A4[GPS], W4[GPS];   // the groups' a_r, w_r of the lane's rows (re-read from the slot)
#pragma unroll
            for (int g = 0; g < GPS; ++g) {
                A4[g] = *reinterpret_cast<const float4*>(hslot + g * GB + KS * 1024 + grp * 16);
                W4[g] = (SIM == SIM_EUCLIDEAN || SIM == SIM_COSINE)
                            ? *reinterpret_cast<const float4*>(hslot + g * GB + KS * 1024 + 192 + grp * 16)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
            }
            // the rows' quick-test factors: a_r (COSINE a_r/√w_r; a zero row's pairs pass), w_r (EUCLIDEAN)
            float ar[GPS][4], wr[GPS][4];
            bool zr[GPS];
#pragma unroll
            for (int g = 0; g < GPS; ++g) {
                ar[g][0] = A4[g].x; ar[g][1] = A4[g].y; ar[g][2] = A4[g].z; ar[g][3] = A4[g].w;
                wr[g][0] = W4[g].x; wr[g][1] = W4[g].y; wr[g][2] = W4[g].z; wr[g][3] = W4[g].w;
                zr[g] = false;
                if constexpr (SIM == SIM_COSINE) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        zr[g] |= !(wr[g][r] > 0.0f);
                        ar[g][r] = ar[g][r] * __builtin_amdgcn_rsqf(wr[g][r]);   // (0 · ∞ = NaN: passes)
                    }
                }
            }
            uint32_t qmg[GPS];   // per group: the wave's queries with a passing pair (wave-uniform)
#pragma unroll
            for (int g = 0; g < GPS; ++g) {
                uint32_t qm = 0u;
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) {
                    f32x2 t01, t23;
                    quick_t(acc[g][qb], ar[g], wr[g], ca[qb], cb[qb], t01, t23);
                    const float mx = fmaxf(fmaxf(t01.x, t01.y), fmaxf(t23.x, t23.y));   // (NaN terms dropped)
                    const bool any = !(mx < 0.0f) || zr[g];
                    const uint64_t bl = __ballot(any) & qvm[qb];
                    qm |= (uint32_t)((bl | (bl >> 16) | (bl >> 32) | (bl >> 48)) & 0xFFFFull) << (16 * qb);
                }
                qmg[g] = g < hgroups ? qm : 0u;
            }
            uint32_t qany = 0u;
#pragma unroll
            for (int g = 0; g < GPS; ++g) qany |= qmg[g];
            if (!qany || (ablate & 32)) return;
#pragma unroll 1
            for (int g = 0; g < hgroups; ++g) {
                uint32_t qmgg = 0u;   // (g is wave-uniform: selects, no indexed register access)
#pragma unroll
                for (int gg = 0; gg < GPS; ++gg) qmgg = gg == g ? qmg[gg] : qmgg;
                if (!qmgg) continue;
#ifdef OSK_TESTING
                n_events += __popc(qmgg);
#endif
                // group g's dots and row factors again, from its slot (no register array indexed by the
                // runtime g: that would put the step's accumulators in scratch memory)
                const char* gb = hslot + g * GB;
                const char* ga = gb + KS * 1024;
                i32x4 ac[QB];
                group_dots(gb, ac);
                const float4 Ag = *reinterpret_cast<const float4*>(ga + grp * 16);
                const float4 Wg = *reinterpret_cast<const float4*>(ga + 192 + grp * 16);
                float arg[4] = {Ag.x, Ag.y, Ag.z, Ag.w};
                const float wrg[4] = {Wg.x, Wg.y, Wg.z, Wg.w};
                if constexpr (SIM == SIM_COSINE) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) arg[r] = arg[r] * __builtin_amdgcn_rsqf(wrg[r]);
                }
                const int r0 = 16 * (GPS * hst + g);   // rows of the quarter
                const int nr = min(16, hd.nrows - r0);
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
                            sq8_bounds(sim, (float)ac[qb][r], ax[r], qcb, p.gam, p.g2, lo, hi);
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
                            tq[qb] = sq8_quick(sim, thrb > tkey[qb] ? thrb : tkey[qb], sqrtf(qnd[qb]), p.cos_slack);
                            quick_consts<SIM>(tq[qb], sb[qb], inv[qb], QY[qb], QZ[qb], Q0[qb], QW, zq[qb], ig2m, bm,
                                              ca[qb], cb[qb]);
                        }
                    }
                }
            }
        };
#ifdef OSK_TESTING
        const uint64_t c_loop0 = clock64();
#endif
        // (one iteration past the last step: the late waves' quick tests of it; one call site of each phase)
        for (int i = 0; i <= total; ++i) {
            if (i < total) {
#ifdef OSK_TESTING
                const uint64_t c0 = clock64();
#endif
                // this wave's DMAs of step i have landed (steps i+1 … i+NS−3 may still be in flight); every
                // wave's have once all pass the barrier, which also retires every wave's reads of step i − 2's slot
                if (i + NS - 1 - PP <= total) {   // (this wave's LDS-DMA instructions per step: GPS/4 · …)
                    if (dma_rows) vm_wait<(NS - 2 - PP) * (GPS / 4) * (nf + HT)>();
                    else vm_wait<(NS - 2 - PP) * (GPS / 4)>();
                } else {
                    vm_wait<0>();
                }
                if (!(ablate & 8)) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#ifdef OSK_TESTING
                cyc_wait += clock64() - c0;
#endif
                if (i + NS - 1 - PP < total) {
                    issue(s_issue);
                    s_issue = s_issue + 1 == NS ? 0 : s_issue + 1;
                }
            }
            if (ablate & 64) continue;   // (A/B: the ring alone)
#pragma unroll 1
            for (int ph = 0; ph < 2; ++ph) {
            if (held && (late ? ph == 0 : ph == 1)) {
                quick_phase();
                held = false;
            }
            if (ph == 1 || i == total) continue;
            if (pq < 0 || ++pst == steps_of(pq)) {   // a new quarter: flush the last one, take its floors
                if (pq >= 0 && !pilot) flush(s_quart[pq]);
                do ++pq; while (steps_of(pq) == 0);
                pst = 0;
                const int sh = s_quart[pq].shard;
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) {
                    const int qi = wq0 + qb * 16 + col;
                    const uint32_t f = floor_lds ? s_floor[sh * kWideQ + qi] : floor_of(qi, sh);
                    tkey[qb] = (uint64_t)f << 32;
                    tq[qb] = sq8_quick(sim, tkey[qb], sqrtf(qnd[qb]), p.cos_slack);
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
            hgroups = min(GPS, ((s_quart[pq].nrows + 15) >> 4) - GPS * pst);   // (< GPS: the quarter's last step)
            if (pilot) {
                const WideQuarter& hd = s_quart[hq];
            {   // the quarter's first 64 rows: per query the best lower-bound key → pilot_keys
                uint64_t pbest[QB];
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) pbest[qb] = 0ull;
#pragma unroll 1
                for (int g = 0; g < hgroups; ++g) {
                    const char* gb = hslot + g * GB;
                    const char* ga = gb + KS * 1024;
                    const int r0 = 16 * g, nr = min(16, hd.nrows - r0);
                    i32x4 acc[QB];
                    group_dots(gb, acc);
                    float4 ax[4];
                    row_terms(ga, ax);
#pragma unroll
                    for (int qb = 0; qb < QB; ++qb) {
                        const int qi = wq0 + qb * 16 + col;
                        const float4 qc = s_qc[qi];
                        uint64_t best = 0ull;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int rr = 4 * grp + r;
                            float xnd = 0.0f;
                            if constexpr (SIM == SIM_COSINE) xnd = *reinterpret_cast<const float*>(ga + 288 + rr * 4);
                            float lo, hi;
                            sq8_bounds(sim, (float)acc[qb][r], ax[r], qc, p.gam, p.g2, lo, hi);
                            const float lb = SIM == SIM_EUCLIDEAN ? score_f32_l2(hi) : score_f32(sim, lo, qnd[qb], xnd);
                            const uint64_t key = rr < nr ? make_key(lb, hd.vrow0 + (uint32_t)(r0 + rr)) : 0ull;
                            best = key > best ? key : best;
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
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) {
                    const int qi = wq0 + qb * 16 + col;
                    if (grp == 0 && qi < p.q_count && !(ablate & 16))
                        p.pilot_keys[(size_t)qi * n_quarters + hd.list] = pbest[qb];
                    // the two-pass main pass reads the second pass's list maxima as empty until it writes them
                    if (grp == 0 && qi < p.q_count) p.list_lbmax[(size_t)(p.q0 + qi) * p.n_lists + hd.list] = 0u;
                }
            }
                continue;
            }
            {   // read and multiply step i
                const char* slot = hslot;
            // Every LDS read of the step first (the 4 groups' A fragments and maxima), then the step's 4·KS·QB
            // MFMAs as straight-line code: one exposed LDS latency per step.  Groups past the quarter's end (its
            // last step) hold valid rows of its first group; their passes are masked.
            i32x4 a[GPS][KS];
            long ah[GPS];
#pragma unroll
            for (int g = 0; g < GPS; ++g) {
                const char* gb = slot + g * GB;
#pragma unroll
                for (int s = 0; s < KS; ++s)
                    a[g][s] = s < nf ? *reinterpret_cast<const i32x4*>(gb + s * 1024 + lane * 16) : i32x4{0, 0, 0, 0};
                ah[g] = ht ? *reinterpret_cast<const long*>(gb + nf * 1024 + tail_off) : 0l;
            }
#pragma unroll
            for (int g = 0; g < GPS; ++g)
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) acc[g][qb] = i32x4{0, 0, 0, 0};
            if (ablate & 2) {
#pragma unroll
                for (int g = 0; g < GPS; ++g)
#pragma unroll
                    for (int s = 0; s < KS; ++s) acc[g][0] ^= a[g][s];
            } else {
#pragma unroll
                for (int g = 0; g < GPS; ++g) {
#pragma unroll
                    for (int s = 0; s < KS; ++s)
                        if (s < nf)
#pragma unroll
                            for (int qb = 0; qb < QB; ++qb)
                                acc[g][qb] =
                                    __builtin_amdgcn_mfma_i32_16x16x64_i8(a[g][s], bfr[s][qb], acc[g][qb], 0, 0, 0);
                    if (ht)   // (own accumulators, added after: no K=64 → K=32 MFMA accumulator chain)
#pragma unroll
                        for (int qb = 0; qb < QB; ++qb)
                            acc[g][qb] += __builtin_amdgcn_mfma_i32_16x16x32_i8(ah[g], bfh[qb], i32x4{0, 0, 0, 0}, 0, 0, 0);
                }
            }
            if (ablate & 1) {
                if (acc[0][0][0] + acc[3][QB - 1][3] == 0x7FFFFFFF && bm.x == 1.0f) s_lp[tid] = 1u;
                held = false;
            }
            }
            held = !(ablate & 1);
            }
        }
        vm_wait<0>();
#ifdef OSK_TESTING
        cyc_loop += clock64() - c_loop0;
#endif
        if (pq >= 0 && !pilot) flush(s_quart[pq]);
    }
#ifdef OSK_TESTING
    if (!pilot && p.counters) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) n_pairs += __shfl_xor(n_pairs, o);
        if (lane == 0) {
            atomicAdd(&p.counters[4], (unsigned long long)n_events);
            atomicAdd(&p.counters[5], (unsigned long long)n_pairs);
            if (wave == 0) {
                atomicAdd(&p.counters[6], (unsigned long long)cyc_wait);
                atomicAdd(&p.counters[8], (unsigned long long)cyc_loop);
            }
        }
    }
#endif
}

using WideFn = void (*)(Sq8Params);
// ring depth per KS: the deepest ring that leaves room for the lists, the floors of ≤ 16 shards and the
// quarter descriptors in 160 KiB (one workgroup per CU): KS = 2 → 8 steps (75 KB), KS = 4 → 4 (70 KB)
#define OSK_WIDE_SIMS(KS, HT, NS) \
    {sq8_wide<KS, HT, 0, NS>, sq8_wide<KS, HT, 1, NS>, sq8_wide<KS, HT, 2, NS>, sq8_wide<KS, HT, 3, NS>}
// [KS = 4][HT]: HT = 1 when the last slab holds ≤ 2 chunks of dims (u8 ≤ 6 / ≤ 14; fewer dims: zero slabs)
static const WideFn kWide[2][2][4] = {{OSK_WIDE_SIMS(2, 0, 4), OSK_WIDE_SIMS(2, 1, 4)},
                                      {OSK_WIDE_SIMS(4, 0, 4), OSK_WIDE_SIMS(4, 1, 4)}};
static constexpr int kWideNS[2] = {4, 4};
static constexpr size_t kLdsCap = 160 * 1024;

static size_t sq8_wide_lds(int ks, int sim, int n_shards, int n_mine) {
    const size_t slot = (size_t)(ks == 2 ? 8 : 4) * (ks * 1024 + (sim == SIM_COSINE ? kAuxGroupF4 : 18) * 16);
    return (size_t)kWideNS[ks == 4] * slot + (size_t)kWideQ * kKQ * 12 + (size_t)kWideQ * 16 + (size_t)kWideQ * 4 +
           (n_shards <= kWideMaxFloorShards ? (size_t)n_shards * kWideQ * 4 : 0) + (size_t)n_mine * sizeof(WideQuarter);
}

hipError_t launch_sq8_wide(const Sq8Params& p, hipStream_t s, hipEvent_t ev_start, hipEvent_t ev_stop) {
    if (!sq8_wide_supported(p.units8) || p.q_count < 1 || p.q_count > kWideQ || p.accept || p.gtiles ||
        p.sim < 0 || p.sim > 3 || !p.rows8t || !p.auxt || p.n_lists != 4 * p.n_tiles || p.k < 1 || p.k > kKQ ||
        p.n_shards < 1 || p.wide_grid < 1 || (p.pilot && !p.pilot_keys) || (!p.pilot && !p.quarter_bm))
        return hipErrorInvalidValue;
    const int ks = p.units8 <= 8 ? 2 : 4;
    const int ht = 0;   // (the K = 32 tail variant measured slower: C4 b256 13.3 vs 12.7 ms; kept for study)
    const auto fn = kWide[ks == 4][ht][p.sim];
    const int nq4 = (p.quarter_end > 0 ? p.quarter_end : 4 * p.n_tiles) - p.quarter_begin;
    if (p.quarter_begin < 0 || nq4 < 1 || p.quarter_begin + nq4 > 4 * p.n_tiles || (p.quarter_begin && p.pilot))
        return hipErrorInvalidValue;
    int grid = std::min(p.wide_grid, std::max(1, nq4));
    // more workgroups (rounds of the chip) when one CU's share of quarter descriptors does not fit
    while (sq8_wide_lds(ks, p.sim, p.n_shards, (nq4 + grid - 1) / grid) > kLdsCap) grid *= 2;
    const size_t lds = sq8_wide_lds(ks, p.sim, p.n_shards, (nq4 + grid - 1) / grid);
    if (ev_start || ev_stop)
        hipExtLaunchKernelGGL(fn, dim3(grid), dim3(kWideThreads), lds, s, ev_start, ev_stop, 0, p);
    else
        hipLaunchKernelGGL(fn, dim3(grid), dim3(kWideThreads), lds, s, p);
    return hipGetLastError();
}

}  // namespace osk
