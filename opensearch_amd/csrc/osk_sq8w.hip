// osk_sq8w.hip — the certified int8 prefilter on MFMA for large batches: one corpus pass per 256 queries.
//
// sq8_mfma (osk_sq8.hip) takes 32 queries per launch, so a batch of B queries streams the int8 corpus
// B / 32 times: at 100M × 96 and B = 1024 that is 32 passes over 14 GB, 91 ms per batch at 0.49 of HBM
// (VERDICT r3).  A batched search is compute-light per byte — 96 int8 MACs per (row, query) — so the
// corpus should be read once per as many queries as the chip can score while it streams:
//
//   * one workgroup per (tile, quarter): the quarter is exactly the row range of one scan-wave list
//     of the settle (list = tile·4 + quarter, scan_R = kMfmaScanR), so the settle, its exact re-scan of an
//     overflowed list and the per-shard merge are sq8_mfma's, unchanged;
//   * its 4 waves share the quarter's rows: steps of 64 rows (one 16-row block per wave) stream from the
//     MFMA-tiled int8 copy into an LDS ring by LDS-DMA (global_load_lds_dwordx4, sources permuted so each
//     wave's A fragments are one conflict-free ds_read_b128 per 64-dim slab), with their 16-B bound terms
//     and the block's precomputed maxima; one barrier per step;
//   * each wave owns 64 of the launch's 256 queries: B fragments in VGPRs for the whole launch, 4 query
//     blocks × KS v_mfma_i32_16x16x64_i8 per 16-row block, exact int32 dots;
//   * the quick test per (row, query) is one fma and one compare: the bound's query-dependent error terms
//     are relaxed to the step's row maxima (sq8_block_max), so what stays per pair is I·s_x against a
//     per-(step, query) threshold (EUCLIDEAN: against a per-row affine function of |x|²) — provably no
//     stricter than sq8_bounds' upper side (derivation at quick_consts); the rare pairs that pass take the
//     precise bound and sq8_mfma's list insertion, into lists per (quarter, query) in LDS;
//   * pilot = 1: each workgroup bounds its quarter's first 64 rows and writes the best lower-bound key per
//     query; their k-th best per (query, shard) (merge_shards, one key per quarter) floors every list's
//     threshold in the main pass (the sq8_mfma pilot argument: k distinct rows score ≥ T, so a row with
//     ub < T cannot enter or tie into the top k).
// Results are bit-identical to sq8_mfma's, the fp32 streaming scan's and the oracle's.
#include <hip/hip_ext.h>

#include "osk_device.h"
#include "osk_internal.h"
#include "osk_wave.h"

namespace osk {

int sq8_wide_supported(int u8) { return u8 >= 1 && u8 <= 16 ? 1 : 0; }   // KS = 2 (≤ 128 dims) or 4 (≤ 256)

__global__ __launch_bounds__(kBlock) void sq8_block_max(const float4* __restrict__ aux, int64_t n_rows,
                                                        float4* __restrict__ out) {
    const int64_t nb = (n_rows + 15) / 16;
    for (int64_t b = (int64_t)blockIdx.x * kBlock + threadIdx.x; b < nb; b += (int64_t)gridDim.x * kBlock) {
        float y = 0.0f, z = 0.0f, w = 0.0f, wmin = __builtin_inff();
        for (int i = 0; i < 16; ++i) {
            const int64_t r = b * 16 + i;
            if (r >= n_rows) break;
            const float4 a = aux[r];
            y = fmaxf(y, a.y);
            z = fmaxf(z, a.z);
            w = fmaxf(w, a.w);
            wmin = fminf(wmin, a.w);
        }
        out[b] = make_float4(y, z, w, wmin);
    }
}

hipError_t launch_sq8_block_max(const float4* aux, int64_t n_rows, float4* out, hipStream_t s) {
    const int64_t nb = std::max<int64_t>(1, (n_rows + 15) / 16);
    const int64_t blocks = std::min<int64_t>(4096, (nb + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(sq8_block_max, dim3((unsigned)blocks), dim3(kBlock), 0, s, aux, n_rows, out);
    return hipGetLastError();
}

// The per-(step, query) constants of the quick test, from the step's row maxima bm = {max s·|q|, max |δ|,
// max |x|², min |x|²} (rows r of the step: a_r = s_x, w_r = |x|², y_r = s_x|q_x|, z_r = |δ_x|) and the
// query's terms (tq the list's quick threshold of sq8_quick, sb = s_b, QY/QZ/Q0 sq8_mfma's coefficients,
// zq = qc.z / s_b ≥ |q_b|).  In exact arithmetic sq8_mfma's quick test passes a pair when
//   DOT, MIP:   I·a_r·sb + E_r ≥ tq,            E_r = y_r·QY + z_r·QZ + w_r·QW + Q0
//   COSINE:     I·a_r·sb + E_r ≥ tq·√w_r
//   EUCLIDEAN:  2·I·a_r·sb ≥ w_r(1 − m) + Q0 − y_r·QY − z_r·QZ − tq / g2m
// and it is no stricter than sq8_bounds' upper side (sq8_mfma's derivation).  E_r and y_r·QY + z_r·QZ are
// at most their step maxima E, Em (every term ≥ 0), and √w_r ≥ √(min w), so each pass implies
//   DOT, MIP:   I·a_r ≥ (tq − E) / sb                               =: ca
//   COSINE:     I·(a_r / √w_r) ≥ (tq − E / √(min w)) / sb           =: ca
//   EUCLIDEAN:  I·a_r ≥ w_r·(1 − m)/(2sb) + (Q0 − Em − tq/g2m)/(2sb) =: w_r·ca + cb
// ca and cb are rounded DOWN by margins far above every float rounding here: 2^-18 of the magnitudes
// entering each numerator, then 2^-16 of |c| + B, B ≥ |I·a_r| (Cauchy–Schwarz on the integer vectors:
// |I|·a_r ≤ y_r·|q_b|; COSINE ÷ √w_r).  The pair test fma(I, a, −c) is one rounding of an exact value, so
// it keeps its sign: every pair sq8_mfma's quick test passes, this one passes.  A zero query (sb = 0), a
// list that is not full (tq = ∓∞) or a zero row (COSINE a/√w = NaN: !(NaN < 0) holds) passes every pair.
template <int SIM>
__device__ __forceinline__ void quick_consts(float tq, float sb, float QY, float QZ, float Q0, float QW, float zq,
                                             float g2m, float4 bm, float& ca, float& cb) {
    cb = 0.0f;
    if constexpr (SIM == SIM_EUCLIDEAN) {
        if (!(sb > 0.0f) || !(tq < __builtin_inff())) {
            ca = 0.0f;
            cb = -__builtin_inff();
            return;
        }
        const float Em = fmaf(bm.x, QY, bm.y * QZ);
        const float T = tq / g2m;
        const float num = (Q0 - Em - T) - 0x1p-18f * (Q0 + Em + fabsf(T));
        const float inv2 = 0.5f / sb;
        ca = (1.0f - 0x1p-17f) * inv2 * (1.0f - 0x1p-20f);
        cb = num * inv2;
        cb -= 0x1p-16f * (bm.z * ca + fabsf(cb) + bm.x * zq);
        return;
    } else {
        if (!(sb > 0.0f) || !(tq > -__builtin_inff())) {
            ca = -__builtin_inff();
            return;
        }
        float E = fmaf(bm.x, QY, fmaf(bm.y, QZ, fmaf(bm.z, QW, Q0)));
        float B = bm.x * zq;
        if constexpr (SIM == SIM_COSINE) {
            const float sxmin = sqrtf(bm.w);
            E = E / sxmin * (1.0f + 0x1p-20f);
            B = B / sxmin;
        }
        const float num = (tq - E) - 0x1p-18f * (fabsf(tq) + E);
        const float c = num / sb;
        ca = c - 0x1p-16f * (fabsf(c) + B);
    }
}

// One quarter of a workgroup's share (persistent kernel), described once in LDS so that no global load of
// tile or segment metadata sits between the ring's LDS-DMAs (a compiler-inserted vmcnt(0) would drain it).
struct WideQuarter {
    const int4* xt;       // the tiled int8 rows from the quarter's first 16-row block
    const float4* ax;     // bound terms from its first row
    const float4* bm;     // block maxima from its first block
    const float* xn;      // COSINE: device-order |x|² from its first row
    uint32_t vrow0;       // view row of its first row
    int32_t nrows;        // (the pilot: its first 64 rows at most)
    int32_t list;         // tile·4 + quarter: the settle's list, the pilot's slot
    int32_t shard;
    int32_t seg;
    int32_t pad[3];
};
constexpr int kWideMaxFloorShards = 16;   // per-(shard, query) floors held in LDS up to this many shards

// Persistent: gridDim.x workgroups (one per CU), workgroup w takes quarters w, w + G, w + 2G, … of the
// tile order (tiles interleaved over shards), as ONE continuous stream of 64-row steps through an NS-deep
// LDS-DMA ring, so the ring never drains at a quarter boundary and the queries' B fragments, constants and
// floors are set up once per launch.  Each wave flushes its queries' lists when its quarter ends.
template <int KS, int SIM, int NS>
__global__ __launch_bounds__(kBlock, 1) void sq8_wide(Sq8Params p) {
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    constexpr int QB = kWideQB;
    constexpr int GB = KS * 1024 + 17 * 16;   // one 16-row group in a slot: KS slabs, 16 rows' bound terms, block maxima
    constexpr int SLOT = 4 * GB;              // one step: 4 groups, the DMA of one wave each
    constexpr int OPS = KS + 1;               // LDS-DMA instructions per wave per step
    constexpr int sim = SIM;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int col = lane & 15, grp = lane >> 4;
    const int u8 = p.units8, S = p.n_shards;
    const bool pilot = p.pilot != 0;
#ifdef OSK_TESTING
    // A/B timing only (results wrong): 1 skip the quick tests and lists, 2 skip the MFMAs, 4 lane-linear DMA
    // sources (no operand permutation), 8 no barrier between steps
    const int ablate = p.ablate;
#else
    constexpr int ablate = 0;
#endif
    const int G = gridDim.x, n_quarters = 4 * p.n_tiles;
    const int n_mine = blockIdx.x < n_quarters ? (n_quarters - 1 - (int)blockIdx.x) / G + 1 : 0;
    const bool floor_lds = S <= kWideMaxFloorShards;

    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint64_t* s_lk = reinterpret_cast<uint64_t*>(smem + NS * SLOT);      // [kWideQ][kKQ] upper-bound keys
    uint32_t* s_lp = reinterpret_cast<uint32_t*>(s_lk + kWideQ * kKQ);   // their lower bounds
    float4* s_qc = reinterpret_cast<float4*>(s_lp + kWideQ * kKQ);        // [kWideQ] query bound terms
    uint32_t* s_floor = reinterpret_cast<uint32_t*>(s_qc + kWideQ);       // [S][kWideQ] the pilot's floor scores
    WideQuarter* s_quart = reinterpret_cast<WideQuarter*>(s_floor + (floor_lds ? S * kWideQ : 0));
    for (int i = tid; i < kWideQ * kKQ; i += kBlock) {
        s_lk[i] = 0ull;
        s_lp[i] = 0u;
    }
    for (int i = tid; i < kWideQ; i += kBlock) s_qc[i] = i < p.q_count ? p.qc[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    // the floor T of (query, shard): the k-th best sampled lower bound (its score's sortable bits; 0 = none)
    auto floor_of = [&](int qi, int sh) -> uint32_t {
        if (pilot || !p.thr_keys || qi >= p.q_count) return 0u;
        const size_t o = (size_t)qi * S + sh;
        if (p.thr_counts[o] < p.k) return 0u;
        const uint64_t t = p.thr_keys[o * p.k + p.k - 1];
        return key_score(t) > 0.0f ? (uint32_t)(t >> 32) : 0u;   // (a floor at the score-0 clamp would drop ties)
    };
    if (floor_lds)
        for (int i = tid; i < S * kWideQ; i += kBlock) s_floor[i] = floor_of(i % kWideQ, i / kWideQ);
    for (int i = tid; i < n_mine; i += kBlock) {
        const int j = (int)blockIdx.x + i * G;
        const int tix = p.tile_order ? p.tile_order[j >> 2] : j >> 2, quarter = j & 3;
        const TileDev tile = p.tiles[tix];
        const int64_t trows = tile.row_end - tile.row_begin;
        const int64_t spw = ((trows + 4 * kMfmaScanR - 1) / (4 * kMfmaScanR)) * kMfmaScanR;
        const int64_t rb = min(tile.row_begin + quarter * spw, tile.row_end);
        const int64_t re = min(rb + spw, tile.row_end);
        WideQuarter d;
        d.xt = p.rows8t[tile.seg] + (rb >> 4) * (KS * 64);
        d.ax = p.aux[tile.seg] + rb;
        d.bm = p.bmax[tile.seg] + (rb >> 4);
        d.xn = SIM == SIM_COSINE ? p.segs[tile.seg].xnorm_f + rb : nullptr;
        d.vrow0 = (uint32_t)(p.seg_vrow[tile.seg] + rb);
        d.nrows = (int32_t)(pilot ? min<int64_t>(64, re - rb) : re - rb);   // the pilot: one 64-row step
        d.list = tix * 4 + quarter;
        d.shard = tile.shard;
        d.seg = tile.seg;
        s_quart[i] = d;
    }

    // this lane's queries: wq0 + qb·16 + col
    const int wq0 = wave * 64;
    i32x4 bfr[KS][QB];
    float sb[QB], QY[QB], QZ[QB], Q0[QB], zq[QB], tq[QB], qnd[QB];   // qnd: |q|² in the device lane order (COSINE)
    uint64_t tkey[QB], qvm[QB];
    const float QW = __double2float_ru((double)p.gam * (1.0 + 0x1p-18));
    const float g2m = 1.0f - p.g2;
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

    // the workgroup's steps: its quarters' 64-row steps back to back (empty quarters take none)
    auto steps_of = [&](int q) { return (s_quart[q].nrows + 63) >> 6; };
    int total = 0;
    for (int q = 0; q < n_mine; ++q) total += steps_of(q);
    const uint32_t ring_lds =
        __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(__attribute__((address_space(3))) char*)smem);
    int iq = 0, ist = 0;   // the next step to issue: quarter iq of mine, its step ist
    while (iq < n_mine && steps_of(iq) == 0) ++iq;
    auto advance = [&](int& q, int& st) {
        if (++st < steps_of(q)) return;
        st = 0;
        do ++q; while (q < n_mine && steps_of(q) == 0);
    };
    // this wave's group of the step → slot; rows past the quarter load a valid group (masked later)
    auto issue = [&](int slot) {
        const WideQuarter& d = s_quart[iq];
        const int r0 = 16 * (4 * ist + wave);
        const int rv = r0 < d.nrows ? r0 : 0;
        const uint32_t dst = ring_lds + (uint32_t)(slot * SLOT + wave * GB);
        const int perm = (ablate & 4) ? lane : (lane & 15) * 4 + (lane >> 4);   // MFMA operand order: row lane & 15,
                                                                                  // 16-B chunk lane >> 4
        const int4* src = d.xt + (rv >> 4) * (KS * 64);
#pragma unroll
        for (int s = 0; s < KS; ++s) glds16(src + s * 64 + perm, dst + s * 1024);
        if (lane <= 16) {
            const void* asrc = lane < 16 ? static_cast<const void*>(d.ax + min(rv + lane, d.nrows - 1))
                                         : static_cast<const void*>(d.bm + (rv >> 4));
            glds16(asrc, dst + KS * 1024);
        }
        advance(iq, ist);
    };

#ifdef OSK_TESTING
    uint32_t n_events = 0, n_pairs = 0;   // insertion events (wave-uniform) and quick-test passes (per lane)
#endif
    float ca[QB], cb[QB];
    // a quarter ends: its lists (this wave's queries, 4 per pass of 16 lanes) → the settle's arrays, zeroed
    auto flush = [&](const WideQuarter& d) {
        const int q_end = min(wq0 + 64, p.q_count);
        for (int q0 = wq0; q0 < q_end; q0 += 4) {
            const int qg = q0 + (lane >> 4), e = lane & 15;
            const uint64_t lkb = s_lk[qg * kKQ + e];
            const uint32_t lpb = s_lp[qg * kKQ + e];
            uint32_t m = lkb ? lpb : 0u;
#pragma unroll
            for (int o = 8; o >= 1; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
            if (qg < q_end) {
                const size_t l = (size_t)(p.q0 + qg) * p.n_lists + d.list;
                p.cand[l * kKQ + e] = lkb;
                p.cand_lb[l * kKQ + e] = lpb;
                if (e == 0) p.list_lbmax[l] = m;
                s_lk[qg * kKQ + e] = 0ull;
                s_lp[qg * kKQ + e] = 0u;
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
                if (grp == 0 && qi < p.q_count) p.pilot_keys[(size_t)qi * n_quarters + d.list] = 0ull;
            }
        } else {
            flush(d);   // (the LDS lists are all zero here)
        }
    }
    if (total > 0) {
        for (int st = 0; st < NS - 1 && st < total; ++st) issue(st);
        int s_issue = (NS - 1) % NS, s_read = 0;
        int pq = -1, pst = 0;   // the step being processed: quarter pq of mine, its step pst
        for (int i = 0; i < total; ++i) {
            // this wave's DMAs of step i have landed (steps i+1 … i+NS−2 may still be in flight); every wave's
            // have once all pass the barrier, which also retires every wave's reads of step i − 1's slot
            if (i + NS - 1 <= total)
                vm_wait<(NS - 2) * OPS>();
            else
                vm_wait<0>();
            if (!(ablate & 8)) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            if (i + NS - 1 < total) {
                issue(s_issue);
                s_issue = s_issue + 1 == NS ? 0 : s_issue + 1;
            }
            const char* slot = smem + s_read * SLOT;
            s_read = s_read + 1 == NS ? 0 : s_read + 1;
            if (pq < 0 || ++pst == steps_of(pq)) {   // a new quarter: flush the last one, take its floors
                if (pq >= 0 && !pilot) flush(s_quart[pq]);
                do ++pq; while (steps_of(pq) == 0);
                pst = 0;
                const int sh = s_quart[pq].shard;
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) {
                    const int qi = wq0 + qb * 16 + col;
                    const uint32_t f = floor_lds ? (qi < kWideQ ? s_floor[sh * kWideQ + qi] : 0u) : floor_of(qi, sh);
                    tkey[qb] = (uint64_t)f << 32;
                    tq[qb] = sq8_quick(sim, tkey[qb], sqrtf(qnd[qb]), p.cos_slack);
                }
            }
            const WideQuarter& d = s_quart[pq];
            const int n_groups = (d.nrows + 15) >> 4;
            // the step's row maxima (the four blocks' precomputed ones) → this step's quick-test constants
            float4 bm = *reinterpret_cast<const float4*>(slot + KS * 1024 + 256);
#pragma unroll
            for (int g = 1; g < 4; ++g) {
                const float4 b = *reinterpret_cast<const float4*>(slot + g * GB + KS * 1024 + 256);
                bm = make_float4(fmaxf(bm.x, b.x), fmaxf(bm.y, b.y), fmaxf(bm.z, b.z), fminf(bm.w, b.w));
            }
#pragma unroll
            for (int qb = 0; qb < QB; ++qb)
                quick_consts<SIM>(tq[qb], sb[qb], QY[qb], QZ[qb], Q0[qb], QW, zq[qb], g2m, bm, ca[qb], cb[qb]);
            uint64_t pbest[QB] = {0ull, 0ull, 0ull, 0ull};   // the pilot: per query the best sampled key
            for (int g = 0; g < 4; ++g) {
                const int gi = 4 * pst + g;
                if (gi >= n_groups) break;
                const char* gb = slot + g * GB;
                const float4* gaux = reinterpret_cast<const float4*>(gb + KS * 1024);
                const int r0 = 16 * gi;   // rows of the quarter
                const int nr = min(16, d.nrows - r0);
                i32x4 a[KS];
#pragma unroll
                for (int s = 0; s < KS; ++s) a[s] = *reinterpret_cast<const i32x4*>(gb + s * 1024 + lane * 16);
                float ar[4], wr[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float4 x = gaux[4 * grp + r];
                    ar[r] = x.x;
                    wr[r] = x.w;
                    if constexpr (SIM == SIM_COSINE) ar[r] = x.x / __builtin_amdgcn_sqrtf(x.w);   // (0/0 = NaN: passes)
                }
                i32x4 acc[QB];
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) acc[qb] = i32x4{0, 0, 0, 0};
                if (ablate & 2) {
#pragma unroll
                    for (int s = 0; s < KS; ++s) acc[0] ^= a[s];
                } else {
#pragma unroll
                    for (int s = 0; s < KS; ++s)
#pragma unroll
                        for (int qb = 0; qb < QB; ++qb)
                            acc[qb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[s], bfr[s][qb], acc[qb], 0, 0, 0);
                }
                if (pilot) {   // the quarter's first 64 rows: per query the best lower-bound key → pbest
#pragma unroll
                    for (int qb = 0; qb < QB; ++qb) {
                        const int qi = wq0 + qb * 16 + col;
                        const float4 qc = s_qc[qi];
                        uint64_t best = 0ull;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int rr = 4 * grp + r;
                            const float4 ax = gaux[rr];
                            float xnd = 0.0f;
                            if (SIM == SIM_COSINE && rr < nr) xnd = d.xn[r0 + rr];
                            float lo, hi;
                            sq8_bounds(sim, (float)acc[qb][r], ax, qc, p.gam, p.g2, lo, hi);
                            const float lb = SIM == SIM_EUCLIDEAN ? score_f32_l2(hi) : score_f32(sim, lo, qnd[qb], xnd);
                            const uint64_t key = rr < nr ? make_key(lb, d.vrow0 + (uint32_t)(r0 + rr)) : 0ull;
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
                    continue;
                }
                if (ablate & 1) {
                    if (acc[0][0] + acc[QB - 1][3] == 0x7FFFFFFF && ar[0] == 1.0f) s_lp[tid] = 1u;
                    continue;
                }
                // the quick test: one fma + one compare per (row, query); a lane's passing pairs of query block
                // qb folded into one mask right away (the insertion loop re-evaluates the few it needs)
                auto quick = [&](int qb, int r) {
                    const float I = (float)acc[qb][r];
                    float t;
                    if constexpr (SIM == SIM_EUCLIDEAN) t = fmaf(I, ar[r], -fmaf(wr[r], ca[qb], cb[qb]));
                    else t = fmaf(I, ar[r], -ca[qb]);
                    return !(t < 0.0f) && 4 * grp + r < nr;
                };
                uint64_t qm = 0ull;   // the wave's queries with a passing pair (wave-uniform)
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) {
                    const bool any = quick(qb, 0) | quick(qb, 1) | quick(qb, 2) | quick(qb, 3);   // (no short-circuit)
                    const uint64_t bl = __ballot(any) & qvm[qb];
                    qm |= ((bl | (bl >> 16) | (bl >> 32) | (bl >> 48)) & 0xFFFFull) << (16 * qb);
                }
#ifdef OSK_TESTING
                n_events += __popcll(qm);
#endif
                // The passing pairs, one query at a time.  A list that is not full is unordered: its rows are
                // appended (no insertion sort per row); when it fills it is sorted once and from then on
                // keeps its best kKQ by upper bound (sq8_mfma's insertion), its 16th key the threshold.
                while (qm) {
                    const int b = __builtin_ctzll(qm);
                    qm &= qm - 1ull;
                    const int bq = b >> 4, bc = b & 15;
                    const int qg = wq0 + b;
                    const int o0 = qg * kKQ;
                    uint64_t lkb = lane < kKQ ? s_lk[o0 + lane] : 0ull;
                    const int cnt = __popcll(__ballot(lkb != 0ull));   // (keys are never 0)
                    const float4 qcb = s_qc[qg];
#pragma unroll
                    for (int qb = 0; qb < QB; ++qb) {
                        if (qb != bq) continue;   // (wave-uniform)
                        uint64_t key[4];
                        uint32_t lbs[4];
                        bool o[4];
                        int n = 0;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int rr = 4 * grp + r;
                            o[r] = quick(qb, r) && col == bc;
                            const float4 ax = gaux[rr];
                            float xnd = 0.0f;
                            if (SIM == SIM_COSINE && o[r]) xnd = d.xn[r0 + rr];
                            float lo, hi;
                            sq8_bounds(sim, (float)acc[qb][r], ax, qcb, p.gam, p.g2, lo, hi);
                            const float ub = SIM == SIM_EUCLIDEAN ? score_f32_l2(lo) : score_f32(sim, hi, qnd[qb], xnd);
                            const float lb = SIM == SIM_EUCLIDEAN ? score_f32_l2(hi) : score_f32(sim, lo, qnd[qb], xnd);
                            key[r] = o[r] ? make_key(ub, d.vrow0 + (uint32_t)(r0 + rr)) : 0ull;
                            o[r] = o[r] && key[r] > tkey[qb];   // below the floor: cannot enter the top k
                            lbs[r] = float_to_sortable(lb);
                            n += __popcll(__ballot(o[r]));
#ifdef OSK_TESTING
                            n_pairs += o[r] ? 1 : 0;
#endif
                        }
                        if (cnt + n < kKQ) {   // append: the list stays below kKQ rows
                            int base = cnt;
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                const uint64_t m = __ballot(o[r]);
                                if (o[r]) {
                                    const int pos = base + __popcll(m & ((1ull << lane) - 1ull));
                                    s_lk[o0 + pos] = key[r];
                                    s_lp[o0 + pos] = lbs[r];
                                }
                                base += __popcll(m);
                            }
                            continue;
                        }
                        // the list fills (or is full): sorted descending in lanes 0..kKQ-1, zeros last, then
                        // sq8_mfma's insertion with the 16th key as the threshold
                        uint32_t lpb = lane < kKQ ? s_lp[o0 + lane] : 0u;
                        if (cnt < kKQ) {   // (once per list: ranks from LDS, no readlane chain holding SGPRs)
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
                        for (int r = 0; r < 4; ++r) wave_offer2(key[r], lbs[r], o[r], lkb, lpb, thrb, lane, kKQ);
                        if (lane < kKQ) {
                            s_lk[o0 + lane] = lkb;
                            s_lp[o0 + lane] = lpb;
                        }
                        if (col == bc && thrb) {   // full: its 16th key joins the floor under the threshold
                            tq[qb] = sq8_quick(sim, thrb > tkey[qb] ? thrb : tkey[qb], sqrtf(qnd[qb]), p.cos_slack);
                            quick_consts<SIM>(tq[qb], sb[qb], QY[qb], QZ[qb], Q0[qb], QW, zq[qb], g2m, bm, ca[qb], cb[qb]);
                        }
                    }
                }
            }
            if (pilot) {   // (a pilot quarter is one step)
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) {
                    const int qi = wq0 + qb * 16 + col;
                    if (grp == 0 && qi < p.q_count) p.pilot_keys[(size_t)qi * n_quarters + d.list] = pbest[qb];
                }
            }
        }
        vm_wait<0>();
        if (pq >= 0 && !pilot) flush(s_quart[pq]);
    }
#ifdef OSK_TESTING
    if (!pilot && p.counters) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) n_pairs += __shfl_xor(n_pairs, o);
        if (lane == 0) {
            atomicAdd(&p.counters[4], (unsigned long long)n_events);
            atomicAdd(&p.counters[5], (unsigned long long)n_pairs);
        }
    }
#endif
}

using WideFn = void (*)(Sq8Params);
// ring depth per KS: the deepest ring that leaves room for the lists, the floors of ≤ 16 shards and ~96
// quarter descriptors in 160 KiB (one workgroup per CU): KS = 2 → 8 steps (74 KB), KS = 4 → 4 (70 KB)
#define OSK_WIDE_SIMS(KS, NS) {sq8_wide<KS, 0, NS>, sq8_wide<KS, 1, NS>, sq8_wide<KS, 2, NS>, sq8_wide<KS, 3, NS>}
static const WideFn kWide[2][4] = {OSK_WIDE_SIMS(2, 8), OSK_WIDE_SIMS(4, 4)};
static constexpr int kWideNS[2] = {8, 4};
static constexpr size_t kLdsCap = 160 * 1024;

static size_t sq8_wide_lds(int ks, int n_shards, int n_mine) {
    const size_t slot = (size_t)4 * (ks * 1024 + 17 * 16);
    return (size_t)kWideNS[ks == 4] * slot + (size_t)kWideQ * kKQ * 12 + (size_t)kWideQ * 16 +
           (n_shards <= kWideMaxFloorShards ? (size_t)n_shards * kWideQ * 4 : 0) + (size_t)n_mine * sizeof(WideQuarter);
}

hipError_t launch_sq8_wide(const Sq8Params& p, hipStream_t s, hipEvent_t ev_start, hipEvent_t ev_stop) {
    if (!sq8_wide_supported(p.units8) || p.q_count < 1 || p.q_count > kWideQ || p.accept || p.gtiles ||
        p.sim < 0 || p.sim > 3 || !p.rows8t || !p.bmax || p.n_lists != 4 * p.n_tiles || p.k < 1 || p.k > kKQ ||
        p.n_shards < 1 || p.wide_grid < 1 || (p.pilot && !p.pilot_keys))
        return hipErrorInvalidValue;
    const int ks = p.units8 <= 8 ? 2 : 4;
    const auto fn = kWide[ks == 4][p.sim];
    const int nq4 = 4 * p.n_tiles;
    int grid = std::min(p.wide_grid, std::max(1, nq4));
    // more workgroups (rounds of the chip) when one CU's share of quarter descriptors does not fit
    while (sq8_wide_lds(ks, p.n_shards, (nq4 + grid - 1) / grid) > kLdsCap) grid *= 2;
    const size_t lds = sq8_wide_lds(ks, p.n_shards, (nq4 + grid - 1) / grid);
    if (ev_start || ev_stop)
        hipExtLaunchKernelGGL(fn, dim3(grid), dim3(kBlock), lds, s, ev_start, ev_stop, 0, p);
    else
        hipLaunchKernelGGL(fn, dim3(grid), dim3(kBlock), lds, s, p);
    return hipGetLastError();
}

}  // namespace osk
