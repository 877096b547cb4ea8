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
//   * pilot = 1: each workgroup bounds its quarter's first 16 rows and writes the best lower-bound key per
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

// NS: ring depth in 64-row steps.  KS = 2 with NS = 3 fits two workgroups per CU (81 KB of LDS each).
template <int KS, int SIM, int NS>
__global__ __launch_bounds__(kBlock, 2) void sq8_wide(Sq8Params p) {
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    constexpr int QB = kWideQB;
    constexpr int GB = KS * 1024 + 17 * 16;   // one 16-row group in a slot: KS slabs, 16 rows' bound terms, block maxima
    constexpr int SLOT = 4 * GB;              // one step: 4 groups, the DMA of one wave each
    constexpr int OPS = KS + 1;               // LDS-DMA instructions per wave per step
    constexpr int sim = SIM;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int col = lane & 15, grp = lane >> 4;
    const int tix = blockIdx.x >> 2, quarter = blockIdx.x & 3;
    const TileDev tile = p.tiles[tix];
    const SegDev seg = p.segs[tile.seg];
    const int4* __restrict__ XT = p.rows8t[tile.seg];   // tiled: [row / 16][KS][16 rows][4 chunks]
    const float4* __restrict__ AX = p.aux[tile.seg];
    const float4* __restrict__ BM = p.bmax[tile.seg];
    const uint32_t vbase = (uint32_t)p.seg_vrow[tile.seg];
    const int u8 = p.units8;
    const bool pilot = p.pilot != 0;
#ifdef OSK_TESTING
    const int ablate = p.ablate;   // A/B timing only (results wrong): 1 skip the quick tests and lists, 2 skip the MFMAs
#else
    constexpr int ablate = 0;
#endif
    // the quarter: the settle's scan-wave split of the tile with scan_R = kMfmaScanR (list = tile·4 + quarter)
    const int64_t trows = tile.row_end - tile.row_begin;
    const int64_t spw = ((trows + 4 * kMfmaScanR - 1) / (4 * kMfmaScanR)) * kMfmaScanR;
    const int64_t rb = min(tile.row_begin + quarter * spw, tile.row_end);
    const int64_t re = min(rb + spw, tile.row_end);
    const int n_groups = pilot ? (re > rb ? 1 : 0) : (int)((re - rb + 15) / 16);
    const int n_steps = (n_groups + 3) / 4;

    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint64_t* s_lk = reinterpret_cast<uint64_t*>(smem + NS * SLOT);   // [kWideQ][kKQ] upper-bound keys
    uint32_t* s_lp = reinterpret_cast<uint32_t*>(s_lk + kWideQ * kKQ);   // their lower bounds
    float4* s_qc = reinterpret_cast<float4*>(s_lp + kWideQ * kKQ);        // [kWideQ] query bound terms
    for (int i = tid; i < kWideQ * kKQ; i += kBlock) {
        s_lk[i] = 0ull;
        s_lp[i] = 0u;
    }
    for (int i = tid; i < kWideQ; i += kBlock) s_qc[i] = i < p.q_count ? p.qc[i] : make_float4(0.f, 0.f, 0.f, 0.f);

    // this lane's queries: wq0 + qb·16 + col
    const int wq0 = wave * 64;
    i32x4 bfr[KS][QB];
    float sb[QB], QY[QB], QZ[QB], Q0[QB], zq[QB], tq[QB], sqn[QB];
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
        sqn[qb] = (SIM == SIM_COSINE && qv) ? sqrtf(p.qn_dev[qi]) : 0.0f;
        uint64_t t = 0ull;   // the pilot's floor key of (query, this tile's shard)
        if (!pilot && p.thr_keys && qv) {
            const size_t o = (size_t)qi * p.n_shards + tile.shard;
            if (p.thr_counts[o] >= p.k) t = p.thr_keys[o * p.k + p.k - 1];
            if (!(key_score(t) > 0.0f)) t = 0ull;   // (a floor at the score-0 clamp would drop ties: sq8_mfma)
        }
        tkey[qb] = t;
        tq[qb] = sq8_quick(sim, t, sqn[qb], p.cos_slack);
        qvm[qb] = __ballot(qv);
    }
    __syncthreads();   // lists zeroed, s_qc written

    const uint32_t ring_lds =
        __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(__attribute__((address_space(3))) char*)smem);
    // step st: this wave's group 4·st + wave → slot; rows past the quarter load a valid group (masked later)
    auto issue = [&](int st, int slot) {
        const int64_t r0 = rb + 16 * (int64_t)(4 * st + wave);
        const int64_t rv = r0 < re ? r0 : rb;
        const int4* src = XT + (rv >> 4) * (KS * 64);
        const uint32_t dst = ring_lds + (uint32_t)(slot * SLOT + wave * GB);
        const int perm = (lane & 15) * 4 + (lane >> 4);   // MFMA operand order: row lane & 15, 16-B chunk lane >> 4
#pragma unroll
        for (int s = 0; s < KS; ++s) glds16(src + s * 64 + perm, dst + s * 1024);
        if (lane <= 16) {
            const int64_t ra = min(rv + lane, re - 1);
            const void* asrc = lane < 16 ? static_cast<const void*>(AX + ra) : static_cast<const void*>(BM + (rv >> 4));
            glds16(asrc, dst + KS * 1024);
        }
    };

    float ca[QB], cb[QB];
    auto all_consts = [&](float4 bm) {
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
            quick_consts<SIM>(tq[qb], sb[qb], QY[qb], QZ[qb], Q0[qb], QW, zq[qb], g2m, bm, ca[qb], cb[qb]);
    };

    if (n_steps > 0) {
        for (int st = 0; st < NS - 1 && st < n_steps; ++st) issue(st, st);
        int s_issue = (NS - 1) % NS, s_read = 0;
        for (int i = 0; i < n_steps; ++i) {
            // this wave's DMAs of step i have landed (steps i+1 … i+NS−2 may still be in flight); every wave's
            // have once all pass the barrier, which also retires every wave's reads of step i − 1's slot
            if (i + NS - 1 <= n_steps)
                vm_wait<(NS - 2) * OPS>();
            else
                vm_wait<0>();
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            if (i + NS - 1 < n_steps) {
                issue(i + NS - 1, s_issue);
                s_issue = s_issue + 1 == NS ? 0 : s_issue + 1;
            }
            const char* slot = smem + s_read * SLOT;
            s_read = s_read + 1 == NS ? 0 : s_read + 1;
            // the step's row maxima (the four blocks' precomputed ones) → this step's quick-test constants
            float4 bm = *reinterpret_cast<const float4*>(slot + KS * 1024 + 256);
#pragma unroll
            for (int g = 1; g < 4; ++g) {
                const float4 b = *reinterpret_cast<const float4*>(slot + g * GB + KS * 1024 + 256);
                bm = make_float4(fmaxf(bm.x, b.x), fmaxf(bm.y, b.y), fmaxf(bm.z, b.z), fminf(bm.w, b.w));
            }
            all_consts(bm);
            for (int g = 0; g < 4; ++g) {
                const int gi = 4 * i + g;
                if (gi >= n_groups) break;
                const char* gb = slot + g * GB;
                const float4* gaux = reinterpret_cast<const float4*>(gb + KS * 1024);
                const int64_t r0 = rb + 16 * (int64_t)gi;
                const int nr = (int)min<int64_t>(16, re - r0);
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
                if (pilot) {   // the quarter's first 16 rows: per query the best lower-bound key → pilot_keys
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
                            if (SIM == SIM_COSINE && rr < nr) xnd = seg.xnorm_f[r0 + rr];
                            float lo, hi;
                            sq8_bounds(sim, (float)acc[qb][r], ax, qc, p.gam, p.g2, lo, hi);
                            const float lb = SIM == SIM_EUCLIDEAN ? score_f32_l2(hi)
                                                                  : score_f32(sim, lo, sqn[qb] * sqn[qb], xnd);
                            const uint64_t key = rr < nr ? make_key(lb, vbase + (uint32_t)(r0 + rr)) : 0ull;
                            best = key > best ? key : best;
                        }
#pragma unroll
                        for (int o = 16; o <= 32; o <<= 1) {
                            const uint64_t other = ((uint64_t)(uint32_t)__shfl_xor((int)(best >> 32), o) << 32) |
                                                   (uint32_t)__shfl_xor((int)(uint32_t)best, o);
                            best = other > best ? other : best;
                        }
                        if (grp == 0 && qi < p.q_count)
                            p.pilot_keys[(size_t)qi * (4 * p.n_tiles) + blockIdx.x] = best;
                    }
                    continue;
                }
                if (ablate & 1) {
                    if (acc[0][0] + acc[QB - 1][3] == 0x7FFFFFFF && ar[0] == 1.0f) s_lp[tid] = 1u;
                    continue;
                }
                // the quick test: one fma + one compare per (row, query)
                uint64_t pm[QB][4];
#pragma unroll
                for (int qb = 0; qb < QB; ++qb)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float I = (float)acc[qb][r];
                        float t;
                        if constexpr (SIM == SIM_EUCLIDEAN) t = fmaf(I, ar[r], -fmaf(wr[r], ca[qb], cb[qb]));
                        else t = fmaf(I, ar[r], -ca[qb]);
                        pm[qb][r] = __ballot(!(t < 0.0f));
                    }
                uint64_t vm[4] = {~0ull, ~0ull, ~0ull, ~0ull};
                if (nr < 16) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) vm[r] = __ballot(4 * grp + r < nr);
                }
                uint64_t qm = 0ull;   // the wave's queries with a passing pair (wave-uniform)
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) {
                    const uint64_t bl =
                        ((pm[qb][0] & vm[0]) | (pm[qb][1] & vm[1]) | (pm[qb][2] & vm[2]) | (pm[qb][3] & vm[3])) & qvm[qb];
                    qm |= ((bl | (bl >> 16) | (bl >> 32) | (bl >> 48)) & 0xFFFFull) << (16 * qb);
                }
                while (qm) {   // rare once the floor and the lists are set
                    const int b = __builtin_ctzll(qm);
                    qm &= qm - 1ull;
                    const int bq = b >> 4, bc = b & 15;
                    const int qg = wq0 + b;
                    const int o0 = qg * kKQ;
                    uint64_t lkb = lane < kKQ ? s_lk[o0 + lane] : 0ull;
                    uint32_t lpb = lane < kKQ ? s_lp[o0 + lane] : 0u;
                    uint64_t thrb = readlane64(lkb, kKQ - 1);
                    const float4 qcb = s_qc[qg];
#pragma unroll
                    for (int qb = 0; qb < QB; ++qb) {
                        if (qb != bq) continue;   // (wave-uniform)
                        const float qnb = sqn[qb] * sqn[qb];
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int rr = 4 * grp + r;
                            bool o = ((pm[qb][r] >> lane) & 1ull) && rr < nr && col == bc;
                            const float4 ax = gaux[rr];
                            float xnd = 0.0f;
                            if (SIM == SIM_COSINE && o) xnd = seg.xnorm_f[r0 + rr];
                            float lo, hi;
                            sq8_bounds(sim, (float)acc[qb][r], ax, qcb, p.gam, p.g2, lo, hi);
                            const float ub = SIM == SIM_EUCLIDEAN ? score_f32_l2(lo) : score_f32(sim, hi, qnb, xnd);
                            const float lb = SIM == SIM_EUCLIDEAN ? score_f32_l2(hi) : score_f32(sim, lo, qnb, xnd);
                            const uint64_t key = o ? make_key(ub, vbase + (uint32_t)(r0 + rr)) : 0ull;
                            o = o && key > tkey[qb];   // below the floor: cannot enter the top k
                            wave_offer2(key, float_to_sortable(lb), o, lkb, lpb, thrb, lane, kKQ);
                        }
                        if (col == bc) {
                            tq[qb] = sq8_quick(sim, thrb > tkey[qb] ? thrb : tkey[qb], sqn[qb], p.cos_slack);
                            quick_consts<SIM>(tq[qb], sb[qb], QY[qb], QZ[qb], Q0[qb], QW, zq[qb], g2m, bm, ca[qb], cb[qb]);
                        }
                    }
                    if (lane < kKQ) {
                        s_lk[o0 + lane] = lkb;
                        s_lp[o0 + lane] = lpb;
                    }
                }
            }
        }
        vm_wait<0>();
    }
    if (pilot) return;
    if (p.visited && p.q0 == 0 && tid == 0 && re > rb) atomicAdd(&p.visited[tile.seg], (unsigned long long)(re - rb));
    // the lists, 4 queries per pass (16 lanes each): keys, lower bounds and each list's best lower bound
    const int q_end = min(wq0 + 64, p.q_count);
    for (int q0 = wq0; q0 < q_end; q0 += 4) {
        const int qg = q0 + (lane >> 4), e = lane & 15;
        const uint64_t lkb = s_lk[qg * kKQ + e];
        const uint32_t lpb = s_lp[qg * kKQ + e];
        uint32_t m = lkb ? lpb : 0u;
#pragma unroll
        for (int o = 8; o >= 1; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
        if (qg < q_end) {
            const size_t l = (size_t)(p.q0 + qg) * p.n_lists + blockIdx.x;   // = tile·4 + quarter
            p.cand[l * kKQ + e] = lkb;
            p.cand_lb[l * kKQ + e] = lpb;
            if (e == 0) p.list_lbmax[l] = m;
        }
    }
}

using WideFn = void (*)(Sq8Params);
#define OSK_WIDE_SIMS(KS, NS) {sq8_wide<KS, 0, NS>, sq8_wide<KS, 1, NS>, sq8_wide<KS, 2, NS>, sq8_wide<KS, 3, NS>}
static const WideFn kWide[2][4] = {OSK_WIDE_SIMS(2, 3), OSK_WIDE_SIMS(4, 3)};
static constexpr int kWideNS = 3;

static size_t sq8_wide_lds(int ks) {
    return (size_t)kWideNS * 4 * (ks * 1024 + 17 * 16) + (size_t)kWideQ * kKQ * 12 + (size_t)kWideQ * 16;
}

hipError_t launch_sq8_wide(const Sq8Params& p, hipStream_t s, hipEvent_t ev_start, hipEvent_t ev_stop) {
    if (!sq8_wide_supported(p.units8) || p.q_count < 1 || p.q_count > kWideQ || p.accept || p.gtiles ||
        p.sim < 0 || p.sim > 3 || !p.rows8t || !p.bmax || p.n_lists != 4 * p.n_tiles || p.k < 1 || p.k > kKQ ||
        (p.pilot && !p.pilot_keys))
        return hipErrorInvalidValue;
    const int ks = p.units8 <= 8 ? 2 : 4;
    const auto fn = kWide[ks == 4][p.sim];
    const size_t lds = sq8_wide_lds(ks);
    if (ev_start || ev_stop)
        hipExtLaunchKernelGGL(fn, dim3(4 * p.n_tiles), dim3(kBlock), lds, s, ev_start, ev_stop, 0, p);
    else
        hipLaunchKernelGGL(fn, dim3(4 * p.n_tiles), dim3(kBlock), lds, s, p);
    return hipGetLastError();
}

}  // namespace osk
