// osk_select.hip — exact top-k for any k ≤ OSK_MAX_K (10000): the select path.
//
// The streaming scans keep each wave's top-k in lanes 0..k-1 (k ≤ 64) and the certified prefilter
// keeps 16-entry wave lists (k ≤ 12).  OpenSearch allows k (and from+size) up to
// index.max_result_window = 10000 (S/index/IndexSettings.java:223-226), and k = 100 is a routine k-NN
// request.  HBM is plentiful, so instead of wider lists this path materialises one small record per
// row and selects on it:
//
//   writer      one record per view row for this query (0 = not an accepted row):
//                 bounds mode (float32 fields, int8 prefilter copy): sortable lower- and upper-bound
//                 scores LB/UB (u32 each) of the certified int8 bound (osk_sq8.hip);
//                 exact mode: the 64-bit hit key (sortable score << 32 | ~doc), the score computed
//                 with the streaming scan's exact arithmetic (fp32 lane order / exact int32 bytes).
//   radix       per shard, T = the k-th largest LB (3 passes of 11-bit digits) or the k-th largest
//               key (6 passes): LDS histograms
//               per tile, global per-shard histograms, one wave picks the digit (RadixState).  A shard
//               with fewer than k accepted rows takes all of them.
//   collect     bounds: rows with UB ≥ T → candidate rows (every row that can reach the shard's top k:
//               k rows have exact ≥ LB ≥ T, so the k-th exact score ≥ T, and a row with UB < T scores
//               below it); exact: keys ≥ T → exactly min(k, accepted) keys.  Wave-aggregated appends.
//   rescore     bounds: each candidate re-scored exactly (the streaming scan's arithmetic) → its key.
//   sort        per shard, the top k of the candidates sorted best first: few candidates → one LDS
//               bitonic sort; many → a radix select of the k-th candidate key (LDS, or global memory past
//               kSelCap = 16384), the k keys ≥ it sorted.  The candidate buffer holds every row of the
//               shard, so nothing can overflow and no host round trip is needed.
// The coordinator merge of large lists (merge_rank): every hit's global rank by binary search in the
// other (sorted) shard lists — (score desc, shardIndex asc, doc asc), [L] TopDocs.merge's order
// (S/action/search/SearchPhaseController.java:224-246) — so S × min(k, from+size) is unbounded.
#include <hip/hip_ext.h>

#include <algorithm>

#include "osk_device.h"
#include "osk_internal.h"
#include "osk_wave.h"

namespace osk {

namespace {

constexpr int kSelThreads = 256;

__device__ __forceinline__ bool row_accepted(const uint64_t* abits, const SegDev& seg, int64_t row, int32_t& doc) {
    doc = seg.ord_to_doc ? seg.ord_to_doc[row] : (int32_t)row;
    return !abits || ((abits[doc >> 6] >> (doc & 63)) & 1ull);
}

// a tile's wave rows: the scans' split (per_wave = ⌈rows / 4R⌉·R)
template <int R>
__device__ __forceinline__ void wave_rows(const TileDev& tile, int wave, int64_t& wb, int64_t& we) {
    const int64_t rows = tile.row_end - tile.row_begin;
    const int64_t per_wave = ((rows + 4 * R - 1) / (4 * R)) * R;
    wb = tile.row_begin + wave * per_wave;
    we = min(wb + per_wave, tile.row_end);
}

// ---- writers ---------------------------------------------------------------------------------

template <int L, int V, bool L2K>
__global__ __launch_bounds__(kSelThreads) void sel_keys_f32(SelParams p) {
    constexpr int R = 64 / L;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform: scalar loop control
    const int t = lane & (L - 1), g = lane / L;
    const TileDev tile = p.tiles[blockIdx.x];
    const SegDev seg = p.segs[tile.seg];
    const uint64_t* abits = p.accept ? p.accept[tile.seg] : nullptr;
    const float4* __restrict__ Q = static_cast<const float4*>(p.q);
    float4 qf[V];
#pragma unroll
    for (int j = 0; j < V; ++j) qf[j] = Q[t + j * L];
    const float qn = (!L2K && p.sim == SIM_COSINE) ? p.qnorm[0] : 0.0f;
    const float4* __restrict__ X = static_cast<const float4*>(seg.rows);
    const int64_t vbase = p.seg_vrow[tile.seg];
    int64_t wb, we;
    wave_rows<R>(tile, wave, wb, we);
    uint32_t nvis = 0;
    for (int64_t r0 = wb; r0 < we; r0 += R) {
        const int64_t row = r0 + g;
        const bool in = row < we;
        int32_t doc = 0;
        const bool valid = in && row_accepted(abits, seg, row, doc);
        const float xn = (!L2K && p.sim == SIM_COSINE && valid) ? seg.xnorm_f[row] : 0.0f;
        const float sc = settle_exact<L, V, L2K>(X + (in ? row : 0) * p.units, valid, p.units, t, qf, p.sim, qn, xn);
        nvis += __popcll(__ballot(t == 0 && valid));
        if (in && t == 0) p.keys[vbase + row] = valid ? make_key(sc, (uint32_t)(seg.doc_base + doc)) : 0ull;
    }
    if (p.visited) add_visited_wg(&p.visited[tile.seg], (uint32_t)nvis);
}

// Byte vectors, exact keys: byte-unit lane configs (L lanes × V 16-B units ≥ the row's units, sq8_scan's),
// U row groups loaded (unconditional, clamped, masked) before any is reduced, and each iteration's U·R
// contiguous rows' keys stored by one instruction (lane j ← row r0 + j).
template <int L, int V, int U>
__global__ __launch_bounds__(kSelThreads) void sel_keys_i8(SelParams p) {
    constexpr int R = 64 / L;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform: scalar loop control
    const int t = lane & (L - 1), g = lane / L;
    const TileDev tile = p.tiles[blockIdx.x];
    const SegDev seg = p.segs[tile.seg];
    const uint64_t* abits = p.accept ? p.accept[tile.seg] : nullptr;
    const int4* __restrict__ Q = static_cast<const int4*>(p.q);
    const int units = p.units;
    int4 qf[V];
    int qn = 0;   // Σq², exact (scan_i8's)
#pragma unroll
    for (int j = 0; j < V; ++j) {
        const int f = t + j * L;
        const int m = f < units ? -1 : 0;
        const int4 v = Q[f < units ? f : 0];
        qf[j] = make_int4(v.x & m, v.y & m, v.z & m, v.w & m);
        qn = __builtin_amdgcn_sdot4(qf[j].x, qf[j].x, qn, false);
        qn = __builtin_amdgcn_sdot4(qf[j].y, qf[j].y, qn, false);
        qn = __builtin_amdgcn_sdot4(qf[j].z, qf[j].z, qn, false);
        qn = __builtin_amdgcn_sdot4(qf[j].w, qf[j].w, qn, false);
    }
    qn = lane_sum<L>(qn);
    const int4* __restrict__ X = static_cast<const int4*>(seg.rows);
    const int64_t vbase = p.seg_vrow[tile.seg];
    int64_t wb, we;
    wave_rows<R>(tile, wave, wb, we);
    uint32_t nvis = 0;
    for (int64_t r0 = wb; r0 < we; r0 += R * U) {
        int4 xv[U][V];
        int32_t xn[U], doc[U];
        bool valid[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t row = r0 + u * R + g;
            const bool in = row < we;
            doc[u] = 0;
            valid[u] = in && row_accepted(abits, seg, row, doc[u]);
            const int64_t rc = in ? row : wb;
            const int4* xr = X + rc * units;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const int f = t + j * L;
                const int4 x = load_i4_nt(xr + (f < units ? f : 0));
                const int m = (valid[u] && f < units) ? -1 : 0;
                xv[u][j] = make_int4(x.x & m, x.y & m, x.z & m, x.w & m);
            }
            xn[u] = seg.xnorm_i[rc];
        }
        uint64_t kv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int acc = 0;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                acc = __builtin_amdgcn_sdot4(xv[u][j].x, qf[j].x, acc, false);
                acc = __builtin_amdgcn_sdot4(xv[u][j].y, qf[j].y, acc, false);
                acc = __builtin_amdgcn_sdot4(xv[u][j].z, qf[j].z, acc, false);
                acc = __builtin_amdgcn_sdot4(xv[u][j].w, qf[j].w, acc, false);
            }
            acc = lane_sum<L>(acc);
            const int32_t x2 = valid[u] ? xn[u] : 0;
            const int32_t sv = p.sim == SIM_EUCLIDEAN ? qn + x2 - 2 * acc : acc;
            const float sc = score_i8(p.sim, sv, qn, x2, p.dim);
            nvis += __popcll(__ballot(t == 0 && valid[u]));
            kv[u] = valid[u] ? make_key(sc, (uint32_t)(seg.doc_base + doc[u])) : 0ull;
        }
        const int src = (lane % R) * L;
        uint64_t ko = 0ull;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)kv[u], src);
            const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(kv[u] >> 32), src);
            if (lane / R == u) ko = ((uint64_t)hi << 32) | lo;
        }
        if (lane < U * R && r0 + lane < we) p.keys[vbase + r0 + lane] = ko;
    }
    if (p.visited) add_visited_wg(&p.visited[tile.seg], (uint32_t)nvis);
}

// COSINE bounds without Java's double transform.  LB/UB only have to bracket the exact score: with
// c = d/√(qn·xn) evaluated in fp32 (two v_rsq, two products: ≤ 2^-20·|c| from the real quotient) and
// Java's (float)(d / sqrt((double)qn·xn)) then (1 + c)/2 within 2^-23 of the real value, an absolute
// slack of 2^-17·max(1, |c|) keeps ub ≥ score(hi) ≥ the exact score ≥ score(lo) ≥ lb.  Degenerate norms
// (0, inf, NaN) take the exact transform.
__device__ __forceinline__ void cos_bounds_fast(float lo, float hi, float qn, float xn, float& lb, float& ub) {
    const float r = rsqrtf(qn) * rsqrtf(xn);
    const float ch = hi * r, cl = lo * r;
    ub = fmaf(0.5f, ch, 0.5f) + 0x1p-17f * fmaxf(1.0f, fabsf(ch));
    lb = fmaxf(0.0f, fmaf(0.5f, cl, 0.5f) - 0x1p-17f * fmaxf(1.0f, fabsf(cl)));
}

// bounds mode: the int8 prefilter copy's certified [lb, ub] score interval per row (sq8_scan's bound),
// U row groups loaded before any is reduced (≈ U·V KiB in flight per wave, as sq8_scan).  FAST: COSINE
// through cos_bounds_fast instead of Java's double transform.
template <int L, int V, bool FILT, int U, bool FAST>
__global__ __launch_bounds__(kSelThreads) void sel_bounds(SelParams p) {
    constexpr int R = 64 / L;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform: scalar loop control
    const int t = lane & (L - 1), g = lane / L;
    const TileDev tile = p.tiles[blockIdx.x];
    const SegDev seg = p.segs[tile.seg];
    const uint64_t* abits = p.accept ? p.accept[tile.seg] : nullptr;
    const int4* __restrict__ X = p.rows8[tile.seg];
    const float4* __restrict__ AX = p.aux[tile.seg];
    const int u8 = p.units8, sim = p.sim;
    int4 qf[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
        const int f = t + j * L;
        const int msk = f < u8 ? -1 : 0;
        const int4 v = p.q8[f < u8 ? f : 0];
        qf[j] = make_int4(v.x & msk, v.y & msk, v.z & msk, v.w & msk);
    }
    const float4 qc = p.qc[0];
    const float qnd = sim == SIM_COSINE ? p.qnorm[0] : 0.0f;
    const int64_t vbase = p.seg_vrow[tile.seg];
    int64_t wb, we;
    wave_rows<R>(tile, wave, wb, we);
    uint32_t nvis = 0;
    for (int64_t r0 = wb; r0 < we; r0 += R * U) {
        int64_t row[U];
        bool in[U], valid[U];
        int4 xv[U][V];
        float4 ax[U];
        uint32_t lbv[U], ubv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            row[u] = r0 + u * R + g;
            in[u] = row[u] < we;
            int32_t doc = 0;
            // (FILT is compile-time: a runtime accept test put a branch with a full load wait between
            // the row groups, so their loads no longer overlapped)
            valid[u] = in[u];
            if constexpr (FILT) valid[u] = valid[u] && (!abits || row_accepted(abits, seg, row[u], doc));
            // loads on a clamped row, results masked (no load under a branch: those serialise)
            const int64_t rc = in[u] ? row[u] : wb;
            const int4* xr = X + rc * u8;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const int f = t + j * L;
                const int4 x = load_i4_nt(xr + (f < u8 ? f : 0));
                const int m = (valid[u] && f < u8) ? -1 : 0;
                xv[u][j] = make_int4(x.x & m, x.y & m, x.z & m, x.w & m);
            }
            ax[u] = AX[rc];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int acc = 0;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                acc = __builtin_amdgcn_sdot4(xv[u][j].x, qf[j].x, acc, false);
                acc = __builtin_amdgcn_sdot4(xv[u][j].y, qf[j].y, acc, false);
                acc = __builtin_amdgcn_sdot4(xv[u][j].z, qf[j].z, acc, false);
                acc = __builtin_amdgcn_sdot4(xv[u][j].w, qf[j].w, acc, false);
            }
            acc = lane_sum<L>(acc);
            float lo, hi;
            sq8_bounds(sim, (float)acc, ax[u], qc, p.gam, p.g2, lo, hi);
            const float xnd = (sim == SIM_COSINE && valid[u]) ? seg.xnorm_f[row[u]] : 0.0f;
            float ub, lb;
            const bool degen = !(qnd > 0.0f && qnd < __builtin_inff() && xnd > 0.0f && xnd < __builtin_inff());
            if (FAST && sim == SIM_COSINE && !__ballot(valid[u] && degen)) {   // (wave-uniform)
                cos_bounds_fast(lo, hi, qnd, xnd, lb, ub);
            } else {
                ub = sim == SIM_EUCLIDEAN ? score_f32_l2(lo) : score_f32(sim, hi, qnd, xnd);
                lb = sim == SIM_EUCLIDEAN ? score_f32_l2(hi) : score_f32(sim, lo, qnd, xnd);
            }
            nvis += __popcll(__ballot(t == 0 && valid[u]));
            // every real score is ≥ 0, whose sortable form is ≥ 2^31: 0 = no row.  A NaN bound (COSINE with a zero
            // query or row: its exact score is NaN too) is no row either — a NaN is never a hit (make_key), and
            // the select must not count it among the k it keeps
            const bool cand = valid[u] && lb == lb && ub == ub;
            lbv[u] = cand ? float_to_sortable(lb) : 0u;
            ubv[u] = cand ? float_to_sortable(ub) : 0u;
        }
        // the iteration's U·R rows are contiguous (r0 + u·R + g): lane j < U·R gathers row r0 + j's values
        // from the lane holding them (t = 0 of group g = j mod R) and the wave stores them as one
        // contiguous run per array (one store instruction each instead of U partial ones)
        const int j = lane;
        const int src = (j % R) * L;
        uint32_t lbo = 0u, ubo = 0u;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t a = (uint32_t)__shfl((int)lbv[u], src), b = (uint32_t)__shfl((int)ubv[u], src);
            if (j / R == u) {
                lbo = a;
                ubo = b;
            }
        }
        if (j < U * R && r0 + j < we) {
            p.lb[vbase + r0 + j] = lbo;
            p.ub[vbase + r0 + j] = ubo;
        }
    }
    if (p.visited) add_visited_wg(&p.visited[tile.seg], (uint32_t)nvis);
}

// ---- radix select of the k-th largest LB (u32) / key (u64) per shard ---------------------------

// grid: n_shards × kSelRep workgroups, each zeroing one replica (8 bins per thread)
__global__ __launch_bounds__(256) void sel_init(SelParams p) {
    if (blockIdx.x == 0)
        for (int s = threadIdx.x; s < p.n_shards; s += 256) p.state[s] = RadixState{0ull, p.k, 0, 0};
    uint4* h = reinterpret_cast<uint4*>(p.hist + (size_t)blockIdx.x * kSelBins);
    h[2 * threadIdx.x] = make_uint4(0u, 0u, 0u, 0u);
    h[2 * threadIdx.x + 1] = make_uint4(0u, 0u, 0u, 0u);
}

// digit `pass` of a 32-bit (bounds: LB) or 64-bit (exact: key) value: 11-bit digits from the top
__device__ __host__ __forceinline__ void sel_digit(int exact, int pass, int& shift, int& width) {
    const int bits = exact ? 64 : 32;
    const int hi = bits - kSelDigit * pass;   // bits above the digit's top are decided
    width = hi >= kSelDigit ? kSelDigit : hi;
    shift = hi - width;
}

// EXACT is a template parameter: a runtime choice between the two arrays inside the unrolled loop made
// the compiler wait for every load before issuing the next (collect: 145 µs instead of ≈15 at C3)
template <bool EXACT>
__global__ __launch_bounds__(kSelThreads) void sel_hist(SelParams p, int pass) {
    __shared__ uint32_t h[kSelBins];
    const int tid = threadIdx.x;
    const TileDev tile = p.tiles[blockIdx.x];
    const RadixState st = p.state[tile.shard];
    if (st.all) return;   // (block-uniform)
    int shift, width;
    sel_digit(EXACT, pass, shift, width);
    for (int i = tid; i < kSelBins; i += kSelThreads) h[i] = 0u;
    __syncthreads();
    const uint64_t mask = shift + width >= 64 ? 0ull : (~0ull << (shift + width));
    const uint64_t want = st.prefix & mask;
    const uint32_t dmask = (1u << width) - 1u;
    const int64_t vbase = p.seg_vrow[tile.seg];
    for (int64_t r0 = tile.row_begin; r0 < tile.row_end; r0 += 4 * kSelThreads) {
        uint64_t key[4];   // four independent loads in flight per thread
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            // clamped index, unconditional load, masked value: a conditional load made the compiler wait
            // for each load before the next
            const int64_t r = r0 + u * kSelThreads + tid;
            const int64_t rc = min(r, tile.row_end - 1);
            const uint64_t v = EXACT ? p.keys[vbase + rc] : (uint64_t)p.lb[vbase + rc];
            key[u] = r < tile.row_end ? v : 0ull;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            // scores cluster, so a wave's keys often share one bin: one LDS atomic for the wave then
            // (a per-lane atomic on one address serialises 64-fold)
            const bool hit = key[u] && (key[u] & mask) == want;
            const uint32_t bin = (uint32_t)(key[u] >> shift) & dmask;
            const uint64_t act = __ballot(hit);
            if (!act) continue;
            const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)bin, __builtin_ctzll(act));
            const uint64_t same = __ballot(hit && bin == b0);
            if (same == act) {
                if ((threadIdx.x & 63) == __builtin_ctzll(act)) atomicAdd(&h[b0], (uint32_t)__popcll(act));
            } else if (hit) {
                atomicAdd(&h[bin], 1u);
            }
        }
    }
    __syncthreads();
    uint32_t* g = p.hist + ((size_t)tile.shard * kSelRep + blockIdx.x % kSelRep) * kSelBins;
    for (int i = tid; i < kSelBins; i += kSelThreads)
        if (h[i]) atomicAdd(&g[i], h[i]);
}

// one workgroup per shard: the digit holding the krem-th largest value.  Thread i sums bins
// 8i … 8i+7 over the replicas (zeroing them for the next pass), a suffix scan over threads finds the
// owner, the owner walks its bins.
__global__ __launch_bounds__(256) void sel_pick(SelParams p, int pass) {
    __shared__ uint32_t s_wave[4];
    const int s = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform: scalar loop control
    RadixState st = p.state[s];
    if (st.all) return;   // (block-uniform)
    int shift, width;
    sel_digit(p.exact, pass, shift, width);
    uint32_t h[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    uint4* hs = reinterpret_cast<uint4*>(p.hist + (size_t)s * kSelRep * kSelBins);
#pragma unroll
    for (int r = 0; r < kSelRep; ++r) {
        uint4* q = hs + (size_t)r * (kSelBins / 4) + 2 * tid;
        const uint4 a = q[0], b = q[1];
        q[0] = make_uint4(0u, 0u, 0u, 0u);
        q[1] = make_uint4(0u, 0u, 0u, 0u);
        h[0] += a.x; h[1] += a.y; h[2] += a.z; h[3] += a.w;
        h[4] += b.x; h[5] += b.y; h[6] += b.z; h[7] += b.w;
    }
    uint32_t sum = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) sum += h[i];
    uint32_t incl = sum;   // Σ over threads ≥ this one: within the wave, then the higher waves
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_down(incl, o);
        if (lane + o < 64) incl += y;
    }
    if (lane == 0) s_wave[wave] = incl;
    __syncthreads();
    uint32_t total = 0;
    for (int w = 0; w < 4; ++w) {
        total += s_wave[w];
        if (w > wave) incl += s_wave[w];
    }
    const uint32_t above = incl - sum;
    if (pass == 0 && (int64_t)total <= (int64_t)st.krem) {   // ≤ k rows: take every one
        if (tid == 0) {
            st.all = 1;
            p.state[s] = st;
        }
        return;
    }
    if ((int64_t)above < (int64_t)st.krem && (int64_t)st.krem <= (int64_t)incl) {
        uint32_t cum = above;
        for (int i = 7; i >= 0; --i) {
            if ((int64_t)cum + h[i] >= (int64_t)st.krem) {
                st.prefix |= (uint64_t)(tid * 8 + i) << shift;
                st.krem -= (int32_t)cum;
                break;
            }
            cum += h[i];
        }
        p.state[s] = st;
    }
}

// ---- collect / rescore / sort -----------------------------------------------------------------

// Each tile appends its takes (in row order) to its own slots of the shard's candidate region,
// [tile_coff, tile_coff + rows): no atomics.  (One device atomic per wave on a per-shard counter
// serialised on those 8 addresses: 144 µs at C3, k = 100.)  Bounds mode stores the segment row.
template <bool EXACT>
__global__ __launch_bounds__(kSelThreads) void sel_collect(SelParams p) {
    __shared__ int s_wave[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform: scalar loop control
    const TileDev tile = p.tiles[blockIdx.x];
    const int s = tile.shard;
    const RadixState st = p.state[s];
    const uint64_t thr = st.all ? 1ull : st.prefix;
    const int64_t vbase = p.seg_vrow[tile.seg];
    uint64_t* out = p.cand + (size_t)s * p.cap + p.tile_coff[blockIdx.x];
    int run = 0;   // takes so far (block-uniform)
    for (int64_t r0 = tile.row_begin; r0 < tile.row_end; r0 += 4 * kSelThreads) {
        uint64_t val[4];
        bool take[4];
        int c = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t r = r0 + u * kSelThreads + tid;
            const int64_t rc = min(r, tile.row_end - 1);   // unconditional loads (see sel_hist)
            const uint64_t v = EXACT ? p.keys[vbase + rc] : (uint64_t)p.ub[vbase + rc];
            val[u] = r < tile.row_end ? v : 0ull;
        }
        // a thread's takes are ordered u-major; the tile's order only has to be deterministic
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            take[u] = val[u] && val[u] >= thr;
            if (!EXACT) val[u] = (uint64_t)(r0 + u * kSelThreads + tid);
            c += take[u];
        }
        int incl = c;   // wave prefix of the takes
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        if (lane == 63) s_wave[wave] = incl;
        __syncthreads();
        int base = run + incl - c, tot = 0;
        for (int w = 0; w < 4; ++w) {
            const int sw = s_wave[w];
            tot += sw;
            if (w < wave) base += sw;
        }
        __syncthreads();   // s_wave is rewritten by the next iteration
        run += tot;
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (take[u]) out[base++] = val[u];   // ≤ the tile's rows: inside its slots
    }
    if (tid == 0) p.tile_count[blockIdx.x] = run;
}

// bounds mode: one workgroup per tile re-scores its candidates (segment rows) exactly → hit keys
template <int L, int V, bool L2K>
__global__ __launch_bounds__(kSelThreads) void sel_rescore(SelParams p) {
    constexpr int R = 64 / L;
    const int n = p.tile_count[blockIdx.x];
    if (n == 0) return;   // (block-uniform; most tiles)
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform: scalar loop control
    const int t = lane & (L - 1), gr = lane / L;
    const TileDev tile = p.tiles[blockIdx.x];
    const SegDev seg = p.segs[tile.seg];
    const float4* __restrict__ Q = static_cast<const float4*>(p.q);
    float4 qf[V];
#pragma unroll
    for (int j = 0; j < V; ++j) qf[j] = Q[t + j * L];
    const float qn = (!L2K && p.sim == SIM_COSINE) ? p.qnorm[0] : 0.0f;
    uint64_t* c = p.cand + (size_t)tile.shard * p.cap + p.tile_coff[blockIdx.x];
    for (int i0 = wave * R; i0 < n; i0 += 4 * R) {
        const int ci = i0 + gr;
        const bool valid = ci < n;
        // (clamped into the tile: a row index outside it is never loaded)
        const int64_t ord = min(max(valid ? (int64_t)c[ci] : tile.row_begin, tile.row_begin), tile.row_end - 1);
        const int32_t doc = valid ? (seg.ord_to_doc ? seg.ord_to_doc[ord] : (int32_t)ord) : 0;
        const float xn = (!L2K && p.sim == SIM_COSINE && valid) ? seg.xnorm_f[ord] : 0.0f;
        const float sc = settle_exact<L, V, L2K>(static_cast<const float4*>(seg.rows) + ord * p.units, valid, p.units,
                                                 t, qf, p.sim, qn, xn);
        if (valid && t == 0) c[ci] = make_key(sc, (uint32_t)(seg.doc_base + doc));
    }
}

// bitonic sort (descending) of np (a power of two) keys in LDS by 1024 threads
__device__ __forceinline__ void bitonic_desc(uint64_t* sk, int np, int tid) {
    for (int size = 2; size <= np; size <<= 1) {
        for (int j = size >> 1; j > 0; j >>= 1) {
            __syncthreads();
            for (int i = tid; i < np; i += 1024) {
                const int l = i ^ j;
                if (l > i) {
                    const uint64_t a = sk[i], b = sk[l];
                    if ((i & size) == 0 ? a < b : a > b) {
                        sk[i] = b;
                        sk[l] = a;
                    }
                }
            }
        }
    }
    __syncthreads();
}

// The hits of a sorted (descending, zeros last) list of kk keys: its non-zero prefix.  (Candidate keys are
// distinct and non-zero — a NaN score is no candidate, make_key — so this is kk; counted, never assumed.)
__device__ __forceinline__ void sel_count_hits(const uint64_t* sk, int kk, int tid, int32_t* out) {
    if (tid == 0 && (kk == 0 || sk[0] == 0ull)) *out = 0;
    for (int i = tid; i < kk; i += 1024)
        if (sk[i] != 0ull && (i + 1 == kk || sk[i + 1] == 0ull)) *out = i + 1;
}

// per shard: the top k of its n candidate keys (distinct), sorted best first.  Few candidates
// (n ≤ 2k + 256, in LDS): one bitonic sort.  Otherwise: a radix select (8-bit digits, LDS histogram)
// of the kk-th largest key over the candidates (in LDS when n ≤ kSelCap, else in global memory), the
// kk keys ≥ it gathered into the output slots, then sorted in LDS.
// The shard's tiles' candidate runs are packed first (into LDS, or cand2 past kSelCap): 1024 tiles
// at a time, their counts block-scanned, one wave copying each tile's run.
__global__ __launch_bounds__(1024) void sel_sort(SelParams p) {
    extern __shared__ __attribute__((aligned(16))) uint64_t sk[];
    __shared__ uint32_t h[256];
    __shared__ int s_off[1024], s_coff[1024];
    __shared__ int s_wsum[16];
    __shared__ uint64_t s_prefix;
    __shared__ int s_krem, s_ctr;
    const int s = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform: scalar loop control
    const int tb = p.shard_tile_begin[s], te = p.shard_tile_begin[s + 1];
    const uint64_t* c = p.cand + (size_t)s * p.cap;
    // n = Σ tile counts
    int part = 0;
    for (int t = tb + tid; t < te; t += 1024) part += p.tile_count[t];
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
    if (lane == 0) s_wsum[wave] = part;
    __syncthreads();
    int n = 0;
    for (int w = 0; w < 16; ++w) n += s_wsum[w];
    n = min(n, p.cap);
    const int kk = min(p.k, n);
    uint64_t* ok = p.out_keys + (size_t)s * p.k;
    const bool in_lds = n <= kSelCap;
    uint64_t* dst = in_lds ? sk : p.cand2 + (size_t)s * p.cap;
    // pack: per 1024 tiles, their counts block-scanned into s_off, then every entry of the chunk copied
    // by one thread (its tile found by binary search over s_off): all loads independent
    int base = 0;
    for (int t0 = tb; t0 < te; t0 += 1024) {
        __syncthreads();   // s_wsum / s_off / s_coff of the previous round are consumed
        const int t = t0 + tid;
        const int cnt = t < te ? p.tile_count[t] : 0;
        int incl = cnt;
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        if (lane == 63) s_wsum[wave] = incl;
        __syncthreads();
        int pre = incl - cnt, tot = 0;
        for (int w = 0; w < 16; ++w) {
            tot += s_wsum[w];
            if (w < wave) pre += s_wsum[w];
        }
        s_off[tid] = pre;   // chunk-relative start of tile t0 + tid's run
        s_coff[tid] = t < te ? p.tile_coff[t] : 0;
        __syncthreads();
        const int nj = min(1024, te - t0);
        for (int e = tid; e < tot; e += 1024) {
            int lo = 0, hi = nj - 1;   // the last tile whose run starts at or before e
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (s_off[mid] <= e) lo = mid; else hi = mid - 1;
            }
            if (base + e < n) dst[base + e] = c[s_coff[lo] + (e - s_off[lo])];
        }
        base += tot;
    }
    __syncthreads();   // (cand2 is written and read by this workgroup only)
    if (in_lds && n <= 2 * kk + 256) {
        int np = 2;
        while (np < n) np <<= 1;
        for (int i = n + tid; i < np; i += 1024) sk[i] = 0ull;
        bitonic_desc(sk, np, tid);
        for (int i = tid; i < p.k; i += 1024) ok[i] = i < kk ? sk[i] : 0ull;
        sel_count_hits(sk, kk, tid, p.out_counts + s);
        return;
    }
    const uint64_t* src = dst;
    if (tid == 0) {
        s_prefix = 0ull;
        s_krem = kk;
        s_ctr = 0;
    }
    for (int shift = 56; shift >= 0; shift -= 8) {
        if (tid < 256) h[tid] = 0u;
        __syncthreads();
        const uint64_t mask = shift == 56 ? 0ull : (~0ull << (shift + 8));
        const uint64_t want = s_prefix & mask;
        for (int i = tid; i < n; i += 1024) {
            const uint64_t key = src[i];
            if ((key & mask) == want) atomicAdd(&h[(key >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (tid < 64) {   // one wave: 4 bins per lane, suffix scan, the owning lane walks its bins
            uint32_t hb[4], sum = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) sum += (hb[i] = h[tid * 4 + i]);
            uint32_t incl = sum;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_down(incl, o);
                if (tid + o < 64) incl += y;
            }
            const int krem = s_krem;
            const uint32_t above = incl - sum;
            if ((int64_t)above < krem && krem <= (int64_t)incl) {
                uint32_t cum = above;
                for (int i = 3; i >= 0; --i) {
                    if ((int64_t)cum + hb[i] >= krem) {
                        s_prefix |= (uint64_t)(tid * 4 + i) << shift;
                        s_krem = krem - (int)cum;
                        break;
                    }
                    cum += hb[i];
                }
            }
        }
        __syncthreads();
    }
    const uint64_t kth = s_prefix;   // the kk-th largest key: exactly kk keys are ≥ it
    for (int i = tid; i < n; i += 1024) {
        const uint64_t key = src[i];
        if (key >= kth && key != 0ull) {   // (keys are distinct but for empty ones: never more than kk survive)
            const int pos = atomicAdd(&s_ctr, 1);
            if (pos < kk) ok[pos] = key;
        }
    }
    __syncthreads();
    const int ns = min(s_ctr, kk);
    int np = 2;
    while (np < kk) np <<= 1;
    for (int i = tid; i < np; i += 1024) sk[i] = i < ns ? ok[i] : 0ull;
    bitonic_desc(sk, np, tid);
    for (int i = tid; i < p.k; i += 1024) ok[i] = i < kk ? sk[i] : 0ull;
    sel_count_hits(sk, kk, tid, p.out_counts + s);
}

// ---- coordinator merge of large lists ----------------------------------------------------------

struct MergeArgs {
    const uint64_t* keys;
    const int32_t* counts;      // null: a list's hits are its non-zero keys (best first, zero-padded)
    const int32_t* shard_index;
    int n_ranks, sl, k, from, size, nq;
    float* scores;
    int32_t* docs;
    int32_t* shard_out;
    int32_t* count;
    int64_t* total_hits;
    float* max_score;
    XLayout x;
    size_t rw;                  // u64 words per rank block
    int sis;                    // int32 between ranks' shard index arrays
};

// keys of list s = (rank r, local shard j) of query b
__device__ __forceinline__ size_t merge_list(const MergeArgs& a, int b, int s) {
    const int r = s / a.sl, j = s - r * a.sl;
    return (size_t)r * a.rw + ((size_t)b * a.sl + j) * a.k;
}
__device__ __forceinline__ int32_t merge_sidx(const MergeArgs& a, int s) {
    const int r = s / a.sl, j = s - r * a.sl;
    return a.shard_index[r * a.sis + j];
}

// hits of list s (not cut): the count, or the number of non-zero keys (binary search)
__device__ __forceinline__ int merge_hits(const MergeArgs& a, int b, int s) {
    if (a.counts) {
        const int r = s / a.sl, j = s - r * a.sl;
        return a.counts[(size_t)(r * a.nq + b) * a.sl + j];
    }
    const uint64_t* l = a.keys + merge_list(a, b, s);
    int lo = 0, hi = a.k;   // first zero key
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (l[mid]) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// number of entries of a best-first list of n keys whose score is > su (strict) or ≥ su
__device__ __forceinline__ int count_better(const uint64_t* l, int n, uint32_t su, bool or_equal) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const uint32_t v = (uint32_t)(l[mid] >> 32);
        if (or_equal ? v >= su : v > su) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(kSelThreads) void merge_rank(MergeArgs a) {
    if (a.x.hdr) {   // mismatched exchange blocks: merge_stats writes count −1, nothing to rank
        bool bad = false;
        for (int e = 0; e < (a.n_ranks - 1) * kXHdrWords && !bad; ++e)
            bad = a.x.hdr[(size_t)(1 + e / kXHdrWords) * a.rw + e % kXHdrWords] != a.x.hdr[e % kXHdrWords];
        if (bad) return;
    }
    const int b = blockIdx.y;
    const int topn = min(a.k, a.from + a.size);
    const int S = a.n_ranks * a.sl;
    const int64_t e = (int64_t)blockIdx.x * kSelThreads + threadIdx.x;
    if (e >= (int64_t)S * topn) return;
    const int s = (int)(e / topn), i = (int)(e - (int64_t)s * topn);
    const int cs = min(merge_hits(a, b, s), topn);
    if (i >= cs) return;
    const uint64_t key = a.keys[merge_list(a, b, s) + i];
    const uint32_t su = (uint32_t)(key >> 32);
    const int32_t si = merge_sidx(a, s);
    int64_t rank = i;
    for (int s2 = 0; s2 < S && rank < a.from + a.size; ++s2) {
        if (s2 == s) continue;
        const int c2 = min(merge_hits(a, b, s2), topn);
        // another shard's hit ranks before this one on a higher score, or an equal score with a
        // lower shardIndex ([L] TopDocs.merge tie-break; shard indices are distinct)
        rank += count_better(a.keys + merge_list(a, b, s2), c2, su, merge_sidx(a, s2) < si);
    }
    if (rank >= a.from && rank < a.from + a.size) {
        const size_t o = (size_t)b * a.size + (rank - a.from);
        a.scores[o] = sortable_to_float(su);
        a.docs[o] = key_doc(key);
        a.shard_out[o] = si;
    }
}

// per query: TopDocsStats (Σ hits, max top score), the emitted count, empty slots past it
__global__ __launch_bounds__(kSelThreads) void merge_stats(MergeArgs a) {
    __shared__ int64_t s_tot[kSelThreads / 64], s_cut[kSelThreads / 64];
    __shared__ uint32_t s_max[kSelThreads / 64];
    __shared__ int s_bad;
    const int b = blockIdx.x, tid = threadIdx.x;
    if (a.x.hdr) {
        if (tid < 64) {
            const int bad = xchg_header_check(a.x, a.n_ranks, a.rw, tid);
            if (tid == 0) s_bad = bad;
        }
        __syncthreads();
        if (s_bad) {
            if (tid == 0) {
                a.count[b] = -1;
                a.total_hits[b] = -1;
                a.max_score[b] = __builtin_nanf("");
            }
            return;
        }
    }
    const int topn = min(a.k, a.from + a.size);
    const int S = a.n_ranks * a.sl;
    int64_t tot = 0, cut = 0;
    uint32_t mx = 0u;
    for (int s = tid; s < S; s += kSelThreads) {
        const int h = merge_hits(a, b, s);
        tot += h;
        cut += min(h, topn);
        if (h > 0) mx = max(mx, (uint32_t)(a.keys[merge_list(a, b, s)] >> 32));
    }
    for (int o = 32; o > 0; o >>= 1) {
        tot += __shfl_xor(tot, o);
        cut += __shfl_xor(cut, o);
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    }
    if ((tid & 63) == 0) {
        s_tot[tid >> 6] = tot;
        s_cut[tid >> 6] = cut;
        s_max[tid >> 6] = mx;
    }
    __syncthreads();
    tot = cut = 0;
    mx = 0u;
    for (int w = 0; w < kSelThreads / 64; ++w) {
        tot += s_tot[w];
        cut += s_cut[w];
        mx = max(mx, s_max[w]);
    }
    const int got = (int)max<int64_t>(0, min<int64_t>(a.size, cut - a.from));
    for (int r = got + tid; r < a.size; r += kSelThreads) {
        const size_t o = (size_t)b * a.size + r;
        a.scores[o] = -__builtin_inff();
        a.docs[o] = 0x7FFFFFFF;
        a.shard_out[o] = -1;
    }
    if (tid == 0) {
        a.count[b] = got;
        a.total_hits[b] = tot;
        a.max_score[b] = tot > 0 ? sortable_to_float(mx) : __builtin_nanf("");
    }
}

using SelFn = void (*)(SelParams);
#define OSK_SEL_F32(L, V) {sel_keys_f32<L, V, false>, sel_keys_f32<L, V, true>}
static const SelFn kSelKeysF32[9][2] = {OSK_SEL_F32(4, 2),  OSK_SEL_F32(8, 2),  OSK_SEL_F32(8, 4),
                                        OSK_SEL_F32(16, 4), OSK_SEL_F32(16, 8), OSK_SEL_F32(16, 12),
                                        OSK_SEL_F32(32, 8), OSK_SEL_F32(64, 8), OSK_SEL_F32(64, 16)};
// byte-unit configs (sel_bounds_cfg of the row's 16-B units), 4 row groups per iteration
static const SelFn kSelKeysI8[8] = {sel_keys_i8<4, 1, 4>,  sel_keys_i8<8, 1, 4>,  sel_keys_i8<16, 1, 4>,
                                    sel_keys_i8<16, 2, 4>, sel_keys_i8<16, 3, 4>, sel_keys_i8<16, 4, 4>,
                                    sel_keys_i8<32, 4, 4>, sel_keys_i8<64, 4, 4>};
#define OSK_SEL_RS(L, V) {sel_rescore<L, V, false>, sel_rescore<L, V, true>}
static const SelFn kSelRescore[9][2] = {OSK_SEL_RS(4, 2),  OSK_SEL_RS(8, 2),  OSK_SEL_RS(8, 4),
                                        OSK_SEL_RS(16, 4), OSK_SEL_RS(16, 8), OSK_SEL_RS(16, 12),
                                        OSK_SEL_RS(32, 8), OSK_SEL_RS(64, 8), OSK_SEL_RS(64, 16)};
// int8 prefilter lane configs by 16-byte units (sq8_cfg's) × writer variant (tune sel_writer):
// 0 = U 4, Java transform; 1 = U 4, fast COSINE bounds; 2 = U 2, fast; 3 = U 1, fast
#define OSK_SEL_B(L, V)                                                                                          \
    {{sel_bounds<L, V, false, 4, false>, sel_bounds<L, V, true, 4, false>},                                   \
     {sel_bounds<L, V, false, 4, true>, sel_bounds<L, V, true, 4, true>},                                     \
     {sel_bounds<L, V, false, 2, true>, sel_bounds<L, V, true, 2, true>},                                     \
     {sel_bounds<L, V, false, 1, true>, sel_bounds<L, V, true, 1, true>}}
static const SelFn kSelBounds[8][4][2] = {OSK_SEL_B(4, 1),  OSK_SEL_B(8, 1),  OSK_SEL_B(16, 1), OSK_SEL_B(16, 2),
                                          OSK_SEL_B(16, 3), OSK_SEL_B(16, 4), OSK_SEL_B(32, 4), OSK_SEL_B(64, 4)};
static int sel_bounds_cfg(int u8) {
    return u8 <= 4 ? 0 : u8 <= 8 ? 1 : u8 <= 16 ? 2 : u8 <= 32 ? 3 : u8 <= 48 ? 4 : u8 <= 64 ? 5 : u8 <= 128 ? 6 : 7;
}

}  // namespace

hipError_t launch_select_one(const SelParams& p, int cfg, hipStream_t s, hipEvent_t ev_start, hipEvent_t ev_stop) {
    if (p.n_tiles <= 0) return hipSuccess;
    const dim3 tg(p.n_tiles), tb(kSelThreads);
    hipLaunchKernelGGL(sel_init, dim3(p.n_shards * kSelRep), dim3(256), 0, s, p);
    // the writer (stamped by the profile events when given)
    SelFn writer = p.exact ? (p.enc == ENC_BYTE ? kSelKeysI8[sel_bounds_cfg(p.units)]
                                                : kSelKeysF32[cfg][p.sim == SIM_EUCLIDEAN ? 1 : 0])
                           : kSelBounds[sel_bounds_cfg(p.units8)][p.writer & 3][p.accept ? 1 : 0];
    if (ev_start || ev_stop)
        hipExtLaunchKernelGGL(writer, tg, tb, 0, s, ev_start, ev_stop, 0, p);
    else
        hipLaunchKernelGGL(writer, tg, tb, 0, s, p);
    const int passes = ((p.exact ? 64 : 32) + kSelDigit - 1) / kSelDigit;   // 6 (u64) or 3 (u32)
    for (int i = 0; i < passes; ++i) {
        hipLaunchKernelGGL(p.exact ? sel_hist<true> : sel_hist<false>, tg, tb, 0, s, p, i);
        hipLaunchKernelGGL(sel_pick, dim3(p.n_shards), dim3(256), 0, s, p, i);
    }
    hipLaunchKernelGGL(p.exact ? sel_collect<true> : sel_collect<false>, tg, tb, 0, s, p);
    if (!p.exact)
        hipLaunchKernelGGL(kSelRescore[cfg][p.sim == SIM_EUCLIDEAN ? 1 : 0], tg, tb, 0, s, p);
    hipLaunchKernelGGL(sel_sort, dim3(p.n_shards), dim3(1024), (size_t)kSelCap * 8, s, p);
    return hipGetLastError();
}

hipError_t launch_merge_rank(const uint64_t* keys, const int32_t* counts, const int32_t* shard_index, int nq,
                             int n_ranks, int sl, int k, int from, int size, float* scores, int32_t* docs,
                             int32_t* shard_out, int32_t* count, int64_t* total_hits, float* max_score,
                             hipStream_t s, const XLayout& x) {
    MergeArgs a{keys, counts, shard_index, n_ranks, sl, k, from, size, nq, scores, docs, shard_out, count,
                total_hits, max_score, x, x.rank_words ? x.rank_words : (size_t)nq * sl * k,
                x.si_stride ? x.si_stride : sl};
    const int topn = std::min(k, from + size);
    const int64_t n = (int64_t)n_ranks * sl * topn;
    hipLaunchKernelGGL(merge_stats, dim3(nq), dim3(kSelThreads), 0, s, a);
    if (n > 0)
        hipLaunchKernelGGL(merge_rank, dim3((unsigned)((n + kSelThreads - 1) / kSelThreads), nq), dim3(kSelThreads), 0,
                           s, a);
    return hipGetLastError();
}

hipError_t launch_coord_reduce(const uint64_t* shard_keys, const int32_t* shard_counts, const int32_t* shard_index,
                               int nq, int n_ranks, int sl, int k, int from, int size, float* scores, int32_t* docs,
                               int32_t* shard_out, int32_t* count, int64_t* total_hits, float* max_score,
                               hipStream_t s, const XLayout& x) {
    // merge_coord ranks every hit against every other in one workgroup: best for few hits (k = 10:
    // 80 per query); beyond a few hundred the parallel binary-search ranking wins (k = 100, 8 shards:
    // 105 µs → ≈10 µs)
    if ((int64_t)n_ranks * sl * std::min(k, from + size) <= 256)
        return launch_merge_coord(shard_keys, shard_counts, shard_index, nq, n_ranks, sl, k, from, size, scores, docs,
                                  shard_out, count, total_hits, max_score, s, x);
    return launch_merge_rank(shard_keys, shard_counts, shard_index, nq, n_ranks, sl, k, from, size, scores, docs,
                             shard_out, count, total_hits, max_score, s, x);
}

}  // namespace osk
