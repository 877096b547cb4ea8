// osk_kernels.hip — CDNA4 (gfx950) kernels of the exact k-NN scoring path.
//
//   scan_f32 / scan_i8   HBM-streaming exact scoring of a shard's segments fused with a
//                        wavefront top-k select (replaces [L] AbstractKnnVectorQuery.exactSearch's
//                        per-doc VectorSimilarityFunction.compare loop + HitQueue, driven from
//                        S/search/internal/ContextIndexSearcher.java:203-218).
//   merge_shards         per-shard top-k out of the per-tile lists ([L] TopDocs.merge(k, perLeaf)
//                        inside AbstractKnnVectorQuery.rewrite).
//   merge_coord          coordinator reduce (S/action/search/SearchPhaseController.java:224-246,
//                        [L] TopDocs.merge(from, size, …): score desc, shardIndex asc, doc asc).
//   row_norms_*, synth_*, pad_rows   staging helpers.
//
// Design notes (full rationale in DESIGN.md):
//   * A row is scored by L lanes of one wavefront (lane_cfg(dim)); each lane streams V 16-byte
//     units with global_load_dwordx4, so one wave-instruction moves 1 KiB of contiguous-per-row
//     bytes.  The batch-1 path is HBM-bound by ~30x over the VALU; nothing is staged in LDS.
//   * Scores never round-trip through HBM: every wavefront keeps a sorted top-k list in lanes
//     0..k-1 of a register and a wave-uniform threshold; a row-group only costs a ballot unless a
//     score beats the threshold (rare after the first few hundred rows).
#include <hip/hip_ext.h>

#include "osk_device.h"
#include "osk_internal.h"
#include "osk_wave.h"

namespace osk {

// ------------------------------------------------------------------------------------------------
// streaming scan, float32
// ------------------------------------------------------------------------------------------------
// NT: corpus loads carry the non-temporal hint (global_load_dwordx4 … nt): every corpus byte is read
// exactly once per launch, so there is nothing to gain from keeping it in L2 / the Infinity Cache.
template <bool NT>
__device__ __forceinline__ float4 load_row4(const float4* p) {
    if constexpr (NT) {
        typedef float f4v __attribute__((ext_vector_type(4)));
        const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
        return make_float4(v.x, v.y, v.z, v.w);
    } else {
        return *p;
    }
}

template <int L, int V, int NQ, bool L2K, bool NT>
__global__ __launch_bounds__(kBlock) void scan_f32(ScanParams p) {
    constexpr int R = 64 / L;                 // rows per wave-iteration
    constexpr int UP = L * V;                 // padded float4s per query
    constexpr bool QREG = NQ * V * 4 <= 64;   // query fragments in VGPRs, else read from LDS
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float4* sq = reinterpret_cast<float4*>(smem);
    uint64_t* slist = reinterpret_cast<uint64_t*>(smem + (QREG ? 0 : NQ * UP * 16));

    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform: scalar loop control
    const int t = lane & (L - 1), g = lane / L;
    const TileDev tile = p.tiles[blockIdx.x];
    const SegDev seg = p.segs[tile.seg];
    const float4* __restrict__ X = static_cast<const float4*>(seg.rows);
    const float4* __restrict__ Q = static_cast<const float4*>(p.q);
    const int units = p.units;

    float4 qf[QREG ? NQ : 1][QREG ? V : 1];
    if constexpr (QREG) {
#pragma unroll
        for (int b = 0; b < NQ; ++b)
#pragma unroll
            for (int j = 0; j < V; ++j) qf[b][j] = Q[b * UP + t + j * L];
    } else {
        for (int i = tid; i < NQ * UP; i += kBlock) sq[i] = Q[i];
        __syncthreads();
    }
    // COSINE: |q|² in the same lane layout as the row norms (identical bits to row_norms_f32 on the
    // padded query), computed here instead of by a separate launch.
    float qn[NQ];
#pragma unroll
    for (int b = 0; b < NQ; ++b) {
        qn[b] = 0.0f;
        if (!L2K && p.sim == SIM_COSINE) {
            float ax = 0.f, ay = 0.f, az = 0.f, aw = 0.f;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const float4 qv = QREG ? qf[QREG ? b : 0][QREG ? j : 0] : sq[b * UP + t + j * L];
                ax = fmaf(qv.x, qv.x, ax); ay = fmaf(qv.y, qv.y, ay);
                az = fmaf(qv.z, qv.z, az); aw = fmaf(qv.w, qv.w, aw);
            }
            float s = (ax + ay) + (az + aw);
            s = lane_sum<L>(s);
            qn[b] = s;
        }
    }

    const int64_t rows = tile.row_end - tile.row_begin;
    const int64_t per_wave = ((rows + 4 * R - 1) / (4 * R)) * R;
    const int64_t wb = tile.row_begin + wave * per_wave;
    const int64_t we = min(wb + per_wave, tile.row_end);
    const uint64_t* abits = p.accept ? p.accept[tile.seg] : nullptr;
    const int sim = p.sim, k = p.k;

    uint64_t lk[NQ], thr[NQ];
#pragma unroll
    for (int b = 0; b < NQ; ++b) { lk[b] = 0ull; thr[b] = 0ull; }
    uint32_t nvis = 0;

    walk_rows<R>(wb, we, abits, seg.ord_to_doc, lane, g, [&](const int64_t row, bool valid, bool accepted_known) {
        int32_t doc = 0;
        if (valid) {
            doc = seg.ord_to_doc ? seg.ord_to_doc[row] : (int32_t)row;
            if (abits && !accepted_known) valid = (abits[doc >> 6] >> (doc & 63)) & 1ull;
        }
        float4 xv[V];
        const float4* xr = X + row * units;
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const int f = t + j * L;
            xv[j] = (valid && f < units) ? load_row4<NT>(xr + f) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        float xn = 0.0f;
        if (!L2K && sim == SIM_COSINE && valid) xn = seg.xnorm_f[row];
        nvis += __popcll(__ballot(t == 0 && valid));

#pragma unroll
        for (int b = 0; b < NQ; ++b) {
            float ax = 0.f, ay = 0.f, az = 0.f, aw = 0.f;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const float4 qv = QREG ? qf[QREG ? b : 0][QREG ? j : 0] : sq[b * UP + t + j * L];
                if constexpr (L2K) {
                    const float dx = xv[j].x - qv.x, dy = xv[j].y - qv.y;
                    const float dz = xv[j].z - qv.z, dw = xv[j].w - qv.w;
                    ax = fmaf(dx, dx, ax); ay = fmaf(dy, dy, ay);
                    az = fmaf(dz, dz, az); aw = fmaf(dw, dw, aw);
                } else {
                    ax = fmaf(xv[j].x, qv.x, ax); ay = fmaf(xv[j].y, qv.y, ay);
                    az = fmaf(xv[j].z, qv.z, az); aw = fmaf(xv[j].w, qv.w, aw);
                }
            }
            float s = (ax + ay) + (az + aw);
            s = lane_sum<L>(s);
            float sc;
            if constexpr (L2K) sc = score_f32_l2(s);
            else sc = score_f32(sim, s, qn[b], xn);
            const uint64_t key = valid ? make_key(sc, (uint32_t)(seg.doc_base + doc)) : 0ull;
            wave_offer(key, t == 0, lk[b], thr[b], lane, k);
        }
    });

    if (p.visited && p.q0 == 0) add_visited_wg(&p.visited[tile.seg], (uint32_t)nvis);

#pragma unroll
    for (int b = 0; b < NQ; ++b) slist[(b * 4 + wave) * 64 + lane] = lane < k ? lk[b] : 0ull;
    __syncthreads();
    if (wave == 0) {
#pragma unroll
        for (int b = 0; b < NQ; ++b) {
            block_fold(slist + b * 4 * 64, lk[b], thr[b], lane, k);
            if (b < p.q_count && lane < k)
                p.cand[((size_t)(p.q0 + b) * p.n_tiles + blockIdx.x) * k + lane] = lk[b];
        }
    }
}

// ------------------------------------------------------------------------------------------------
// streaming scan, int8 (exact int32 sums: Σab via v_dot4_i32_i8; d² = |q|² + |x|² − 2Σab)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int dot4_i8(int a, int b, int c) {
    return __builtin_amdgcn_sdot4(a, b, c, false);
}

template <int L, int V, int NQ>
__global__ __launch_bounds__(kBlock) void scan_i8(ScanParams p) {
    constexpr int R = 64 / L;
    constexpr int UP = L * V;
    constexpr bool QREG = NQ * V * 4 <= 64;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int4* sq = reinterpret_cast<int4*>(smem);
    uint64_t* slist = reinterpret_cast<uint64_t*>(smem + (QREG ? 0 : NQ * UP * 16));

    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform: scalar loop control
    const int t = lane & (L - 1), g = lane / L;
    const TileDev tile = p.tiles[blockIdx.x];
    const SegDev seg = p.segs[tile.seg];
    const int4* __restrict__ X = static_cast<const int4*>(seg.rows);
    const int4* __restrict__ Q = static_cast<const int4*>(p.q);
    const int units = p.units;

    int4 qf[QREG ? NQ : 1][QREG ? V : 1];
    if constexpr (QREG) {
#pragma unroll
        for (int b = 0; b < NQ; ++b)
#pragma unroll
            for (int j = 0; j < V; ++j) qf[b][j] = Q[b * UP + t + j * L];
    } else {
        for (int i = tid; i < NQ * UP; i += kBlock) sq[i] = Q[i];
        __syncthreads();
    }
    int32_t qn[NQ];   // Σq² (exact) over this wave's L-lane group
#pragma unroll
    for (int b = 0; b < NQ; ++b) {
        int acc = 0;
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const int4 qv = QREG ? qf[QREG ? b : 0][QREG ? j : 0] : sq[b * UP + t + j * L];
            acc = dot4_i8(qv.x, qv.x, acc); acc = dot4_i8(qv.y, qv.y, acc);
            acc = dot4_i8(qv.z, qv.z, acc); acc = dot4_i8(qv.w, qv.w, acc);
        }
        acc = lane_sum<L>(acc);
        qn[b] = acc;
    }

    const int64_t rows = tile.row_end - tile.row_begin;
    const int64_t per_wave = ((rows + 4 * R - 1) / (4 * R)) * R;
    const int64_t wb = tile.row_begin + wave * per_wave;
    const int64_t we = min(wb + per_wave, tile.row_end);
    const uint64_t* abits = p.accept ? p.accept[tile.seg] : nullptr;
    const int sim = p.sim, k = p.k, dim = p.dim;

    uint64_t lk[NQ], thr[NQ];
#pragma unroll
    for (int b = 0; b < NQ; ++b) { lk[b] = 0ull; thr[b] = 0ull; }
    uint32_t nvis = 0;

    walk_rows<R>(wb, we, abits, seg.ord_to_doc, lane, g, [&](const int64_t row, bool valid, bool accepted_known) {
        int32_t doc = 0;
        if (valid) {
            doc = seg.ord_to_doc ? seg.ord_to_doc[row] : (int32_t)row;
            if (abits && !accepted_known) valid = (abits[doc >> 6] >> (doc & 63)) & 1ull;
        }
        int4 xv[V];
        const int4* xr = X + row * units;
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const int f = t + j * L;
            xv[j] = (valid && f < units) ? xr[f] : make_int4(0, 0, 0, 0);
        }
        const int32_t xn = valid ? seg.xnorm_i[row] : 0;
        nvis += __popcll(__ballot(t == 0 && valid));

#pragma unroll
        for (int b = 0; b < NQ; ++b) {
            int acc = 0;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const int4 qv = QREG ? qf[QREG ? b : 0][QREG ? j : 0] : sq[b * UP + t + j * L];
                acc = dot4_i8(xv[j].x, qv.x, acc);
                acc = dot4_i8(xv[j].y, qv.y, acc);
                acc = dot4_i8(xv[j].z, qv.z, acc);
                acc = dot4_i8(xv[j].w, qv.w, acc);
            }
            acc = lane_sum<L>(acc);
            const int32_t s = sim == SIM_EUCLIDEAN ? qn[b] + xn - 2 * acc : acc;
            const float sc = score_i8(sim, s, qn[b], xn, dim);
            const uint64_t key = valid ? make_key(sc, (uint32_t)(seg.doc_base + doc)) : 0ull;
            wave_offer(key, t == 0, lk[b], thr[b], lane, k);
        }
    });

    if (p.visited && p.q0 == 0) add_visited_wg(&p.visited[tile.seg], (uint32_t)nvis);

#pragma unroll
    for (int b = 0; b < NQ; ++b) slist[(b * 4 + wave) * 64 + lane] = lane < k ? lk[b] : 0ull;
    __syncthreads();
    if (wave == 0) {
#pragma unroll
        for (int b = 0; b < NQ; ++b) {
            block_fold(slist + b * 4 * 64, lk[b], thr[b], lane, k);
            if (b < p.q_count && lane < k)
                p.cand[((size_t)(p.q0 + b) * p.n_tiles + blockIdx.x) * k + lane] = lk[b];
        }
    }
}

// ------------------------------------------------------------------------------------------------
// byte vectors, one query, no filter (the C5 int8 case): scan_i8's arithmetic on sq8_scan's loop —
// exact-width lane configs (L lanes × V 16-B units ≥ the row's units, not the fp32 table's), U row
// groups loaded (non-temporal, clamped rows, masked values) before any is scored, so a wave keeps
// ≈ U·V KiB in flight.  Scores are exact int32 sums, so results equal scan_i8's bit for bit.
// ------------------------------------------------------------------------------------------------
template <int L, int V, int U>
__global__ __launch_bounds__(kBlock) void scan_i8_stream(ScanParams p) {
    constexpr int R = 64 / L;
    __shared__ uint64_t slist[4 * 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int t = lane & (L - 1), g = lane / L;
    const TileDev tile = p.tiles[blockIdx.x];
    const SegDev seg = p.segs[tile.seg];
    const int4* __restrict__ X = static_cast<const int4*>(seg.rows);
    const int4* __restrict__ Q = static_cast<const int4*>(p.q);
    const int units = p.units;
    int4 qf[V];
    int qn = 0;   // Σq² (exact)
#pragma unroll
    for (int j = 0; j < V; ++j) {
        const int f = t + j * L;
        const int m = f < units ? -1 : 0;
        const int4 v = Q[f < units ? f : 0];
        qf[j] = make_int4(v.x & m, v.y & m, v.z & m, v.w & m);
        qn = dot4_i8(qf[j].x, qf[j].x, qn); qn = dot4_i8(qf[j].y, qf[j].y, qn);
        qn = dot4_i8(qf[j].z, qf[j].z, qn); qn = dot4_i8(qf[j].w, qf[j].w, qn);
    }
    qn = lane_sum<L>(qn);
    const int64_t rows = tile.row_end - tile.row_begin;
    const int64_t per_wave = ((rows + 4 * R - 1) / (4 * R)) * R;
    const int64_t wb = tile.row_begin + wave * per_wave;
    const int64_t we = min(wb + per_wave, tile.row_end);
    const int sim = p.sim, k = p.k, dim = p.dim;
    uint64_t lk = 0ull, thr = 0ull;
    uint32_t nvis = 0;
    for (int64_t r0 = wb; r0 < we; r0 += R * U) {
        int64_t row[U];
        bool valid[U];
        int4 xv[U][V];
        int32_t xn[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            row[u] = r0 + u * R + g;
            valid[u] = row[u] < we;
            const int64_t rc = valid[u] ? row[u] : wb;   // clamped row: every load is unconditional
            const int4* xr = X + rc * units;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const int f = t + j * L;
                const int4 x = load_i4_nt(xr + (f < units ? f : 0));
                const int m = f < units ? -1 : 0;
                xv[u][j] = make_int4(x.x & m, x.y & m, x.z & m, x.w & m);
            }
            xn[u] = seg.xnorm_i[rc];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int acc = 0;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                acc = dot4_i8(xv[u][j].x, qf[j].x, acc); acc = dot4_i8(xv[u][j].y, qf[j].y, acc);
                acc = dot4_i8(xv[u][j].z, qf[j].z, acc); acc = dot4_i8(xv[u][j].w, qf[j].w, acc);
            }
            acc = lane_sum<L>(acc);
            nvis += __popcll(__ballot(t == 0 && valid[u]));
            const int32_t s = sim == SIM_EUCLIDEAN ? qn + xn[u] - 2 * acc : acc;
            const float sc = score_i8(sim, s, qn, xn[u], dim);
            const int32_t doc = seg.ord_to_doc ? seg.ord_to_doc[valid[u] ? row[u] : wb] : (int32_t)row[u];
            const uint64_t key = valid[u] ? make_key(sc, (uint32_t)(seg.doc_base + doc)) : 0ull;
            wave_offer(key, t == 0, lk, thr, lane, k);
        }
    }
    if (p.visited && p.q0 == 0) add_visited_wg(&p.visited[tile.seg], (uint32_t)nvis);
    slist[wave * 64 + lane] = lane < k ? lk : 0ull;
    __syncthreads();
    if (wave == 0) {
        block_fold(slist, lk, thr, lane, k);
        if (lane < k) p.cand[((size_t)p.q0 * p.n_tiles + blockIdx.x) * k + lane] = lk;
    }
}

// ------------------------------------------------------------------------------------------------
// dispatch tables: lane configs × NQ ∈ {1,2,4,8} × {L2, dot-family}
// ------------------------------------------------------------------------------------------------
int cfg_index(int units) {
    if (units <= 8) return 0;
    if (units <= 16) return 1;
    if (units <= 32) return 2;
    if (units <= 64) return 3;
    if (units <= 128) return 4;
    if (units <= 192) return 5;
    if (units <= 256) return 6;
    if (units <= 512) return 7;
    return 8;
}

using ScanFn = void (*)(ScanParams);

#define OSK_F32_ROW_NT(L, V, NT)                                                                 \
    scan_f32<L, V, 1, true, NT>, scan_f32<L, V, 2, true, NT>, scan_f32<L, V, 4, true, NT>,         \
        scan_f32<L, V, 8, true, NT>, scan_f32<L, V, 1, false, NT>, scan_f32<L, V, 2, false, NT>,   \
        scan_f32<L, V, 4, false, NT>, scan_f32<L, V, 8, false, NT>
#define OSK_F32_ROW(L, V) {OSK_F32_ROW_NT(L, V, false), OSK_F32_ROW_NT(L, V, true)}
#define OSK_I8_ROW(L, V) {scan_i8<L, V, 1>, scan_i8<L, V, 2>, scan_i8<L, V, 4>, scan_i8<L, V, 8>}

static const ScanFn kScanF32[9][16] = {
    OSK_F32_ROW(4, 2),  OSK_F32_ROW(8, 2),  OSK_F32_ROW(8, 4),
    OSK_F32_ROW(16, 4), OSK_F32_ROW(16, 8), OSK_F32_ROW(16, 12),
    OSK_F32_ROW(32, 8), OSK_F32_ROW(64, 8), OSK_F32_ROW(64, 16)};
static const ScanFn kScanI8[9][4] = {
    OSK_I8_ROW(4, 2),  OSK_I8_ROW(8, 2),  OSK_I8_ROW(8, 4),
    OSK_I8_ROW(16, 4), OSK_I8_ROW(16, 8), OSK_I8_ROW(16, 12),
    OSK_I8_ROW(32, 8), OSK_I8_ROW(64, 8), OSK_I8_ROW(64, 16)};
static const int kCfgLV[9][2] = {{4, 2}, {8, 2}, {8, 4}, {16, 4}, {16, 8}, {16, 12},
                                 {32, 8}, {64, 8}, {64, 16}};

// scan_i8_stream's exact-width configs by 16-byte units (sq8_scan's): ≤4 (4,1) ≤8 (8,1) ≤16 (16,1)
// ≤32 (16,2) ≤48 (16,3) ≤64 (16,4) ≤128 (32,4) ≤256 (64,4)
static const ScanFn kScanI8Stream[8] = {scan_i8_stream<4, 1, 4>,  scan_i8_stream<8, 1, 4>,  scan_i8_stream<16, 1, 4>,
                                        scan_i8_stream<16, 2, 4>, scan_i8_stream<16, 3, 4>, scan_i8_stream<16, 4, 4>,
                                        scan_i8_stream<32, 4, 4>, scan_i8_stream<64, 4, 4>};
static int i8_stream_cfg(int u) {
    return u <= 4 ? 0 : u <= 8 ? 1 : u <= 16 ? 2 : u <= 32 ? 3 : u <= 48 ? 4 : u <= 64 ? 5 : u <= 128 ? 6 : 7;
}

static int nq_slot(int nq) { return nq <= 1 ? 0 : nq <= 2 ? 1 : nq <= 4 ? 2 : 3; }
static int nq_of_slot(int s) { return 1 << s; }

Tuning g_tuning;

hipError_t launch_scan(int enc, int cfg, int nq, const ScanParams& p, hipStream_t s, hipEvent_t ev_start,
                       hipEvent_t ev_stop) {
    const int slot = nq_slot(nq);
    const int NQ = nq_of_slot(slot);
    const int V = kCfgLV[cfg][1], L = kCfgLV[cfg][0];
    const bool qreg = NQ * V * 4 <= 64;
    const size_t lds = (qreg ? 0 : (size_t)NQ * L * V * 16) + (size_t)NQ * 4 * 64 * 8;
    ScanFn fn;
    if (enc == ENC_FLOAT32) {
        const bool l2 = p.sim == SIM_EUCLIDEAN;
        fn = kScanF32[cfg][(g_tuning.scan_nt ? 8 : 0) + (l2 ? 0 : 4) + slot];
    } else if (NQ == 1 && !p.accept && p.units <= 256 && g_tuning.i8_stream) {
        fn = kScanI8Stream[i8_stream_cfg(p.units)];
    } else {
        fn = kScanI8[cfg][slot];
    }
    if (ev_start || ev_stop)
        hipExtLaunchKernelGGL(fn, dim3(p.n_tiles), dim3(kBlock), lds, s, ev_start, ev_stop, 0, p);
    else
        hipLaunchKernelGGL(fn, dim3(p.n_tiles), dim3(kBlock), lds, s, p);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// per-row |x|² in the scan's lane layout (f32) — used for COSINE rows and queries
// ------------------------------------------------------------------------------------------------
template <int L, int V>
__global__ __launch_bounds__(kBlock) void row_norms_f32(const float4* __restrict__ X,
                                                        int64_t n_rows, int units,
                                                        float* __restrict__ out) {
    constexpr int R = 64 / L;
    const int lane = threadIdx.x & 63;
    const int t = lane & (L - 1), g = lane / L;
    const int64_t wave_global = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) >> 6;
    for (int64_t r0 = wave_global * R; r0 < n_rows; r0 += n_waves * R) {
        const int64_t row = r0 + g;
        const bool valid = row < n_rows;
        float ax = 0.f, ay = 0.f, az = 0.f, aw = 0.f;
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const int f = t + j * L;
            const float4 x = (valid && f < units) ? X[row * units + f] : make_float4(0.f, 0.f, 0.f, 0.f);
            ax = fmaf(x.x, x.x, ax); ay = fmaf(x.y, x.y, ay);
            az = fmaf(x.z, x.z, az); aw = fmaf(x.w, x.w, aw);
        }
        float s = (ax + ay) + (az + aw);
        s = lane_sum<L>(s);
        if (valid && t == 0) out[row] = s;
    }
}

using NormFn = void (*)(const float4*, int64_t, int, float*);
static const NormFn kNormF32[9] = {row_norms_f32<4, 2>,  row_norms_f32<8, 2>,  row_norms_f32<8, 4>,
                                   row_norms_f32<16, 4>, row_norms_f32<16, 8>, row_norms_f32<16, 12>,
                                   row_norms_f32<32, 8>, row_norms_f32<64, 8>, row_norms_f32<64, 16>};

static int grid_for(int64_t waves_needed) {
    int64_t blocks = (waves_needed + 3) / 4;
    if (blocks < 1) blocks = 1;
    if (blocks > 8192) blocks = 8192;
    return (int)blocks;
}

hipError_t launch_row_norms_f32(const float4* rows, int64_t n_rows, int units, int cfg, float* out,
                                hipStream_t s) {
    const int R = 64 / kCfgLV[cfg][0];
    hipLaunchKernelGGL(kNormF32[cfg], dim3(grid_for((n_rows + R - 1) / R)), dim3(kBlock), 0, s,
                       rows, n_rows, units, out);
    return hipGetLastError();
}

// byte rows: Σx² exact (order irrelevant); one wave per row.
__global__ __launch_bounds__(kBlock) void row_norms_i8(const int4* __restrict__ X, int64_t n_rows,
                                                       int units, int32_t* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t wave_global = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) >> 6;
    for (int64_t row = wave_global; row < n_rows; row += n_waves) {
        int acc = 0;
        for (int f = lane; f < units; f += 64) {
            const int4 x = X[row * units + f];
            acc = dot4_i8(x.x, x.x, acc); acc = dot4_i8(x.y, x.y, acc);
            acc = dot4_i8(x.z, x.z, acc); acc = dot4_i8(x.w, x.w, acc);
        }
        for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m);
        if (lane == 0) out[row] = acc;
    }
}

hipError_t launch_row_norms_i8(const int4* rows, int64_t n_rows, int units, int32_t* out,
                               hipStream_t s) {
    hipLaunchKernelGGL(row_norms_i8, dim3(grid_for(n_rows)), dim3(kBlock), 0, s, rows, n_rows,
                       units, out);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// synthetic corpus (one wave per row; identical values to osk_synth_host)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void synth_rows(void* __restrict__ out, int64_t n_rows, int dim,
                                                     int units, int enc, uint64_t seed_mix, int dist,
                                                     int64_t row0) {
    const int lane = threadIdx.x & 63;
    const int64_t wave_global = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) >> 6;
    for (int64_t r = wave_global; r < n_rows; r += n_waves) {
        const uint64_t grow = (uint64_t)(row0 + r);
        if (enc == ENC_BYTE) {
            int8_t* orow = static_cast<int8_t*>(out) + r * (int64_t)units * 16;
            for (int f = lane; f < units; f += 64) {
                alignas(16) int8_t v[16];
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int c = f * 16 + e;
                    v[e] = c < dim ? synth_i8(synth_bits(seed_mix, grow, dim, c)) : (int8_t)0;
                }
                *reinterpret_cast<int4*>(orow + f * 16) = *reinterpret_cast<const int4*>(v);
            }
            continue;
        }
        float inv_norm_den = 1.0f;
        if (dist == DIST_NORMALISH_UNIT) {
            float acc = 0.0f;
            for (int c = lane; c < dim; c += 64) {
                const float z = synth_f32_raw(dist, synth_bits(seed_mix, grow, dim, c));
                acc = fmaf(z, z, acc);
            }
            for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m);
            inv_norm_den = sqrtf(acc);
        }
        float4* orow = static_cast<float4*>(out) + r * (int64_t)units;
        for (int f = lane; f < units; f += 64) {
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int c = f * 4 + e;
                float z = c < dim ? synth_f32_raw(dist, synth_bits(seed_mix, grow, dim, c)) : 0.0f;
                if (dist == DIST_NORMALISH_UNIT && c < dim) z = z / inv_norm_den;
                v[e] = z;
            }
            orow[f] = make_float4(v[0], v[1], v[2], v[3]);
        }
    }
}

hipError_t launch_synth(void* rows, int64_t n_rows, int dim, int units, int enc, uint64_t seed,
                        int dist, int64_t row0, hipStream_t s) {
    hipLaunchKernelGGL(synth_rows, dim3(grid_for(n_rows)), dim3(kBlock), 0, s, rows, n_rows, dim,
                       units, enc, splitmix64(seed), dist, row0);
    return hipGetLastError();
}

// copy rows into the padded (16-byte unit) layout; pad bytes are zeroed.
__global__ __launch_bounds__(kBlock) void pad_rows(const uint8_t* __restrict__ src, int64_t src_pitch,
                                                   uint8_t* __restrict__ dst, int64_t dst_pitch,
                                                   int64_t n_rows, int64_t row_bytes) {
    const int lane = threadIdx.x & 63;
    const int64_t wave_global = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) >> 6;
    for (int64_t r = wave_global; r < n_rows; r += n_waves)
        for (int64_t b = lane; b < dst_pitch; b += 64)
            dst[r * dst_pitch + b] = b < row_bytes ? src[r * src_pitch + b] : (uint8_t)0;
}

// Queries → the padded unit layout in one launch: rows [0, nq) copied with zeros past row_bytes,
// rows [nq, nq_pad) (the dummy queries of the last ≤8-query launch) all zero.
__global__ __launch_bounds__(kBlock) void prep_queries(const uint8_t* __restrict__ src, int64_t row_bytes,
                                                       int nq, int4* __restrict__ dst, int units, int nq_pad) {
    const int lane = threadIdx.x & 63;
    const int64_t wave_global = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) >> 6;
    for (int64_t r = wave_global; r < nq_pad; r += n_waves) {
        for (int f = lane; f < units; f += 64) {
            alignas(16) uint8_t v[16];
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int64_t b = (int64_t)f * 16 + e;
                v[e] = (r < nq && b < row_bytes) ? src[r * row_bytes + b] : (uint8_t)0;
            }
            dst[r * units + f] = *reinterpret_cast<const int4*>(v);
        }
    }
}

hipError_t launch_prep_queries(const void* src, int64_t row_bytes, int nq, void* dst, int units, int nq_pad,
                               hipStream_t s) {
    hipLaunchKernelGGL(prep_queries, dim3(grid_for(nq_pad)), dim3(kBlock), 0, s, static_cast<const uint8_t*>(src),
                       row_bytes, nq, static_cast<int4*>(dst), units, nq_pad);
    return hipGetLastError();
}

hipError_t launch_pad_rows(const void* src, int64_t src_pitch, void* dst, int64_t dst_pitch,
                           int64_t n_rows, int64_t row_bytes, hipStream_t s) {
    hipLaunchKernelGGL(pad_rows, dim3(grid_for(n_rows)), dim3(kBlock), 0, s,
                       static_cast<const uint8_t*>(src), src_pitch, static_cast<uint8_t*>(dst),
                       dst_pitch, n_rows, row_bytes);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// per-shard top-k from per-tile lists: one workgroup per (shard, query)
// ------------------------------------------------------------------------------------------------
// (kin: keys per tile in cand — k for tile lists, 1 for one key per tile; the output holds k per shard)
__global__ __launch_bounds__(kBlock) void merge_shards(const uint64_t* __restrict__ cand, int n_tiles,
                                                       const int32_t* __restrict__ shard_tile_begin,
                                                       int n_shards, int k, int kin,
                                                       uint64_t* __restrict__ shard_keys,
                                                       int32_t* __restrict__ shard_counts) {
    __shared__ uint64_t lists[4 * 64];
    const int s = blockIdx.x, b = blockIdx.y;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int t0 = shard_tile_begin[s], t1 = shard_tile_begin[s + 1];
    const uint64_t* c = cand + ((size_t)b * n_tiles + t0) * kin;
    const int64_t n = (int64_t)(t1 - t0) * kin;
    uint64_t lk = 0ull, thr = 0ull;
    for (int64_t base = (int64_t)wave * 64; base < n; base += kBlock) {
        const int64_t i = base + lane;
        const uint64_t key = i < n ? c[i] : 0ull;
        wave_offer(key, true, lk, thr, lane, k);
    }
    lists[wave * 64 + lane] = lane < k ? lk : 0ull;
    __syncthreads();
    if (wave == 0) {
        block_fold(lists, lk, thr, lane, k);
        const size_t o = (size_t)b * n_shards + s;
        if (lane < k) shard_keys[o * k + lane] = lk;
        const int cnt = __popcll(__ballot(lane < k && lk != 0ull));
        if (lane == 0) shard_counts[o] = cnt;
    }
}

hipError_t launch_merge_shards(const uint64_t* cand, int n_tiles, const int32_t* shard_tile_begin,
                               int n_shards, int nq, int k, uint64_t* shard_keys,
                               int32_t* shard_counts, hipStream_t s, int kin) {
    hipLaunchKernelGGL(merge_shards, dim3(n_shards, nq), dim3(kBlock), 0, s, cand, n_tiles,
                       shard_tile_begin, n_shards, k, kin > 0 ? kin : k, shard_keys, shard_counts);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// coordinator reduce: one workgroup per query.  Each shard contributes its first min(k, from+size)
// hits (the shard collector's numDocs cut); hits are ranked by (score desc, shardIndex asc, doc asc)
// and ranks [from, from+size) are emitted.  Σ shard hits → total hits; max top score → max score.
// ------------------------------------------------------------------------------------------------
constexpr int kCoordMax = 4096;   // shard hits considered per query (n_shards · min(k, from+size))

// Slot (s, i) = hit i of shard s, a fixed position: every thread loads its slots' keys at once (no
// per-shard serialisation), then ranks each valid hit against all others.
// Layout: shard s = (rank r, local shard j), s = r·sl + j, its list at ((r·nq + b)·sl + j)·k — the
// rank-major image an all-gather of per-rank [nq][sl][k] lists produces (n_ranks = 1: [nq][S][k]).
// shard_counts null: a list's hits are its non-zero keys (lists are best-first, zero-padded).
__global__ __launch_bounds__(kBlock) void merge_coord(const uint64_t* __restrict__ shard_keys,
                                                      const int32_t* __restrict__ shard_counts,
                                                      const int32_t* __restrict__ shard_index,
                                                      int n_ranks, int sl, int k, int from, int size,
                                                      float* __restrict__ scores,
                                                      int32_t* __restrict__ docs,
                                                      int32_t* __restrict__ shard_out,
                                                      int32_t* __restrict__ count,
                                                      int64_t* __restrict__ total_hits,
                                                      float* __restrict__ max_score, XLayout x) {
    // empty slot = (su 0, shardIndex INT32_MAX, doc INT32_MAX): it never ranks above a hit
    __shared__ __attribute__((aligned(16))) uint32_t s_su[kCoordMax];
    __shared__ __attribute__((aligned(16))) int32_t s_sidx[kCoordMax];
    __shared__ __attribute__((aligned(16))) int32_t s_doc[kCoordMax];
    // per-wave partial sums / maxima (no LDS atomics: a 64-bit LDS atomic add made this one-query
    // kernel 10 µs instead of 3.7 µs — tools/mc_micro.hip)
    __shared__ int s_red_n[kBlock / 64], s_red_total[kBlock / 64];
    __shared__ uint32_t s_red_max[kBlock / 64];
    __shared__ int s_bad;
    const int b = blockIdx.x, tid = threadIdx.x, nq = gridDim.x;
    const int n_shards = n_ranks * sl;
    const int topn = min(k, from + size);
    const int n_slots = n_shards * topn;
    const int n4 = (n_slots + 3) & ~3;   // ≤ kCoordMax (the host checks n_slots ≤ 4096)
    const size_t rw = x.rank_words ? x.rank_words : (size_t)nq * sl * k;
    const int sis = x.si_stride ? x.si_stride : sl;
    // list s = (rank r, local shard j): its count index (r·nq + b)·sl + j (counts exist only for
    // contiguous images), its keys at r·rw + (b·sl + j)·k, its shardIndex at r·sis + j
    auto list = [&](int s) -> size_t {
        const int r = s / sl, j = s - r * sl;
        return ((size_t)(r * nq + b) * sl + j);
    };
    auto keys_of = [&](int s) -> const uint64_t* {
        const int r = s / sl, j = s - r * sl;
        return shard_keys + (size_t)r * rw + ((size_t)b * sl + j) * k;
    };
    auto sidx_of = [&](int s) -> int32_t {
        const int r = s / sl, j = s - r * sl;
        return shard_index[r * sis + j];
    };
    if (x.hdr) {   // every rank's block must come from the same call (xchg_header_check)
        if (tid < 64) {
            const int bad = xchg_header_check(x, n_ranks, rw, tid);
            if (tid == 0) s_bad = bad;
        }
        __syncthreads();
        if (s_bad) {
            if (tid == 0) {
                count[b] = -1;
                total_hits[b] = -1;
                max_score[b] = __builtin_nanf("");
            }
            return;
        }
    }
    // stats (TopDocsStats): Σ hits over the shards, max of their top scores
    int part_total = 0;
    uint32_t part_max = 0u;
    if (shard_counts) {
        for (int s = tid; s < n_shards; s += kBlock) {
            const size_t o = list(s);
            const int c = shard_counts[o];
            const uint64_t top = keys_of(s)[0];
            part_total += c;
            if (c > 0) part_max = max(part_max, (uint32_t)(top >> 32));
        }
    } else if (topn < k) {   // (topn == k: the slot loop below sees every list entry)
        for (int e = tid; e < n_shards * k; e += kBlock) {
            const int s = e / k, i = e - s * k;
            const uint64_t key = keys_of(s)[i];
            part_total += key != 0ull;
            if (i == 0 && key) part_max = max(part_max, (uint32_t)(key >> 32));
        }
    }
    // one round of independent loads per slot (i < topn ≤ k keeps the key load in bounds)
    int mine = 0;
    for (int slot = tid; slot < n4; slot += kBlock) {
        const int s = slot / topn, i = slot - s * topn;
        const bool real = slot < n_slots;
        const uint64_t key = real ? keys_of(s)[i] : 0ull;
        const int c = real && shard_counts ? shard_counts[list(s)] : 0;
        const int32_t si = real ? sidx_of(s) : 0;
        const bool hit = real && (shard_counts ? i < c : key != 0ull);
        s_su[slot] = hit ? (uint32_t)(key >> 32) : 0u;
        s_doc[slot] = hit ? key_doc(key) : INT32_MAX;
        s_sidx[slot] = hit ? si : INT32_MAX;
        mine += hit;
        if (!shard_counts && topn == k && hit && i == 0) part_max = max(part_max, (uint32_t)(key >> 32));
    }
    if (!shard_counts && topn == k) part_total = mine;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mine += __shfl_xor(mine, o);
        part_total += __shfl_xor(part_total, o);
        part_max = max(part_max, (uint32_t)__shfl_xor((int)part_max, o));
    }
    if ((tid & 63) == 0) {
        s_red_n[tid >> 6] = mine;
        s_red_total[tid >> 6] = part_total;
        s_red_max[tid >> 6] = part_max;
    }
    __syncthreads();
    // rank of each hit = number of hits ordered before it.  The slots' 32-bit score keys are read 4
    // at a time (16-byte LDS loads); only a score that occurs more than once (a tie) takes the
    // (shardIndex asc, doc asc) pass.
    for (int i = tid; i < n_slots; i += kBlock) {
        const uint32_t su = s_su[i];
        if (su == 0u && s_sidx[i] == INT32_MAX) continue;   // empty
        const int32_t si = s_sidx[i], d = s_doc[i];
        int rank = 0, eq = 0;
#pragma unroll 4
        for (int j = 0; j < n4; j += 4) {
            const uint4 u4 = *reinterpret_cast<const uint4*>(s_su + j);
            rank += (u4.x > su) + (u4.y > su) + (u4.z > su) + (u4.w > su);
            eq += (u4.x == su) + (u4.y == su) + (u4.z == su) + (u4.w == su);
        }
        if (eq > 1) {
            for (int j = 0; j < n_slots; ++j)
                rank += s_su[j] == su && (s_sidx[j] < si || (s_sidx[j] == si && s_doc[j] < d));
        }
        if (rank >= from && rank < from + size) {
            const size_t o = (size_t)b * size + (rank - from);
            scores[o] = sortable_to_float(su);
            docs[o] = d;
            shard_out[o] = si;
        }
    }
    int n = 0, total = 0;
    uint32_t mx = 0u;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        n += s_red_n[w];
        total += s_red_total[w];
        mx = max(mx, s_red_max[w]);
    }
    const int got = max(0, min(size, n - from));
    for (int r = got + tid; r < size; r += kBlock) {
        const size_t o = (size_t)b * size + r;
        scores[o] = -__builtin_inff();
        docs[o] = 0x7FFFFFFF;
        shard_out[o] = -1;
    }
    if (tid == 0) {
        count[b] = got;
        total_hits[b] = (int64_t)total;
        max_score[b] = total > 0 ? sortable_to_float(mx) : __builtin_nanf("");
    }
}

hipError_t launch_merge_coord(const uint64_t* shard_keys, const int32_t* shard_counts,
                              const int32_t* shard_index, int nq, int n_ranks, int sl, int k, int from,
                              int size, float* scores, int32_t* docs, int32_t* shard_out,
                              int32_t* count, int64_t* total_hits, float* max_score,
                              hipStream_t s, const XLayout& x) {
    hipLaunchKernelGGL(merge_coord, dim3(nq), dim3(kBlock), 0, s, shard_keys, shard_counts,
                       shard_index, n_ranks, sl, k, from, size, scores, docs, shard_out, count,
                       total_hits, max_score, x);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// multi-rank exchange trailer (osk_comm.hip): header + fingerprint of the query bytes + shard indices
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {   // splitmix64 finaliser
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// The fingerprint is Σ mix64(word_i + i·φ) over EVERY 32-bit word of the query bytes (plus the tail bytes
// and the byte count): order-independent, so identical bytes give identical fingerprints on every rank,
// and a batch that differs in any word — its last query only, say — almost surely does not.  (A strided
// sample of 16384 words left up to half of a 22–42-query batch at 768 dims unhashed.)  kXhdrWords per
// workgroup; each adds its partial sum into w[5] (zeroed first by launch_xhdr_fill) with one atomic —
// or, when one workgroup covers the query bytes (≤ 64 KiB: every single-query call), stores it, with no
// memset before; workgroup 0 writes the other header words and the shard indices.
constexpr int64_t kXhdrWords = 16384;
__global__ __launch_bounds__(256) void xhdr_fill(uint64_t* __restrict__ hdr, XHdrWords w,
                                                 const uint8_t* __restrict__ q, int64_t qbytes,
                                                 const int32_t* __restrict__ shard_index, int n_shards, int sl) {
    __shared__ uint64_t s_part[4];
    const int tid = threadIdx.x;
    const int64_t n32 = qbytes >> 2;
    const int64_t e0 = (int64_t)blockIdx.x * kXhdrWords, e1 = min(n32, e0 + kXhdrWords);
    uint64_t h = 0;
    for (int64_t e = e0 + tid; e < e1; e += 256) {
        uint32_t v;
        __builtin_memcpy(&v, q + e * 4, 4);
        h += mix64((uint64_t)v + (uint64_t)e * 0x9E3779B97F4A7C15ull);
    }
    if (blockIdx.x == 0) {
        if (tid < (int)(qbytes & 3)) h += mix64((uint64_t)q[n32 * 4 + tid] + 0xA5A5ull * (uint64_t)(tid + 1));
        if (tid == 0) h += mix64((uint64_t)qbytes);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o);
    if ((tid & 63) == 0) s_part[tid >> 6] = h;
    __syncthreads();
    if (tid == 0) {
        const uint64_t sum = s_part[0] + s_part[1] + s_part[2] + s_part[3];
        if (gridDim.x == 1)
            hdr[5] = sum;
        else
            atomicAdd(reinterpret_cast<unsigned long long*>(hdr + 5), (unsigned long long)sum);
    }
    if (blockIdx.x != 0) return;
    if (tid < kXHdrWords && tid != 5) hdr[tid] = w.w[tid];
    int32_t* si = reinterpret_cast<int32_t*>(hdr + kXHdrWords);
    for (int j = tid; j < sl; j += 256) si[j] = j < n_shards ? shard_index[j] : 0x7FFFFFFF;
}

hipError_t launch_xhdr_fill(uint64_t* hdr, const uint64_t* w, const void* queries, int64_t query_bytes,
                            const int32_t* shard_index, int n_shards, int sl, hipStream_t s) {
    XHdrWords hw;
    for (int i = 0; i < kXHdrWords; ++i) hw.w[i] = w[i];
    const int64_t blocks = std::max<int64_t>(1, ((query_bytes >> 2) + kXhdrWords - 1) / kXhdrWords);
    if (blocks > 1) {   // (one workgroup stores the fingerprint itself)
        hipError_t e = hipMemsetAsync(hdr + 5, 0, sizeof(uint64_t), s);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(xhdr_fill, dim3((unsigned)blocks), dim3(256), 0, s, hdr, hw,
                       static_cast<const uint8_t*>(queries), query_bytes, shard_index, n_shards, sl);
    return hipGetLastError();
}

}  // namespace osk
