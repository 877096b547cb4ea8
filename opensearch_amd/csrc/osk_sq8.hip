// osk_sq8.hip — certified int8 prefilter for exact k-NN over float32 fields (batches below the MFMA
// path).  Lucene analogue: a scalar-quantized copy next to the raw vectors, with the raw vectors
// re-scored ([L] Lucene99ScalarQuantizedVectorsFormat + rescoring); here the re-scoring is exact and
// a per-(query, shard) certificate proves that no row outside the re-scored set can enter the top k,
// so the result is bit-identical to the fp32 streaming scan (osk_kernels.hip scan_f32) — the same
// docs, the same score bits, the same tie order.
//
//   sq8_quantize  fp32 rows (or queries) → int8 (per-row symmetric scale s = max|x|/127) + the
//                 per-row bound terms {s, s·|q|, |x − s·q|, |x|²}, computed in double, rounded up.
//   sq8_scan      streams the int8 copy (¼ of the fp32 bytes): Σ q8_row·q8_query in exact int32
//                 (v_dot4_i32_i8), then for every row an interval [lo, hi] that provably contains the
//                 score the fp32 streaming scan computes for that row (quantisation error bound +
//                 the fp32 rounding bound of the device summation order).  Per tile it keeps the
//                 kKQ rows with the highest upper bound (keys) and their lower bounds.
//   sq8_settle    per (query, slice of 16 tiles): L = k-th best lower bound of the listed rows of
//                 its group of slices; every listed row whose upper bound reaches L is re-scored with the streaming
//                 scan's exact arithmetic; a tile whose list is full and whose last upper bound
//                 reaches L (a dropped row might qualify) is re-scanned exactly, every row.
//
// Soundness: L is the k-th best lower bound among listed rows of a group of slices
// of one shard.  Those k rows have ub ≥ lb ≥ L, so each is re-scored (or lies in an exactly
// re-scanned tile) and scores ≥ L: the shard's k-th exact score T ≥ L.  A row that is neither
// re-scored nor in an exact tile has score ≤ ub < L ≤ T, so it cannot enter the top k; strictness
// (ub < L) makes doc-order ties irrelevant.
#include <hip/hip_ext.h>

#include "osk_device.h"
#include "osk_internal.h"
#include "osk_wave.h"

namespace osk {

// ------------------------------------------------------------------------------------------------
// quantisation (one wave per row).  mode 0 (segment rows): aux = {s, s·|q|, |x − s·q|, |x|²};
// mode 1 (queries): aux = {s, |b − s·q|, s·|q| + |b − s·q|, |b|²}.  |·| are real (double) norms
// rounded up; |x|² is rounded to nearest (the kernels add slack for it).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void sq8_quantize(const float4* __restrict__ X, int64_t n, int units,
                                                       int pitch, int units8, uint32_t* __restrict__ out8,
                                                       float4* __restrict__ aux, int mode) {
    const int lane = threadIdx.x & 63;
    const int64_t wave_global = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) >> 6;
    const int dw = units8 * 4;   // int8 dwords per row (≥ units: one dword per fp32 float4)
    for (int64_t r = wave_global; r < n; r += n_waves) {
        const float4* xr = X + r * pitch;
        float m = 0.0f;
        for (int f = lane; f < units; f += 64) {
            const float4 x = xr[f];
            m = fmaxf(m, fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w))));
        }
        for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
        const float s = m / 127.0f;
        long long sq = 0;
        double se = 0.0, sx = 0.0;
        for (int d = lane; d < dw; d += 64) {
            uint32_t packed = 0u;
            if (d < units) {
                const float4 x = xr[d];
                const float xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    int qi = 0;
                    if (s > 0.0f) qi = (int)fminf(fmaxf(rintf(xs[e] / s), -127.0f), 127.0f);
                    packed |= ((uint32_t)qi & 0xFFu) << (8 * e);
                    sq += (long long)(qi * qi);
                    const double rr = (double)xs[e] - (double)s * (double)qi;   // exact in double
                    se += rr * rr;
                    sx += (double)xs[e] * (double)xs[e];
                }
            }
            out8[r * dw + d] = packed;
        }
        for (int o = 32; o >= 1; o >>= 1) {
            sq += __shfl_xor(sq, o);
            se += __shfl_xor(se, o);
            sx += __shfl_xor(sx, o);
        }
        if (lane == 0) {
            const double A = (double)s * sqrt((double)sq) * (1.0 + 1e-12);
            const double B = sqrt(se) * (1.0 + 1e-12);
            aux[r] = mode == 0 ? make_float4(s, f32_round_up(A), f32_round_up(B), (float)sx)
                               : make_float4(s, f32_round_up(B), f32_round_up((A + B) * (1.0 + 1e-12)), (float)sx);
        }
    }
}

hipError_t launch_sq8_quantize(const float4* x, int64_t n, int units, int pitch, int units8, void* out8,
                               float4* aux, int mode, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int64_t blocks = (n + 3) / 4;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(sq8_quantize, dim3((unsigned)blocks), dim3(kBlock), 0, s, x, n, units, pitch, units8,
                       static_cast<uint32_t*>(out8), aux, mode);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// fused query preparation of the prefilter path (one wave per query, one launch):
//   * the padded fp32 query (UP float4, zeros past dim; zero rows past nq) for the re-score and the
//     exact fallback;
//   * |q|² in the device lane order (identical bits to row_norms_f32 / scan_f32's in-kernel norm);
//   * the int8 quantisation (s = max|b|/127) and its bound terms qc[r];
//     (an int16 query — 256× smaller query error — was measured: 4.4× fewer re-scored rows but a
//     slower scan, its extra sdot4 work is not free at the HBM ceiling; so int8 it is)
//   * flags[r] = 0.
// ------------------------------------------------------------------------------------------------
//   Q6 (single queries of the 6-bit tier, osk_sq6.hip): also its second quantisation of the query, to
//   [-119, 119] (s6 = max|b|/119), split into signed nibbles b = 16·bh + bl and written in sq6_scan's
//   layout (64·C dwords per query) with its bound terms, and the query's floor buckets zeroed.
template <int L, int V, bool Q6>
__global__ __launch_bounds__(kBlock) void sq8_prep(const float* __restrict__ src, int dim, int nq, int nq_pad,
                                                   int UP, int units8, float4* __restrict__ qpad,
                                                   float* __restrict__ qnorm, uint32_t* __restrict__ q8,
                                                   float4* __restrict__ qc, int* __restrict__ flags, Sq6Prep q6) {
    // one workgroup per query: every element is loaded once, by one thread, and the reductions are
    // block-wide (a single wave per query walks 768 floats three times: ~8 µs of latency)
    __shared__ float s_m[4];
    __shared__ long long s_a[2][4];
    __shared__ double s_e[2][4], s_x[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform: scalar loop control
    const int64_t r = blockIdx.x;
    const bool real = r < nq;
    const float* b = src + r * (int64_t)dim;
    auto val = [&](int c) { return (real && c < dim) ? b[c] : 0.0f; };
    const int dw = units8 * 4;   // int8 dwords (4 dims each); dw ≥ UP·… covers every real dim
    // this thread's dwords: d = tid, tid + 256, … (4 dims each; the padded fp32 copy uses the same
    // float4 units where d < UP)
    constexpr int kPer = 4;      // dw ≤ 1024 (OSK_MAX_DIM 4096)
    float4 x[kPer];
    float m = 0.0f;
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        const int d = u * kBlock + tid;
        x[u] = make_float4(val(4 * d), val(4 * d + 1), val(4 * d + 2), val(4 * d + 3));
        if (d < UP) qpad[r * UP + d] = x[u];
        m = fmaxf(m, fmaxf(fmaxf(fabsf(x[u].x), fabsf(x[u].y)), fmaxf(fabsf(x[u].z), fabsf(x[u].w))));
    }
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (lane == 0) s_m[wave] = m;
    if constexpr (Q6)
        for (int i = tid; i < q6.floor_n; i += kBlock) q6.floor[r * q6.floor_n + i] = 0u;
    // device-order |q|² (wave 0): lane t of every L-lane group computes the same partial
    if (wave == 0) {
        const int t = lane & (L - 1);
        float ax = 0.f, ay = 0.f, az = 0.f, aw = 0.f;
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const int f = t + j * L;
            const float x0 = val(4 * f), x1 = val(4 * f + 1), x2 = val(4 * f + 2), x3 = val(4 * f + 3);
            ax = fmaf(x0, x0, ax); ay = fmaf(x1, x1, ay); az = fmaf(x2, x2, az); aw = fmaf(x3, x3, aw);
        }
        float sn = (ax + ay) + (az + aw);
        sn = lane_sum<L>(sn);
        if (lane == 0) qnorm[r] = sn;
    }
    __syncthreads();
    m = fmaxf(fmaxf(s_m[0], s_m[1]), fmaxf(s_m[2], s_m[3]));
    const float s8 = m / 127.0f, s6 = m / 119.0f;
    long long a8 = 0, a6 = 0;
    double e8 = 0.0, e6 = 0.0, sx = 0.0;
    __shared__ uint32_t s_qb[Q6 ? kPer * kBlock : 1];   // Q6: the [-119, 119] codes of every dim, then split
    uint32_t* p0 = q8 + r * dw;
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        const int d = u * kBlock + tid;
        if (!Q6 && d >= dw) break;
        const float xs[4] = {x[u].x, x[u].y, x[u].z, x[u].w};
        uint32_t w0 = 0u, w6 = 0u;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int qi = s8 > 0.0f ? (int)fminf(fmaxf(rintf(xs[e] / s8), -127.0f), 127.0f) : 0;
            w0 |= ((uint32_t)qi & 0xFFu) << (8 * e);
            a8 += (long long)(qi * qi);
            const double r8 = (double)xs[e] - (double)s8 * (double)qi;   // exact in double
            e8 += r8 * r8;
            sx += (double)xs[e] * (double)xs[e];
            if constexpr (Q6) {
                const int q6i = s6 > 0.0f ? (int)fminf(fmaxf(rintf(xs[e] / s6), -119.0f), 119.0f) : 0;
                w6 |= ((uint32_t)q6i & 0xFFu) << (8 * e);
                a6 += (long long)(q6i * q6i);
                const double r6 = (double)xs[e] - (double)s6 * (double)q6i;
                e6 += r6 * r6;
            }
        }
        if (d < dw) p0[d] = w0;
        if constexpr (Q6) s_qb[d] = w6;   // (zero past dim)
    }
    if constexpr (Q6) {
        __syncthreads();
        // dword w = hc·8 + m: m < 4 bh, m ≥ 4 bl of dims 32hc + 8(m & 3) + n in nibble n
        uint32_t* p6 = q6.q6 + r * 64 * q6.C;
        for (int w = tid; w < 64 * q6.C; w += kBlock) {
            const int hc = w >> 3, mm = w & 3;
            const bool low = (w & 4) != 0;
            const uint32_t d0 = s_qb[8 * hc + 2 * mm], d1 = s_qb[8 * hc + 2 * mm + 1];
            uint32_t o = 0u;
#pragma unroll
            for (int n = 0; n < 8; ++n) {
                const int qb = (int)(int8_t)((n < 4 ? d0 >> (8 * n) : d1 >> (8 * (n - 4))) & 0xFFu);
                const int bl = ((qb + 8) & 15) - 8, bh = (qb - bl) >> 4;
                o |= ((uint32_t)(low ? bl : bh) & 15u) << (4 * n);
            }
            p6[w] = o;
        }
    }
    for (int o = 32; o >= 1; o >>= 1) {
        a8 += __shfl_xor(a8, o);
        e8 += __shfl_xor(e8, o);
        sx += __shfl_xor(sx, o);
        if constexpr (Q6) {
            a6 += __shfl_xor(a6, o);
            e6 += __shfl_xor(e6, o);
        }
    }
    if (lane == 0) {
        s_a[0][wave] = a8;
        s_e[0][wave] = e8;
        s_a[1][wave] = a6;
        s_e[1][wave] = e6;
        s_x[wave] = sx;
    }
    __syncthreads();
    if (tid == 0) {
        sx = s_x[0] + s_x[1] + s_x[2] + s_x[3];
        auto terms = [&](int i, float sc) {
            const long long a = s_a[i][0] + s_a[i][1] + s_a[i][2] + s_a[i][3];
            const double e = s_e[i][0] + s_e[i][1] + s_e[i][2] + s_e[i][3];
            const double A = (double)sc * sqrt((double)a) * (1.0 + 1e-12), B = sqrt(e) * (1.0 + 1e-12);
            return make_float4(sc, f32_round_up(B), f32_round_up((A + B) * (1.0 + 1e-12)), (float)sx);
        };
        qc[r] = terms(0, s8);
        if constexpr (Q6) q6.qc6[r] = terms(1, s6);
        if (real) flags[r] = 0;
    }
}

using PrepFn = void (*)(const float*, int, int, int, int, int, float4*, float*, uint32_t*, float4*, int*, Sq6Prep);
#define OSK_PREP_ROW(Q6)                                                                                       \
    {sq8_prep<4, 2, Q6>,   sq8_prep<8, 2, Q6>,  sq8_prep<8, 4, Q6>,  sq8_prep<16, 4, Q6>, sq8_prep<16, 8, Q6>, \
     sq8_prep<16, 12, Q6>, sq8_prep<32, 8, Q6>, sq8_prep<64, 8, Q6>, sq8_prep<64, 16, Q6>}
static const PrepFn kPrep[2][9] = {OSK_PREP_ROW(false), OSK_PREP_ROW(true)};

hipError_t launch_sq8_prep(int cfg, const float* src, int dim, int nq, int nq_pad, int UP, int units8, float4* qpad,
                           float* qnorm, void* q8, float4* qc, int* flags, hipStream_t s, const Sq6Prep& q6) {
    if (q6.C < 0 || q6.C > 8) return hipErrorInvalidValue;
    hipLaunchKernelGGL(kPrep[q6.C > 0][cfg], dim3(nq_pad), dim3(kBlock), 0, s, src, dim, nq, nq_pad, UP, units8, qpad,
                       qnorm, static_cast<uint32_t*>(q8), qc, flags, q6);
    return hipGetLastError();
}

// Reduce-scatter of NQ per-query partial dots over the L lanes of a row: H = min(log2 NQ, log2 L)
// halving stages (lane keeps the half of its queries selected by one lane bit and adds the partner's
// copy of them), then butterflies over the remaining lane bits.  Lane t ends with the full sums of
// queries rs_base(t) + [0, P), P = NQ >> H, replicated over the butterfly bits.  Exact: int32 sums.
constexpr int ilog2c(int x) { return x <= 1 ? 0 : 1 + ilog2c(x >> 1); }
template <int L, int NQ>
struct RsShape {
    static constexpr int H = ilog2c(NQ) < ilog2c(L) ? ilog2c(NQ) : ilog2c(L);
    static constexpr int P = NQ >> H;
    static constexpr int REP = L >> H;   // lanes holding the same (row, query) sums
};
template <int L, int NQ>
__device__ __forceinline__ void rs_reduce(int (&acc)[NQ], int t) {
    constexpr int H = RsShape<L, NQ>::H, P = RsShape<L, NQ>::P;
#pragma unroll
    for (int i = 0; i < H; ++i) {
        const int h = NQ >> (i + 1), msk = L >> (i + 1);
        const bool up = (t & msk) != 0;
#pragma unroll
        for (int j = 0; j < h; ++j) {
            // both values loaded first: a select between two elements' addresses would push
            // acc[] to scratch
            const int lo_v = acc[j], hi_v = acc[h + j];
            const int keep = up ? hi_v : lo_v;
            const int send = up ? lo_v : hi_v;
            acc[j] = keep + __shfl_xor(send, msk);
        }
    }
#pragma unroll
    for (int m = L >> (H + 1); m >= 1; m >>= 1)
#pragma unroll
        for (int q = 0; q < P; ++q) acc[q] += __shfl_xor(acc[q], m);
}
template <int L, int NQ>
__device__ __forceinline__ int rs_base(int t) {
    int b = 0;
#pragma unroll
    for (int i = 0; i < RsShape<L, NQ>::H; ++i) b += (t & (L >> (i + 1))) ? (NQ >> (i + 1)) : 0;
    return b;
}

// ------------------------------------------------------------------------------------------------
// prefilter scan: a row is L lanes × V 16-byte int8 units; U row groups per wave-iteration are
// loaded before any is reduced (≈ U·V·1 KiB in flight per wave).  NQ > 1: the per-query partial
// dots are reduce-scattered (rs_reduce) so each lane finishes the bound and quick test of P
// (row, query) pairs instead of all NQ.
// ------------------------------------------------------------------------------------------------
// MODE: kScanRows (row-range tiles; a filter is walked 64-row window by window: its accepted rows
// compacted to the front of the wave, one load round trip per non-empty window), kScanGather (filtered:
// the grid runs over gather tiles of the compacted accepted ordinals, osk_filter.hip — measured faster
// at every selectivity: C5 1 % 70 → 30 µs, 10 % 227 → 155 µs, 50 % 700 → 663 µs per scan,
// profiles/r02c/c5f_gather_ab.jsonl; a cross-window queue instance of the window walk was retired).
constexpr int kScanRows = 0, kScanGather = 2;

// A gather tile's entry range and its scan wave's share: tile j of nj over cnt accepted ordinals, split
// in 4 contiguous quarters.  A sparse filter uses fewer tiles of the segment — at most one per
// min_entries accepted rows (short wave lists fill with most of their rows, so the settle would
// re-score most rows) — and the others stay empty.  The settle re-derives the same ranges.
__device__ __forceinline__ void gather_wave_range(int64_t cnt, int j, int nj, int min_entries, int wave, int64_t& b,
                                                  int64_t& e) {
    if (min_entries > 0) nj = (int)max<int64_t>(1, min<int64_t>(nj, (cnt + min_entries - 1) / min_entries));
    if (j >= nj) {
        b = e = 0;
        return;
    }
    const int64_t e0 = cnt * j / nj, e1 = cnt * (j + 1) / nj;
    const int64_t pw = (e1 - e0 + 3) / 4;
    b = min(e0 + wave * pw, e1);
    e = min(b + pw, e1);
}

template <int L, int V, int NQ, int U, int MODE = kScanRows>
__global__ __launch_bounds__(kBlock, NQ == 1 && V <= 3 ? (U > 4 ? 3 : 4) : 1) void sq8_scan(Sq8Params p) {   // ≤ 128 VGPRs: 4 waves/SIMD (U = 8: 3)
    constexpr int R = 64 / L;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform: scalar loop control
    const int t = lane & (L - 1), g = lane / L;
    TileDev tile;
    int4 gt = make_int4(0, 0, 0, 1);
    if constexpr (MODE == kScanGather) {
        gt = p.gtiles[blockIdx.x];
        tile = TileDev{gt.x, gt.y, 0, 0};
    } else {
        tile = p.tiles[blockIdx.x];
    }
    const SegDev seg = p.segs[tile.seg];
    const int4* __restrict__ X = p.rows8[tile.seg];
    const float4* __restrict__ AX = p.aux[tile.seg];
    const uint32_t vbase = (uint32_t)p.seg_vrow[tile.seg];
    const int u8 = p.units8, sim = p.sim;

    // NQ == 1: the query fragment and the wave's list in VGPRs.  NQ > 1: all queries in LDS
    // ([NQ][units8] int4) and every wave's per-query lists in LDS ([4][NQ][kKQ] keys + lower bounds),
    // so that no per-query array needs a dynamic register index.
    extern __shared__ __attribute__((aligned(16))) int4 sq[];
    uint64_t* s_lk = reinterpret_cast<uint64_t*>(sq + (NQ > 1 ? NQ * u8 : 0));
    uint32_t* s_lp = reinterpret_cast<uint32_t*>(s_lk + 4 * NQ * kKQ);
    int4 qf[1][NQ == 1 ? V : 1];
    if constexpr (NQ == 1) {
#pragma unroll
        for (int j = 0; j < V; ++j) {
            // clamped index + mask (a select between the global pointer and a zero local would live
            // in scratch)
            const int f = t + j * L;
            const int fc = f < u8 ? f : 0;
            const int msk = f < u8 ? -1 : 0;
            const int4 v = p.q8[fc];
            qf[0][j] = make_int4(v.x & msk, v.y & msk, v.z & msk, v.w & msk);
        }
    } else {
        for (int i = tid; i < NQ * u8; i += kBlock) sq[i] = p.q8[i];
        for (int i = tid; i < 4 * NQ * kKQ; i += kBlock) {
            s_lk[i] = 0ull;
            s_lp[i] = 0u;
        }
        __syncthreads();
    }
    const float4 qc0 = p.qc[0];
    const float qnd0 = sim == SIM_COSINE ? p.qn_dev[0] : 0.0f;
    const float sqn0 = sqrtf(qnd0);

    const int64_t rows = tile.row_end - tile.row_begin;
    const int64_t per_wave = ((rows + 4 * R - 1) / (4 * R)) * R;
    const int64_t wb = tile.row_begin + wave * per_wave;
    const int64_t we = min(wb + per_wave, tile.row_end);
    const uint64_t* abits = p.accept ? p.accept[tile.seg] : nullptr;

    uint64_t lk0 = 0ull, thr0 = 0ull;   // NQ == 1: the wave's list
    uint32_t lp0 = 0u;
    float tq0 = sq8_quick(sim, 0ull, 0.0f, 0.0f);
    // NQ > 1: the P queries this lane finishes after the reduce-scatter, and their thresholds
    constexpr int P = RsShape<L, NQ>::P;
    const int qb = rs_base<L, NQ>(t);
    const bool rep = (t & (RsShape<L, NQ>::REP - 1)) == 0;
    float tql[P];
    float4 qcl[P];
#pragma unroll
    for (int j = 0; j < P; ++j) {
        tql[j] = sq8_quick(sim, 0ull, 0.0f, 0.0f);
        qcl[j] = p.qc[qb + j];   // per-lane load (a select chain over qc[] becomes a scratch index)
    }
    uint32_t nvis = 0;

    // filt = false: rows base + u·R + g (< we); filt = true: the compacted accepted rows of the
    // 64-row window at base (lanes' positions in `pos`), entries i0 + u·R + g of n
    auto process = [&](int64_t base, bool filt, int i0, int n, int pos) {
        int64_t row[U];
        bool valid[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (filt) {
                const int idx = i0 + u * R + g;
                row[u] = base + __shfl(pos, idx < 64 ? idx : 0);
                valid[u] = idx < n;
            } else {
                row[u] = base + u * R + g;
                valid[u] = row[u] < we;
            }
        }
        const bool known = filt;
        // every load is unconditional, on a clamped in-range row, and masked after: a load under a
        // per-lane condition made the compiler wait for each row group before issuing the next
        // (lane 0's entry of a compacted window is always a real row; else the wave's first row)
        const int64_t safe = filt ? base + __shfl(pos, 0) : wb;
        int4 xv[U][V];
        float4 ax[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (valid[u] && abits && !known) {
                const int32_t doc = seg.ord_to_doc ? seg.ord_to_doc[row[u]] : (int32_t)row[u];
                valid[u] = (abits[doc >> 6] >> (doc & 63)) & 1ull;
            }
            const int64_t rc = valid[u] ? row[u] : safe;
            const int4* xr = X + rc * u8;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const int f = t + j * L;
                const int4 x = load_i4_nt(xr + (f < u8 ? f : 0));
                const int m = (valid[u] && f < u8) ? -1 : 0;
                xv[u][j] = make_int4(x.x & m, x.y & m, x.z & m, x.w & m);
            }
            const float4 a = AX[rc];
            ax[u] = valid[u] ? a : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        if constexpr (NQ == 1) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                nvis += __popcll(__ballot(t == 0 && valid[u]));
                const float sx = sim == SIM_COSINE ? __builtin_amdgcn_sqrtf(ax[u].w) : 0.0f;   // (1 ulp ≪ the quick test's slack)
                int acc = 0;
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    acc = __builtin_amdgcn_sdot4(xv[u][j].x, qf[0][j].x, acc, false);
                    acc = __builtin_amdgcn_sdot4(xv[u][j].y, qf[0][j].y, acc, false);
                    acc = __builtin_amdgcn_sdot4(xv[u][j].z, qf[0][j].z, acc, false);
                    acc = __builtin_amdgcn_sdot4(xv[u][j].w, qf[0][j].w, acc, false);
                }
                acc = lane_sum<L>(acc);
                float lo, hi;
                sq8_bounds(sim, (float)acc, ax[u], qc0, p.gam, p.g2, lo, hi);
                const bool pass = valid[u] && sq8_pass(sim, lo, hi, tq0, sx);
                if (__ballot(pass && t == 0)) {   // wave-uniform: rare once the list has filled
                    float xnd = 0.0f;
                    if (sim == SIM_COSINE && pass) xnd = seg.xnorm_f[row[u]];
                    const float ub = sim == SIM_EUCLIDEAN ? score_f32_l2(lo) : score_f32(sim, hi, qnd0, xnd);
                    const float lb = sim == SIM_EUCLIDEAN ? score_f32_l2(hi) : score_f32(sim, lo, qnd0, xnd);
                    const uint64_t key = pass ? make_key(ub, vbase + (uint32_t)row[u]) : 0ull;
                    wave_offer2(key, float_to_sortable(lb), pass && t == 0, lk0, lp0, thr0, lane, kKQ);
                    tq0 = sq8_quick(sim, thr0, sqn0, p.cos_slack);
                }
            }
        } else {
            // every query's fragment is read from LDS once per U row groups (registers hold rows)
            int acc[U][NQ];
#pragma unroll
            for (int b = 0; b < NQ; ++b) {
                int4 qv[V];
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    const int f = t + j * L;
                    qv[j] = sq[b * u8 + (f < u8 ? f : 0)];
                    if (f >= u8) qv[j] = make_int4(0, 0, 0, 0);
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    int a = 0;
#pragma unroll
                    for (int j = 0; j < V; ++j) {
                        a = __builtin_amdgcn_sdot4(xv[u][j].x, qv[j].x, a, false);
                        a = __builtin_amdgcn_sdot4(xv[u][j].y, qv[j].y, a, false);
                        a = __builtin_amdgcn_sdot4(xv[u][j].z, qv[j].z, a, false);
                        a = __builtin_amdgcn_sdot4(xv[u][j].w, qv[j].w, a, false);
                    }
                    acc[u][b] = a;
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                nvis += __popcll(__ballot(t == 0 && valid[u]));
                const float sx = sim == SIM_COSINE ? __builtin_amdgcn_sqrtf(ax[u].w) : 0.0f;   // (1 ulp ≪ the quick test's slack)
                rs_reduce<L, NQ>(acc[u], t);
                bool pass[P];
                float lo[P], hi[P];
                bool anyp = false;
#pragma unroll
                for (int j = 0; j < P; ++j) {
                    sq8_bounds(sim, (float)acc[u][j], ax[u], qcl[j], p.gam, p.g2, lo[j], hi[j]);
                    pass[j] = valid[u] && rep && sq8_pass(sim, lo[j], hi[j], tql[j], sx);
                    anyp |= pass[j];
                }
                if (__ballot(anyp)) {   // wave-uniform: rare once the lists have filled
                    float xnd = 0.0f;
                    if (sim == SIM_COSINE && anyp) xnd = seg.xnorm_f[row[u]];
                    uint32_t qm = 0u;   // queries with a passing lane (wave-uniform)
#pragma unroll
                    for (int j = 0; j < P; ++j) qm |= pass[j] ? (1u << (qb + j)) : 0u;
                    uint32_t wq = 0u;
#pragma unroll
                    for (int b = 0; b < NQ; ++b) wq |= __ballot((qm >> b) & 1u) ? (1u << b) : 0u;
                    while (wq) {
                        const int b = __builtin_ctz(wq);
                        wq &= wq - 1u;
                        // the wave's list of query b: LDS → lanes 0..kKQ-1, insert, back to LDS
                        const int o0 = (wave * NQ + b) * kKQ;
                        uint64_t lkb = lane < kKQ ? s_lk[o0 + lane] : 0ull;
                        uint32_t lpb = lane < kKQ ? s_lp[o0 + lane] : 0u;
                        uint64_t thrb = readlane64(lkb, kKQ - 1);
                        const float qnb = sim == SIM_COSINE ? p.qn_dev[b] : 0.0f;
#pragma unroll
                        for (int j = 0; j < P; ++j) {
                            const bool o = pass[j] && (qb + j == b);
                            const float ub = sim == SIM_EUCLIDEAN ? score_f32_l2(lo[j]) : score_f32(sim, hi[j], qnb, xnd);
                            const float lb = sim == SIM_EUCLIDEAN ? score_f32_l2(hi[j]) : score_f32(sim, lo[j], qnb, xnd);
                            const uint64_t key = o ? make_key(ub, vbase + (uint32_t)row[u]) : 0ull;
                            wave_offer2(key, float_to_sortable(lb), o, lkb, lpb, thrb, lane, kKQ);
                        }
                        if (lane < kKQ) {
                            s_lk[o0 + lane] = lkb;
                            s_lp[o0 + lane] = lpb;
                        }
                        const float nt = sq8_quick(sim, thrb, sqrtf(qnb), p.cos_slack);
#pragma unroll
                        for (int jj = 0; jj < P; ++jj) tql[jj] = (qb + jj == b) ? nt : tql[jj];
                    }
                }
            }
        }
    };

    if constexpr (MODE == kScanGather) {
        // filter pushdown by compaction: this wave's quarter of the gather tile's accepted ordinals,
        // 64 at a time (one coalesced index load, then the rows), any segment layout (dense or sparse)
        // (counts and ordinals are clamped to the segment: a corrupt list can never address outside it)
        int64_t eb, ee;
        gather_wave_range(min<int64_t>(p.scnt[tile.seg], seg.n_rows), gt.z, gt.w, p.gather_min, wave, eb, ee);
        const uint32_t* __restrict__ C = p.comp + vbase;
        for (int64_t e0 = eb; e0 < ee; e0 += 64) {
            const int n = (int)min<int64_t>(64, ee - e0);
            const int pos = lane < n ? (int)min<int64_t>(C[e0 + lane], seg.n_rows - 1) : 0;
            for (int i0 = 0; i0 < n; i0 += R * U) process(0, true, i0, n, pos);
        }
    } else if (abits && !seg.ord_to_doc) {
        // filter pushdown: accepted rows of 64 compacted to the front of the wave (see walk_rows)
        for (int64_t w0 = wb; w0 < we; w0 += 64) {
            const int64_t word = w0 >> 6;
            const int sh = (int)(w0 & 63);
            uint64_t m = abits[word] >> sh;
            if (sh && (word + 1) * 64 < we) m |= abits[word + 1] << (64 - sh);
            if (we - w0 < 64) m &= (1ull << (we - w0)) - 1ull;
            const int n = __popcll(m);
            if (n == 0) continue;
            const bool bit = (m >> lane) & 1ull;
            const int below = __popcll(m & ((1ull << lane) - 1ull));
            const int dst = bit ? below : n + (lane - below);
            const int pos = __builtin_amdgcn_ds_permute(dst << 2, lane);
            for (int i0 = 0; i0 < n; i0 += R * U) process(w0, true, i0, n, pos);
        }
    } else {
        for (int64_t r0 = wb; r0 < we; r0 += R * U) process(r0, false, 0, 0, 0);
    }

    // one list per wave (its own row range of the tile): finer lists overflow the certificate less
    // often than one folded list per tile, and need no LDS fold.  With it, the list's best lower
    // bound (the settle's threshold is selected among these, one distinct row per list).
    for (int b = 0; b < NQ; ++b) {
        uint64_t lkb = lk0;
        uint32_t lpb = lp0;
        if constexpr (NQ > 1) {
            lkb = lane < kKQ ? s_lk[(wave * NQ + b) * kKQ + lane] : 0ull;
            lpb = lane < kKQ ? s_lp[(wave * NQ + b) * kKQ + lane] : 0u;
        }
        uint32_t m = (lane < kKQ && lkb) ? lpb : 0u;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
        if (b < p.q_count) {
            const size_t l = (size_t)(p.q0 + b) * p.n_lists + blockIdx.x * 4 + wave;
            if (lane < kKQ) {
                p.cand[l * kKQ + lane] = lkb;
                p.cand_lb[l * kKQ + lane] = lpb;
            }
            if (lane == 0) p.list_lbmax[l] = m;
        }
    }
    if (p.visited && p.q0 == 0) add_visited_wg(&p.visited[tile.seg], (uint32_t)nvis);   // (after the lists)
}

// int8 lane configs by 16-byte units per row: {L, V} (the int32 sums are exact: any order)
static int sq8_cfg(int u8) {
    return u8 <= 4 ? 0 : u8 <= 8 ? 1 : u8 <= 16 ? 2 : u8 <= 32 ? 3 : u8 <= 48 ? 4 : u8 <= 64 ? 5 : u8 <= 128 ? 6 : 7;
}
int sq8_lanes(int u8) {   // L of the scan's config (its rows per wave-iteration are 64 / L)
    static const int kL[8] = {4, 8, 16, 16, 16, 16, 32, 64};
    return kL[sq8_cfg(u8)];
}
using Sq8Fn = void (*)(Sq8Params);
#define OSK_SQ8_ROW(L, V) {sq8_scan<L, V, 1, 4>, sq8_scan<L, V, 2, 4>, sq8_scan<L, V, 4, 4>, sq8_scan<L, V, 8, 2>}
static const Sq8Fn kSq8[8][4] = {OSK_SQ8_ROW(4, 1),  OSK_SQ8_ROW(8, 1),  OSK_SQ8_ROW(16, 1), OSK_SQ8_ROW(16, 2),
                                 OSK_SQ8_ROW(16, 3), OSK_SQ8_ROW(16, 4), OSK_SQ8_ROW(32, 4), OSK_SQ8_ROW(64, 4)};
// filtered scans over the compacted accepted ordinals (gather tiles)
#define OSK_SQ8_GROW(L, V)                                                                          \
    {sq8_scan<L, V, 1, 4, kScanGather>, sq8_scan<L, V, 2, 4, kScanGather>, sq8_scan<L, V, 4, 4, kScanGather>, \
     sq8_scan<L, V, 8, 2, kScanGather>}
static const Sq8Fn kSq8Gather[8][4] = {OSK_SQ8_GROW(4, 1),  OSK_SQ8_GROW(8, 1),  OSK_SQ8_GROW(16, 1),
                                       OSK_SQ8_GROW(16, 2), OSK_SQ8_GROW(16, 3), OSK_SQ8_GROW(16, 4),
                                       OSK_SQ8_GROW(32, 4), OSK_SQ8_GROW(64, 4)};

// single queries over ≤ 256-dim rows (V = 1) with twice the row groups in flight per wave (U = 8: 8 KiB per wave
// of rows, 3 waves per SIMD) — an A/B variant, off by default (sq8_scan_deep): at C2 b1 it was slower, 0.048 →
// 0.061 ms (profiles/r06/call11/cfg_small_d*.jsonl): the U = 4 scan's 5 waves per SIMD hide the latency better
static const Sq8Fn kSq8Deep[3] = {sq8_scan<4, 1, 1, 8>, sq8_scan<8, 1, 1, 8>, sq8_scan<16, 1, 1, 8>};

hipError_t launch_sq8_scan(int nq, const Sq8Params& p, hipStream_t s, hipEvent_t ev_start, hipEvent_t ev_stop) {
    const int slot = nq <= 1 ? 0 : nq <= 2 ? 1 : nq <= 4 ? 2 : 3;
    // NQ > 1: the queries and the 4 waves' per-query lists in LDS
    const size_t lds = slot == 0 ? 0 : (size_t)(1 << slot) * (p.units8 * 16 + 4 * kKQ * 12);
    const int c = sq8_cfg(p.units8);
    const auto fn = p.gtiles ? kSq8Gather[c][slot]
                    : (slot == 0 && c <= 2 && g_tuning.sq8_scan_deep) ? kSq8Deep[c]
                                                                      : kSq8[c][slot];
    if (ev_start || ev_stop)
        hipExtLaunchKernelGGL(fn, dim3(p.n_tiles), dim3(kBlock), lds, s, ev_start, ev_stop, 0, p);
    else
        hipLaunchKernelGGL(fn, dim3(p.n_tiles), dim3(kBlock), lds, s, p);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// prefilter scan on int8 MFMA: up to 16 queries per launch (batches of 2 and more).  The VALU scan's
// per-(row, query) int32 dot is v_dot4 + cross-lane reductions, so at 8 queries it is VALU-bound
// (2.1 TB/s).  Here a wave takes 16 rows at a time and one v_mfma_i32_16x16x64_i8 per 64 dims gives
// the 16 × 16 exact int32 dots: lane l loads 16 B of row (l & 15) per k-step (chunk l >> 4 of the
// 64-B slab) and reads the same chunk of query (l & 15) from LDS; the product pairs row byte j with
// query byte j of the same chunk, whatever the unit's internal k order (A and B share the layout).
// Lane l then holds dots of rows 4(l >> 4) + i (i = 0..3) × query l & 15 and runs the same bound,
// quick test and list insertion as sq8_scan (lists per (wave, query) in LDS).  Row split and list
// numbering are sq8_scan's with R = 16 rows per wave-iteration (the settle re-scans with scan_R = 16).
// Filter pushdown: accepted rows are compacted 64 at a time; any row can feed any MFMA row slot.
// ------------------------------------------------------------------------------------------------
// sq8_mfma's LDS-DMA ring: a group slot holds the group's 16 rows (row-major, exact width) then their
// 16 bound terms.  The rows take KS LDS-DMA instructions; a slot holds exactly 16·u8 units when the
// last instruction still has a lane of real data (u8 > 4(KS − 1)), else all KS·64 lanes land (clamped
// sources) — either way every instruction has an active lane, so each group is KS + 1 counted ops.
__host__ __device__ __forceinline__ int ring_rows_units(int u8, int ks) {
    return u8 > 4 * (ks - 1) ? 16 * u8 : ks * 64;
}

// A lane's 4 rows' bound terms {s, s·|q|, |x − s·q|, |x|²} as row pairs (rows 0/1, rows 2/3) per component,
// the layout packed fp32 math (v_pk_fma_f32) takes without register shuffles.
typedef float f32x2 __attribute__((ext_vector_type(2)));
struct AuxQ {
    f32x2 x[2], y[2], z[2], w[2];
    __device__ __forceinline__ float4 row(int i) const {
        const int h = i >> 1, j = i & 1;
        return make_float4(x[h][j], y[h][j], z[h][j], w[h][j]);
    }
    __device__ __forceinline__ void set(float4 a0, float4 a1, float4 a2, float4 a3) {
        x[0] = f32x2{a0.x, a1.x};
        y[0] = f32x2{a0.y, a1.y};
        z[0] = f32x2{a0.z, a1.z};
        w[0] = f32x2{a0.w, a1.w};
        x[1] = f32x2{a2.x, a3.x};
        y[1] = f32x2{a2.y, a3.y};
        z[1] = f32x2{a2.z, a3.z};
        w[1] = f32x2{a2.w, a3.w};
    }
};

// QB query blocks of 16 per launch (QB = 2: 32 queries, two MFMA chains sharing the row operand).
// RING (unfiltered launches, KS ≤ 4): rows are not loaded into VGPRs but streamed by LDS-DMA from the
// row-major int8 copy (exact width: no tiled copy, no padding) into a per-wave ring of NS
// 16-row groups, NS − 1 groups ahead of the one being scored, so a wave keeps several groups in
// flight without holding their registers (the register path holds one group: latency-bound at small
// dims, ≈2.8 TB/s loads-only at 96 dims).
// SIM is compile-time: with the similarity a runtime value every (row, query) pair paid the COSINE
// row-norm square root and a switch (≈ 50 VALU + 30 SALU per pair at 96 dims).
// NS: ring depth in 16-row groups per wave (0 = register loads), compile-time so that the per-group
// completion wait is one s_waitcnt of a constant count.
template <int KS, int QB, int NS, int SIM>
// KS = 2 ring instances are capped at 128 VGPRs: their LDS holds four workgroups per CU, and 4 waves per
// SIMD need ≤ 128 (C4 b32: 123 VGPRs 2.71 ms, 131 VGPRs 2.89 ms per 32 queries).  KS = 4 rings fit two.
__global__ __launch_bounds__(kBlock, QB == 1 || (NS == 2 && KS == 2) ? 4 : (NS ? 2 : 3)) void sq8_mfma(Sq8Params p) {
    constexpr bool RING = NS > 0;
    // insertions bounded one pair per lane (see the insertion loop) — not in the 4-workgroup KS = 2, 2-slot ring
    // instances capped at 128 VGPRs (nor KS = 16, QB = 1), where its extra live values spilled inside the loop
    // (the 4-slot ring instances, 2 workgroups per CU, take it)
    constexpr bool LANE_INS = !(RING && KS == 2 && QB == 2 && NS == 2) && !(KS == 16 && QB == 1);
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    constexpr int NQ = 16 * QB, R = 16, UQ = 4 * KS;   // UQ: 16-B units per query in LDS
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform: scalar loop control
    const int col = lane & 15, grp = lane >> 4;
    const TileDev tile = p.tiles[blockIdx.x];
    const SegDev seg = p.segs[tile.seg];
    const int4* __restrict__ XT = p.rows8t[tile.seg];   // tiled: [row / 16][KS][4 chunks][16 rows]
    const float4* __restrict__ AX = p.aux[tile.seg];
    const uint32_t vbase = (uint32_t)p.seg_vrow[tile.seg];
    const int u8 = p.units8;
    constexpr int sim = SIM;
    extern __shared__ __attribute__((aligned(16))) int4 sq[];   // [NQ][UQ] (zero past u8 / q_count)
    // RING: the ring overlays the query block (queries are copied into VGPRs first), lists follow both
    const int ring_rows = RING ? ring_rows_units(u8, KS) : 0;
    const int ring_slot = ring_rows + 16;
    const int lists_off = RING ? max(NQ * UQ, 4 * NS * ring_slot) : NQ * UQ;
    uint64_t* s_lk = reinterpret_cast<uint64_t*>(sq + lists_off);
    uint32_t* s_lp = reinterpret_cast<uint32_t*>(s_lk + 4 * NQ * kKQ);
    for (int i = tid; i < NQ * UQ; i += kBlock) {
        const int b = i / UQ, f = i - b * UQ;
        sq[i] = (b < p.q_count && f < u8) ? p.q8[b * u8 + f] : make_int4(0, 0, 0, 0);
    }
    for (int i = tid; i < 4 * NQ * kKQ; i += kBlock) {
        s_lk[i] = 0ull;
        s_lp[i] = 0u;
    }
    // this lane's queries: qb·16 + col
    bool qv[QB];
    float4 qc[QB];
    float qnd[QB], sqn[QB], tq[QB];
    uint64_t tkey[QB];
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
        const int qi = qb * 16 + col;
        qv[qb] = qi < p.q_count;
        qc[qb] = qv[qb] ? p.qc[qi] : make_float4(0.f, 0.f, 0.f, 0.f);
        qnd[qb] = (sim == SIM_COSINE && qv[qb]) ? p.qn_dev[qi] : 0.0f;
        sqn[qb] = sqrtf(qnd[qb]);
        // the pilot's floor key T of (query qi, this tile's shard): 0 = none (< k sampled rows)
        uint64_t t = 0ull;
        if (!p.pilot && p.thr_keys && qv[qb]) {
            const size_t o = (size_t)qi * p.n_shards + tile.shard;
            if (p.thr_counts[o] >= p.k) t = p.thr_keys[o * p.k + p.k - 1];
            // a floor of score 0 (DOT_PRODUCT / COSINE clamp every negative similarity to 0) would
            // drop rows that tie with it: sq8_quick's test is strict only above the clamp
            if (!(key_score(t) > 0.0f)) t = 0ull;
        }
        tkey[qb] = t;
        tq[qb] = sq8_quick(sim, t, sqn[qb], p.cos_slack);
    }
    // Quick test of DOT / COSINE / MIP as one fma chain per (row, query): hq = I·s_x·s_b + E with
    //   E = |x|_q·QY + |δ_x|·QZ + |x|²·QW + Q0, per-query coefficients rounded up from
    //   QY = (s_b|δ_b| + 2^-18·(s_b|q_b| + |δ_b|))(1 + 2^-18), QZ = (s_b|q_b| + |δ_b|)(1 + 2^-18),
    //   QW = γ(1 + 2^-18), Q0 = γ|b|²(1 + 2^-18).
    // hq ≥ the upper bound sq8_bound_side computes, whatever the rounding: E exceeds its error terms by
    // 2^-18 of themselves plus 2^-18·s_x|q_x|·(s_b|q_b| + |δ_b|) ≥ 2^-18·|I·s_x·s_b| (Cauchy–Schwarz on
    // the integer vectors), more than its 2^-20 slack and every float rounding of both computations
    // (< 2^-21 relative).  So a pair the precise bound would pass always passes here; the rare
    // insertions then evaluate sq8_bounds exactly as before.
    // per query block: the lane's query coefficients (broadcast to both halves of the packed row-pair math)
    float QY[QB], QZ[QB], Q0[QB];
    uint64_t qvm[QB];
    const float QW = __double2float_ru((double)p.gam * (1.0 + 0x1p-18));
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
        if constexpr (SIM == SIM_EUCLIDEAN) {
            // EUCLIDEAN: a lower bound of sq8_bounds' d² lower bound (before its ·(1 − g2)), with the
            // slack m = 2^-17 in place of its 2^-20 and |I·s_x·s_b| ≤ s_x|q_x|·(s_b|q_b| + |δ_b|):
            //   lq = |x|²(1 − m) + Q0 − 2·I·s_x·s_b − |x|_q·QY − |δ_x|·QZ,
            //   QY = (2 + 2m)·s_b|δ_b| + 2m·(s_b|q_b| + |δ_b|) ↑, QZ = (2 + 2m)(s_b|q_b| + |δ_b|) ↑,
            //   Q0 = |b|²(1 − m) ↓.
            // The extra 3·2^-20 of (|x|² + |b|² + 2|approx| + 2·eq) exceeds every rounding of both
            // computations, so lq·(1 − g2) never exceeds the precise side: a pair the precise test
            // passes (d² lower bound ≤ threshold) passes here.
            const double m = 0x1p-17;
            QY[qb] = __double2float_ru((2.0 + 2.0 * m) * (double)qc[qb].y + 2.0 * m * (double)qc[qb].z);
            QZ[qb] = __double2float_ru((2.0 + 2.0 * m) * (double)qc[qb].z);
            Q0[qb] = __double2float_rd((double)qc[qb].w * (1.0 - m));
        } else {
            const double r = 1.0 + 0x1p-18;
            QY[qb] = __double2float_ru(((double)qc[qb].y + 0x1p-18 * (double)qc[qb].z) * r);
            QZ[qb] = __double2float_ru((double)qc[qb].z * r);
            Q0[qb] = __double2float_ru((double)p.gam * (double)qc[qb].w * r);
        }
        qvm[qb] = __ballot(qv[qb]);
    }
    const float g2m = 1.0f - p.g2;   // sq8_bounds' EUCLIDEAN factor, the same float expression
#ifdef OSK_TESTING
    const int ablate = p.ablate;
#else
    constexpr int ablate = 0;   // A/B knobs exist only in libosknn_testing.so
#endif
    const bool pilot = p.pilot != 0;
    bool sampled = false;   // pilot: this wave's first group is done

    const int64_t rows = tile.row_end - tile.row_begin;
    const int64_t per_wave = ((rows + 4 * R - 1) / (4 * R)) * R;
    const int64_t wb = tile.row_begin + wave * per_wave;
    const int64_t we = min(wb + per_wave, tile.row_end);
    const uint64_t* abits = p.accept ? p.accept[tile.seg] : nullptr;
    uint32_t nvis = 0;
    __syncthreads();

    auto load_group = [&](int64_t rowA, bool vA, i32x4 (&a)[KS]) {
        // row rowA's chunk grp of slab s: an aligned 16-row group reads 1 KiB contiguous per slab
        const int64_t ra = vA ? rowA : tile.row_begin;
        const int4* xr = XT + (ra >> 4) * (KS * 64) + grp * 16 + (ra & 15);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int4 v = vA ? load_i4_g(xr + s * 64, p.nt) : make_int4(0, 0, 0, 0);
            a[s] = i32x4{v.x, v.y, v.z, v.w};
        }
    };
    auto load_aux = [&](const int64_t (&ro)[4], const bool (&vo)[4], float4 (&ax)[4]) {
#pragma unroll
        for (int i = 0; i < 4; ++i)   // unconditional (clamped) loads: one wait for all four, not four
            ax[i] = load_f4_g(AX + (vo[i] ? ro[i] : (int64_t)tile.row_begin));
    };
    // RING (KS ≤ 4): the queries' B fragments live in VGPRs for the whole scan (≤ 32), not re-read
    // from LDS per group
    i32x4 bfr[RING ? KS : 1][QB];
    if constexpr (RING) {
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int qb = 0; qb < QB; ++qb) {
                const int4 bv = sq[(qb * 16 + col) * UQ + s * 4 + grp];
                bfr[s][qb] = i32x4{bv.x, bv.y, bv.z, bv.w};
            }
        __syncthreads();   // every wave holds its fragments before any ring write lands on the queries
    }
    auto process_loaded = [&](const i32x4 (&a)[KS], const AuxQ& aq, bool vA, const int64_t (&ro)[4],
                              const bool (&vo)[4]) {
        nvis += __popcll(__ballot(lane < 16 && vA));
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
                for (int qb = 0; qb < QB; ++qb) {
                    i32x4 b;
                    if constexpr (RING) {
                        b = bfr[s][qb];
                    } else {
                        const int4 bv = sq[(qb * 16 + col) * UQ + s * 4 + grp];
                        b = i32x4{bv.x, bv.y, bv.z, bv.w};
                    }
                    acc[qb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[s], b, acc[qb], 0, 0, 0);
                }
        }
        if (ablate & 1) {
            if (acc[0][0] + acc[0][1] + acc[0][2] + acc[0][3] == 0x7FFFFFFF && aq.x[0].x == 1.0f) nvis += 1;
            return;
        }
        uint64_t pm[QB][4];   // lanes whose (row i, query) pair passes the quick test (lane masks; rows
                              // past a partial group's end may be set: masked when folding, vo re-checked)
        uint32_t qm = 0u;     // queries with a passing lane (wave-uniform)
        // both bounds of a pair, for the rare list insertions and the pilot (the quick test reads one)
        auto bounds = [&](int qb, int i, float& lo, float& hi) {
            sq8_bounds(sim, (float)acc[qb][i], aq.row(i), qc[qb], p.gam, p.g2, lo, hi);
        };
        if constexpr (QB == 1) {
            // (one query block: the register-capped 4-workgroup instances keep the precise side)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float4 axi = aq.row(i);
                const float sx = SIM == SIM_COSINE ? __builtin_amdgcn_sqrtf(axi.w) : 0.0f;
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) {
                    const float side = sq8_bound_side(sim, (float)acc[qb][i], axi, qc[qb], p.gam, p.g2);
                    pm[qb][i] = __ballot(sq8_pass(sim, side, side, tq[qb], sx));
                }
            }
        } else {
            // packed over row pairs: 3 + 2 v_pk_fma/mul per (row pair, query block)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                f32x2 sx2 = {1.0f, 1.0f};
                if constexpr (SIM == SIM_COSINE)   // (v_sqrt: 1 ulp ≪ the 2^-16 quick-test slack)
                    sx2 = f32x2{__builtin_amdgcn_sqrtf(aq.w[h].x), __builtin_amdgcn_sqrtf(aq.w[h].y)};
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) {
                    const f32x2 I2 = {(float)acc[qb][2 * h], (float)acc[qb][2 * h + 1]};
                    if constexpr (SIM == SIM_EUCLIDEAN) {
                        const f32x2 E = __builtin_elementwise_fma(
                            aq.z[h], f32x2{-QZ[qb], -QZ[qb]},
                            __builtin_elementwise_fma(aq.y[h], f32x2{-QY[qb], -QY[qb]},
                                                      __builtin_elementwise_fma(aq.w[h], f32x2{1.0f - 0x1p-17f, 1.0f - 0x1p-17f},
                                                                                f32x2{Q0[qb], Q0[qb]})));
                        const f32x2 lq = __builtin_elementwise_fma(I2, aq.x[h] * f32x2{-2.0f * qc[qb].x, -2.0f * qc[qb].x}, E) *
                                         f32x2{g2m, g2m};
                        pm[qb][2 * h] = __ballot(!(lq.x > tq[qb]));
                        pm[qb][2 * h + 1] = __ballot(!(lq.y > tq[qb]));
                        continue;
                    }
                    const f32x2 E = __builtin_elementwise_fma(
                        aq.y[h], f32x2{QY[qb], QY[qb]},
                        __builtin_elementwise_fma(aq.z[h], f32x2{QZ[qb], QZ[qb]},
                                                  __builtin_elementwise_fma(aq.w[h], f32x2{QW, QW}, f32x2{Q0[qb], Q0[qb]})));
                    const f32x2 hq = __builtin_elementwise_fma(I2, aq.x[h] * f32x2{qc[qb].x, qc[qb].x}, E);
                    const f32x2 thr = SIM == SIM_COSINE ? sx2 * f32x2{tq[qb], tq[qb]} : f32x2{tq[qb], tq[qb]};
                    pm[qb][2 * h] = __ballot(!(hq.x < thr.x));
                    pm[qb][2 * h + 1] = __ballot(!(hq.y < thr.y));
                }
            }
        }
        if (!pilot) {
            // rows past a partial group's end hold stale slot data: mask them here, or every wave's
            // last group would run the insertion loop for every query (C2: +0.08 ms per launch)
            uint64_t vm[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) vm[i] = __ballot(vo[i]);
#pragma unroll
            for (int qb = 0; qb < QB; ++qb) {
                const uint64_t bl =
                    ((pm[qb][0] & vm[0]) | (pm[qb][1] & vm[1]) | (pm[qb][2] & vm[2]) | (pm[qb][3] & vm[3])) & qvm[qb];
                qm |= (uint32_t)((bl | (bl >> 16) | (bl >> 32) | (bl >> 48)) & 0xFFFFull) << (16 * qb);
            }
        }
        if (pilot) {   // the sampled rows' lower-bound keys (distinct: they carry the view row)
#pragma unroll
            for (int qb = 0; qb < QB; ++qb) {
                if (!qv[qb]) continue;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float xnd = 0.0f;
                    if (sim == SIM_COSINE && vo[i]) xnd = seg.xnorm_f[ro[i]];
                    float lo, hi;
                    bounds(qb, i, lo, hi);
                    const float lb = sim == SIM_EUCLIDEAN ? score_f32_l2(hi) : score_f32(sim, lo, qnd[qb], xnd);
                    s_lk[(qb * 16 + col) * 64 + wave * 16 + 4 * grp + i] =
                        vo[i] ? make_key(lb, vbase + (uint32_t)ro[i]) : 0ull;
                }
            }
            sampled = true;
            return;
        }
        while (qm) {   // rare once the lists have filled
            const int b = __builtin_ctz(qm);
            qm &= qm - 1u;
            const int bq = b >> 4, bc = b & 15;
            const int o0 = (wave * NQ + b) * kKQ;
            uint64_t lkb = lane < kKQ ? s_lk[o0 + lane] : 0ull;
            uint32_t lpb = lane < kKQ ? s_lp[o0 + lane] : 0u;
            uint64_t thrb = readlane64(lkb, kKQ - 1);
#pragma unroll
            for (int qb = 0; qb < QB; ++qb) {
                if (qb != bq) continue;   // (wave-uniform)
                if constexpr (LANE_INS) {
                    // one pair per lane: lane (col c < 4, grp g) takes row 4g + c of query b — its own row's
                    // terms, the dot from the lane (bc, g) — so the group's 16 candidate rows cost ONE precise
                    // bound per lane instead of four whole-wave bounds (b32 is VALU-bound, round 6:
                    // profiles/r06/sq8_mfma_b32/).  (Selects written out: an index into these arrays put them
                    // in scratch.)
                    const int c4 = col & 3, src = bc + 16 * grp;
                    const bool t1 = c4 == 1, t2 = c4 == 2, t3 = c4 == 3;
                    const int d0 = __shfl(acc[qb][0], src), d1 = __shfl(acc[qb][1], src);
                    const int d2 = __shfl(acc[qb][2], src), d3 = __shfl(acc[qb][3], src);
                    const int I = t3 ? d3 : t2 ? d2 : t1 ? d1 : d0;
                    const float4 r0f = aq.row(0), r1f = aq.row(1), r2f = aq.row(2), r3f = aq.row(3);
                    const float4 ax = make_float4(t3 ? r3f.x : t2 ? r2f.x : t1 ? r1f.x : r0f.x,
                                                  t3 ? r3f.y : t2 ? r2f.y : t1 ? r1f.y : r0f.y,
                                                  t3 ? r3f.z : t2 ? r2f.z : t1 ? r1f.z : r0f.z,
                                                  t3 ? r3f.w : t2 ? r2f.w : t1 ? r1f.w : r0f.w);
                    const int64_t ro0 = ro[0], ro1 = ro[1], ro2 = ro[2], ro3 = ro[3];
                    const int64_t rw = t3 ? ro3 : t2 ? ro2 : t1 ? ro1 : ro0;
                    const bool vo0 = vo[0], vo1 = vo[1], vo2 = vo[2], vo3 = vo[3];
                    const bool vw = t3 ? vo3 : t2 ? vo2 : t1 ? vo1 : vo0;
                    const uint64_t p0 = pm[qb][0], p1 = pm[qb][1], p2 = pm[qb][2], p3 = pm[qb][3];
                    const uint64_t pmw = t3 ? p3 : t2 ? p2 : t1 ? p1 : p0;
                    const float4 qcb = p.qc[b];   // (query b's terms: a wave-uniform load, no VGPRs)
                    const float qndb = sim == SIM_COSINE ? p.qn_dev[b] : 0.0f;
                    const bool o = col < 4 && ((pmw >> src) & 1ull) && vw;
                    float xnd = 0.0f;
                    if (sim == SIM_COSINE && o) xnd = seg.xnorm_f[rw];
                    float lo, hi;
                    sq8_bounds(sim, (float)I, ax, qcb, p.gam, p.g2, lo, hi);
                    const float ub = sim == SIM_EUCLIDEAN ? score_f32_l2(lo) : score_f32(sim, hi, qndb, xnd);
                    const float lb = sim == SIM_EUCLIDEAN ? score_f32_l2(hi) : score_f32(sim, lo, qndb, xnd);
                    const uint64_t key = o ? make_key(ub, vbase + (uint32_t)rw) : 0ull;
                    wave_offer2(key, float_to_sortable(lb), o, lkb, lpb, thrb, lane, kKQ);
                    if (col == bc) tq[qb] = sq8_quick(sim, thrb > tkey[qb] ? thrb : tkey[qb], sqn[qb], p.cos_slack);
                    continue;
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const bool o = ((pm[qb][i] >> lane) & 1ull) && vo[i] && col == bc;
                    float xnd = 0.0f;
                    if (sim == SIM_COSINE && o) xnd = seg.xnorm_f[ro[i]];
                    float lo, hi;
                    bounds(qb, i, lo, hi);
                    const float ub = sim == SIM_EUCLIDEAN ? score_f32_l2(lo) : score_f32(sim, hi, qnd[qb], xnd);
                    const float lb = sim == SIM_EUCLIDEAN ? score_f32_l2(hi) : score_f32(sim, lo, qnd[qb], xnd);
                    const uint64_t key = o ? make_key(ub, vbase + (uint32_t)ro[i]) : 0ull;
                    wave_offer2(key, float_to_sortable(lb), o, lkb, lpb, thrb, lane, kKQ);
                }
                if (col == bc) tq[qb] = sq8_quick(sim, thrb > tkey[qb] ? thrb : tkey[qb], sqn[qb], p.cos_slack);
            }
            if (lane < kKQ) {
                s_lk[o0 + lane] = lkb;
                s_lp[o0 + lane] = lpb;
            }
        }
    };
    auto process = [&](int64_t rowA, bool vA, const int64_t (&ro)[4], const bool (&vo)[4]) {
        i32x4 a[KS];
        load_group(rowA, vA, a);
        float4 ax[4];
        load_aux(ro, vo, ax);
        AuxQ aq;
        aq.set(ax[0], ax[1], ax[2], ax[3]);
        process_loaded(a, aq, vA, ro, vo);
    };

    if constexpr (RING) {   // (launched unfiltered only: the filter paths are not compiled in)
        // group slot: KS·64 units of rows (the group's 16·u8 units, lane-linear; lanes past them load unit
        // 0 again, never read) then 16 units of bound terms.  Per group KS + 1 LDS-DMA instructions.
        constexpr int OPS = KS + 1;
        const int SLOT = ring_slot;
        int4* ring = sq + wave * NS * SLOT;
        const uint32_t ring_lds =
            __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(__attribute__((address_space(3))) int4*)ring);
        const int4* __restrict__ X8 = p.rows8[tile.seg];
        const int n_groups = pilot ? min<int64_t>(1, (we - wb + 15) / 16) : (int)((we - wb + 15) / 16);
        auto issue = [&](int g, int slot_idx) {
            // the slot's previous group was read by this wave's ds_reads: retire them before the DMA
            // can overwrite it (the compiler may sink their consumers past this point)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const int64_t r0 = wb + (int64_t)g * 16;
            const int nu = (int)min<int64_t>(16, we - r0) * u8;
            const int4* src = X8 + r0 * u8;
            const uint32_t dst = ring_lds + (uint32_t)(slot_idx * SLOT * 16);
#pragma unroll
            for (int i = 0; i < KS; ++i) {
                const int u = i * 64 + lane;
                if (u < ring_rows) glds16(src + (u < nu ? u : 0), dst + i * 1024);
            }
            const int nr = (int)min<int64_t>(16, we - r0);
            if (lane < 16) glds16(AX + r0 + (lane < nr ? lane : 0), dst + ring_rows * 16);
        };
        constexpr int D = NS - 1;
        // slots are used round robin: group g in slot g mod NS (kept as running counters, no division)
        int s_issue = 0, s_read = 0;
        for (int g = 0; g < D && g < n_groups; ++g) {
            issue(g, s_issue);
            s_issue = s_issue + 1 == NS ? 0 : s_issue + 1;
        }
        for (int g = 0; g < n_groups; ++g) {
            if (g + D < n_groups) {
                issue(g + D, s_issue);
                s_issue = s_issue + 1 == NS ? 0 : s_issue + 1;
            }
            // this wave's LDS-DMAs issued after group g's: (min(g + D, n − 1) − g) groups
            // groups issued after this one: D in the steady state (one wait of a constant count); in the
            // last D groups nothing more is issued and waiting for everything is exact enough
            if (g + D < n_groups)
                vm_wait<D * OPS>();
            else
                vm_wait<0>();
            const int64_t r0 = wb + (int64_t)g * 16;
            const int nr = (int)min<int64_t>(16, we - r0);   // rows of this group (32-bit tests below)
            const bool vA = col < nr;
            int64_t ro[4];
            bool vo[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                ro[i] = r0 + 4 * grp + i;
                vo[i] = 4 * grp + i < nr;
            }
            const int4* slot = ring + s_read * SLOT;
            s_read = s_read + 1 == NS ? 0 : s_read + 1;
            // No masking: a chunk past the row's u8 units meets zero query bytes (the query block is
            // zero-padded), so whatever it holds adds 0 to the exact int32 dot; rows past the group's end
            // (and their bound terms) only produce lanes that vA / vo exclude.
            i32x4 a[KS];
#pragma unroll
            for (int s8 = 0; s8 < KS; ++s8) {
                const int f = s8 * 4 + grp;
                const int4 v = slot[col * u8 + (f < u8 ? f : 0)];
                a[s8] = i32x4{v.x, v.y, v.z, v.w};
            }
            // bound terms of rows 4·grp + 0..3, read as row pairs per component (ds_read2_b32); unconditional
            // reads (a read under vo[i] waited for each alone)
            const float* af = reinterpret_cast<const float*>(slot + ring_rows + 4 * grp);
            AuxQ aq;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                aq.x[h] = f32x2{af[8 * h + 0], af[8 * h + 4]};
                aq.y[h] = f32x2{af[8 * h + 1], af[8 * h + 5]};
                aq.z[h] = f32x2{af[8 * h + 2], af[8 * h + 6]};
                aq.w[h] = f32x2{af[8 * h + 3], af[8 * h + 7]};
            }
            process_loaded(a, aq, vA, ro, vo);
        }
        vm_wait<0>();
    } else if (abits && !seg.ord_to_doc) {
        // filter pushdown: the accepted rows of each 64-row window, compacted (positions in `pos`)
        for (int64_t w0 = wb; w0 < we && !sampled; w0 += 64) {
            const int64_t word = w0 >> 6;
            const int sh = (int)(w0 & 63);
            uint64_t m = abits[word] >> sh;
            if (sh && (word + 1) * 64 < we) m |= abits[word + 1] << (64 - sh);
            if (we - w0 < 64) m &= (1ull << (we - w0)) - 1ull;
            const int n = __popcll(m);
            if (n == 0) continue;
            const bool bit = (m >> lane) & 1ull;
            const int below = __popcll(m & ((1ull << lane) - 1ull));
            const int dst = bit ? below : n + (lane - below);
            const int pos = __builtin_amdgcn_ds_permute(dst << 2, lane);
            for (int i0 = 0; i0 < n && !sampled; i0 += R) {
                const int ia = i0 + col;
                const bool vA = ia < n;
                const int64_t rowA = w0 + __shfl(pos, vA ? ia : 0);
                int64_t ro[4];
                bool vo[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int io = i0 + 4 * grp + i;
                    vo[i] = io < n;
                    ro[i] = w0 + __shfl(pos, vo[i] ? io : 0);
                }
                process(rowA, vA, ro, vo);
            }
        }
    } else {
        for (int64_t r0 = wb; r0 < we && !sampled; r0 += R) {
            const int64_t rowA = r0 + col;
            const bool vA = rowA < we;
            int64_t ro[4];
            bool vo[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                ro[i] = r0 + 4 * grp + i;
                vo[i] = ro[i] < we;
                if (vo[i] && abits) {   // sparse field: accept by doc
                    const int32_t doc = seg.ord_to_doc ? seg.ord_to_doc[ro[i]] : (int32_t)ro[i];
                    vo[i] = (abits[doc >> 6] >> (doc & 63)) & 1ull;
                }
            }
            process(rowA, vA, ro, vo);
        }
    }

    if (pilot) {
        // the tile's 64 sampled keys per query (s_lk as [NQ][64]; waves with no sampled row leave
        // zeros) → its top k per query → pilot_keys [q][tile][k]: the k-th best of the union of the
        // tiles' top k is the k-th best sampled lower bound of the shard
        if (!sampled)
            for (int qb = 0; qb < QB; ++qb)
                for (int i = 0; i < 4; ++i) s_lk[(qb * 16 + col) * 64 + wave * 16 + 4 * grp + i] = 0ull;
        __syncthreads();
        for (int b = wave; b < p.q_count; b += 4) {
            const uint64_t key = s_lk[b * 64 + lane];
            int rank = 0;
#pragma unroll 8
            for (int j = 0; j < 64; ++j) rank += s_lk[b * 64 + j] > key;
            const int nz = __popcll(__ballot(key != 0ull));
            uint64_t* o = p.pilot_keys + ((size_t)b * p.n_tiles + blockIdx.x) * p.k;
            if (key != 0ull && rank < p.k) o[rank] = key;
            if (lane >= nz && lane < p.k) o[lane] = 0ull;
        }
        return;
    }
    // visited counts accepted rows: with a filter over a sparse field the unaccepted rows were
    // loaded (vA) but do not count
    if (abits && seg.ord_to_doc) {
        nvis = 0;
        for (int64_t r0 = wb + lane; r0 < we; r0 += 64) {
            const int32_t doc = seg.ord_to_doc[r0];
            nvis += (abits[doc >> 6] >> (doc & 63)) & 1ull;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) nvis += __shfl_xor(nvis, o);
    }
    // (per wave: a workgroup-level sum would add static LDS to a kernel whose dynamic LDS is sized to
    // fit 4 workgroups per CU)
    if (p.visited && p.q0 == 0 && lane == 0) atomicAdd(&p.visited[tile.seg], (unsigned long long)nvis);

    for (int b = 0; b < NQ; ++b) {
        const uint64_t lkb = lane < kKQ ? s_lk[(wave * NQ + b) * kKQ + lane] : 0ull;
        const uint32_t lpb = lane < kKQ ? s_lp[(wave * NQ + b) * kKQ + lane] : 0u;
        uint32_t m = (lane < kKQ && lkb) ? lpb : 0u;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
        if (b < p.q_count) {
            const size_t l = (size_t)(p.q0 + b) * p.n_lists + blockIdx.x * 4 + wave;
            if (lane < kKQ) {
                p.cand[l * kKQ + lane] = lkb;
                p.cand_lb[l * kKQ + lane] = lpb;
            }
            if (lane == 0) p.list_lbmax[l] = m;
        }
    }
}

using Sq8MfmaFn = void (*)(Sq8Params);
static const int kMfmaKS[6] = {2, 4, 6, 8, 12, 16};
#define OSK_MFMA_SIMS(KS, QB, RG) {sq8_mfma<KS, QB, RG, 0>, sq8_mfma<KS, QB, RG, 1>, sq8_mfma<KS, QB, RG, 2>, \
                                   sq8_mfma<KS, QB, RG, 3>}
#define OSK_MFMA_ROW(KS) {OSK_MFMA_SIMS(KS, 1, 0), OSK_MFMA_SIMS(KS, 2, 0)}
static const Sq8MfmaFn kSq8Mfma[6][2][4] = {OSK_MFMA_ROW(2), OSK_MFMA_ROW(4), OSK_MFMA_ROW(6),
                                            OSK_MFMA_ROW(8), OSK_MFMA_ROW(12), OSK_MFMA_ROW(16)};
// ring depths 2 (the default: four workgroups per CU) and 4
static const Sq8MfmaFn kSq8MfmaRing[2][2][2][4] = {
    {{OSK_MFMA_SIMS(2, 1, 2), OSK_MFMA_SIMS(2, 2, 2)}, {OSK_MFMA_SIMS(4, 1, 2), OSK_MFMA_SIMS(4, 2, 2)}},
    {{OSK_MFMA_SIMS(2, 1, 4), OSK_MFMA_SIMS(2, 2, 4)}, {OSK_MFMA_SIMS(4, 1, 4), OSK_MFMA_SIMS(4, 2, 4)}}};

int sq8_mfma_supported(int u8) { return u8 <= 4 * kMfmaKS[5]; }
// dynamic LDS of an sq8_mfma launch: queries [NQ][4·KS] units (overlaid by the ring when ns > 1) and
// the 4 waves' lists [4][NQ][kKQ] keys + lower bounds
static size_t sq8_mfma_lds(int u8, int qb, int ns) {
    int c = 0;
    while (c < 5 && 4 * kMfmaKS[c] < u8) ++c;
    const int ks = kMfmaKS[c];
    const size_t queries = (size_t)16 * qb * 4 * ks * 16, lists = (size_t)4 * 16 * qb * kKQ * 12;
    if (ns <= 1) return queries + lists;
    const size_t ring = (size_t)4 * ns * (ring_rows_units(u8, ks) + 16) * 16;
    return std::max(queries, ring) + lists;
}
// LDS-DMA ring depth for sq8_mfma: `want` (> 1), 0 (off), or -1: as many 16-row groups per wave as leave
// two 4-wave workgroups per CU within 160 KiB of LDS (KS = 2, 32 queries: 5; KS = 4: 2)
int sq8_ring_slots(int u8, int qb, int want) {
    int c = 0;
    while (c < 5 && 4 * kMfmaKS[c] < u8) ++c;
    if (c > 1 || want == 0) return 0;
    // the kernel is instantiated at depths 2 and 4: 2 by default (four workgroups per CU; deeper rings
    // measured slower), 4 when asked for a deeper one and it fits one workgroup's LDS — and by
    // default for 32-query launches of ≤ 128 dims since round 6, whose 4-slot instances take the lane-compact
    // insertions (C4 b32 2.84 → 2.67–2.71 ms, profiles/r06/call25/)
    const bool deep = want > 2 || (want < 0 && c == 0 && qb == 2);
    if (deep && sq8_mfma_lds(u8, qb, 4) <= 160 * 1024) return 4;
    return 2;
}
int sq8_mfma_ks(int u8) {
    int c = 0;
    while (c < 5 && 4 * kMfmaKS[c] < u8) ++c;
    return kMfmaKS[c];
}

__global__ __launch_bounds__(kBlock) void sq8_tile(const int4* __restrict__ q8, int64_t n_rows, int u8, int ks,
                                                   int4* __restrict__ out) {
    // one thread per 16-B unit of the tiled copy: block b, slab s, chunk c, row r (chunk-major in the slab:
    // a lane's MFMA fragment — row lane & 15, chunk lane >> 4 — is lane-linear, and the slab's first two
    // chunks, a K = 32 tail, are its first 512 B)
    const int64_t n_units = ((n_rows + 15) / 16) * ks * 64;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n_units; i += (int64_t)gridDim.x * kBlock) {
        const int64_t b = i / (ks * 64);
        const int rem = (int)(i - b * ks * 64);
        const int s = rem >> 6, c = (rem >> 4) & 3, r = rem & 15;
        const int64_t row = b * 16 + r;
        const int f = s * 4 + c;
        out[i] = (row < n_rows && f < u8) ? q8[row * u8 + f] : make_int4(0, 0, 0, 0);
    }
}

hipError_t launch_sq8_tile(const void* q8, int64_t n_rows, int u8, int ks, void* out, hipStream_t s) {
    const int64_t n_units = std::max<int64_t>(1, ((n_rows + 15) / 16) * ks * 64);
    int64_t blocks = (n_units + kBlock - 1) / kBlock;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(sq8_tile, dim3((unsigned)blocks), dim3(kBlock), 0, s, static_cast<const int4*>(q8), n_rows,
                       u8, ks, static_cast<int4*>(out));
    return hipGetLastError();
}

hipError_t launch_sq8_mfma(const Sq8Params& p, hipStream_t s, hipEvent_t ev_start, hipEvent_t ev_stop) {
    int c = 0;
    while (c < 5 && 4 * kMfmaKS[c] < p.units8) ++c;
    if (4 * kMfmaKS[c] < p.units8) return hipErrorInvalidValue;
    const int qb = p.q_count > 16 ? 2 : 1;
    size_t lds = sq8_mfma_lds(p.units8, qb, 0);
    if (p.sim < 0 || p.sim > 3) return hipErrorInvalidValue;
    auto fn = kSq8Mfma[c][qb - 1][p.sim];
    if (p.ring_slots >= 2 && !p.accept && c <= 1) {   // LDS-DMA ring (unfiltered, ≤ 256 dims)
        if (p.ring_slots != 2 && p.ring_slots != 4) return hipErrorInvalidValue;
        fn = kSq8MfmaRing[p.ring_slots == 4][c][qb - 1][p.sim];
        lds = sq8_mfma_lds(p.units8, qb, p.ring_slots);
        if (lds > 160 * 1024) return hipErrorInvalidValue;
    }
    if (ev_start || ev_stop)
        hipExtLaunchKernelGGL(fn, dim3(p.n_tiles), dim3(kBlock), lds, s, ev_start, ev_stop, 0, p);
    else
        hipLaunchKernelGGL(fn, dim3(p.n_tiles), dim3(kBlock), lds, s, p);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// settle, in slices of kSliceLists wave lists (≤ 512 entries), one workgroup per (slice, query), so
// every (query, shard) spreads over many workgroups (one workgroup per (query, shard) is
// latency-bound: ~50 µs):
//   sq8_settle        L_g = the k-th best of the lists' best lower bounds over a group of up to
//                     kLGroupLists lists of the shard (k distinct rows) — at most the shard's k-th
//                     best lower bound, so excluding a row with ub < L_g is sound; the slice's rows
//                     with ub ≥ L_g are re-scored exactly; a
//                     wave list that is full and whose last ub reaches L_g (it may have dropped a
//                     qualifying row) has its row range re-scanned exactly inside the same
//                     workgroup (rare; no fallback launch).
//                     The slice's top k → part.
//   sq8_settle_merge  per (query, shard): the top k of its slices' lists → shard keys / counts.
// ------------------------------------------------------------------------------------------------
constexpr int kSettleThreads = 256;
constexpr int kSettleWaves = kSettleThreads / 64;

template <int L, int V, bool L2K>
__global__ __launch_bounds__(kSettleThreads) void sq8_settle(SettleParams p) {
    constexpr int R = 64 / L, UP = L * V;
    __shared__ uint64_t s_lists[kSettleWaves * 64];
    __shared__ uint64_t s_top[64];
    __shared__ uint32_t s_cand[kSliceLists * kKQ];
    __shared__ __attribute__((aligned(16))) uint64_t s_keys[64];
    __shared__ int s_nc;
    __shared__ uint32_t s_L;
    __shared__ uint32_t s_exact;   // bit i: list l0 + i of the slice is re-scanned exactly
    const int g = blockIdx.x, q = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform: scalar loop control
    const int t = lane & (L - 1), gr = lane / L;
    const int k = p.k, sim = p.sim;
    if (p.trace && tid == 0) p.trace[((size_t)q * p.n_slices + g) * 8 + 0] = wall_clock64();
    const int4 sl = p.slices[g];   // {first list, end list, first list of the L group, its end}
    const int nt = sl.y - sl.x, n = nt * kKQ;
    const size_t base = ((size_t)q * p.n_lists + sl.x) * kKQ;
    constexpr int kEnt = kSliceLists * kKQ / kSettleThreads;   // entries per thread
    uint64_t key[kEnt];
#pragma unroll
    for (int u = 0; u < kEnt; ++u) {
        const int e = u * kSettleThreads + tid;
        key[u] = e < n ? p.cand[base + e] : 0ull;
    }
    // query fragments and norm: independent of everything below, issued first
    const float4* __restrict__ Q = reinterpret_cast<const float4*>(p.q) + (size_t)q * UP;
    float4 qf[V];
#pragma unroll
    for (int j = 0; j < V; ++j) qf[j] = Q[t + j * L];
    const float qn = (!L2K && sim == SIM_COSINE) ? p.qnorm[q] : 0.0f;
    const SegDev seg0 = p.segs[0];   // the common case (one segment per view) needs no lookup below
    if (tid == 0) {
        s_nc = 0;
        s_exact = p.force_fail ? (nt >= 32 ? 0xFFFFFFFFu : (1u << nt) - 1u) : 0u;
    }
    if (tid < 64) s_top[tid] = 0ull;

    // (a) L_g: the k-th best of 64 maxima of the best lower bounds of the group's lists (each over
    // 64 lists).  Each maximum belongs to a distinct row, so L_g ≤ the shard's k-th best lower
    // bound; every block of the group computes the same L_g.  Selection by rank (no serial
    // insertion chain).
    uint32_t mx = 0u;
    {
        constexpr int kPer = kLGroupLists / kSettleThreads;
        const uint32_t* __restrict__ lm = p.list_lbmax + (size_t)q * p.n_lists;
        const int ne = sl.w - sl.z;
        uint32_t m[kPer];
        // thread t holds lists (t & 3)·64 + (t >> 2) + 256·u: the 4 threads of a bucket t >> 2 hold
        // lists ≡ bucket (mod 64), so a group of ≤ 64 lists keeps one list per bucket (exact k-th)
        const int i0 = (tid & 3) * 64 + (tid >> 2);
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int i = u * kSettleThreads + i0;
            m[u] = i < ne ? lm[sl.z + i] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kPer; ++u) mx = max(mx, m[u]);
    }
    if (p.trace && tid == 0) p.trace[((size_t)q * p.n_slices + g) * 8 + 1] = wall_clock64();
    // 4 adjacent threads' maxima → 64 values (one per 64 lists), ranked by 64 threads
#pragma unroll
    for (int o = 1; o <= 2; o <<= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    if ((tid & 3) == 0) s_keys[tid >> 2] = ((uint64_t)mx << 32) | (uint32_t)(tid >> 2);   // distinct
    __syncthreads();
    if (tid < 64) {
        const uint64_t mkey = s_keys[tid];
        int rank = 0;
#pragma unroll
        for (int j = 0; j < 64; j += 2) {
            const ulonglong2 v2 = *reinterpret_cast<const ulonglong2*>(s_keys + j);
            rank += (v2.x > mkey) + (v2.y > mkey);
        }
        if (rank == k - 1) s_L = (uint32_t)(mkey >> 32);   // 0 when fewer than k lists hold rows
    }
    __syncthreads();
    const uint32_t Lb = s_L;
    // (b) overflowed lists → exact row ranges; the other lists' rows with ub ≥ L_g → candidates
    bool reach[kEnt];
#pragma unroll
    for (int u = 0; u < kEnt; ++u) {
        const int e = u * kSettleThreads + tid;
        reach[u] = key[u] && (uint32_t)(key[u] >> 32) >= Lb;
        if (reach[u] && (e % kKQ) == kKQ - 1) atomicOr(&s_exact, 1u << (e / kKQ));
    }
    __syncthreads();
    const uint32_t exact = s_exact;
#pragma unroll
    for (int u = 0; u < kEnt; ++u) {
        const int e = u * kSettleThreads + tid;
        if (reach[u] && !((exact >> (e / kKQ)) & 1u)) s_cand[atomicAdd(&s_nc, 1)] = 0xFFFFFFFFu - (uint32_t)key[u];
    }
    if (tid < 64) s_top[tid] = 0ull;   // every thread has read L_g (barrier above)
    __syncthreads();
    const int nc = s_nc;
    if (p.trace && tid == 0) p.trace[((size_t)q * p.n_slices + g) * 8 + 2] = wall_clock64();
    if (tid == 0) {
        if (exact) {
            if (atomicOr(&p.flags[q], 1) == 0) atomicAdd(&p.counters[0], 1ull);
            atomicAdd(&p.counters[2], (unsigned long long)__popc(exact));
        }
        if (nc) atomicAdd(&p.counters[1], (unsigned long long)nc);
    }

    // (c) exact re-score of the candidates
    uint64_t lk = 0ull, thr = 0ull;
    for (int i0 = wave * R; i0 < nc; i0 += kSettleWaves * R) {
        const int ci = i0 + gr;
        const bool valid = ci < nc;
        const uint32_t vrow = s_cand[valid ? ci : 0];
        int sg = 0;
        for (int j = 1; j < p.n_segs; ++j)
            if ((int64_t)vrow >= p.seg_vrow[j]) sg = j;
        const SegDev seg = sg == 0 ? seg0 : p.segs[sg];
        const int64_t ord = (int64_t)vrow - (sg == 0 ? 0 : p.seg_vrow[sg]);
        const int32_t doc = seg.ord_to_doc ? seg.ord_to_doc[ord] : (int32_t)ord;
        const float xn = (!L2K && sim == SIM_COSINE && valid) ? seg.xnorm_f[ord] : 0.0f;
        const float sc = settle_exact<L, V, L2K>(static_cast<const float4*>(seg.rows) + ord * p.units, valid,
                                                 p.units, t, qf, sim, qn, xn);
        wave_offer(valid ? make_key(sc, (uint32_t)(seg.doc_base + doc)) : 0ull, t == 0, lk, thr, lane, k);
    }
    if (p.trace && tid == 0) p.trace[((size_t)q * p.n_slices + g) * 8 + 3] = wall_clock64();
    // (c') overflowed lists: every accepted row of the scan wave's range (the scan's split of its
    // tile: per_wave = ⌈rows / 4R_s⌉·R_s), walked by this block's 4 waves (filter pushdown included)
    for (uint32_t bits = exact; bits && p.gtiles; bits &= bits - 1u) {
        // gather mode: the scan wave's quarter of its gather tile's compacted ordinals (all accepted)
        const int list = sl.x + __builtin_ctz(bits);
        const int4 gt = p.gtiles[list >> 2];
        const SegDev seg = p.segs[gt.x];
        int64_t lb0, lb1;
        gather_wave_range(min<int64_t>(p.scnt[gt.x], seg.n_rows), gt.z, gt.w, p.gather_min, list & 3, lb0, lb1);
        const uint32_t* __restrict__ C = p.comp + p.seg_vrow[gt.x];
        const int64_t per_wave = ((lb1 - lb0 + kSettleWaves * R - 1) / (kSettleWaves * R)) * R;
        const int64_t wb = lb0 + wave * per_wave;
        const int64_t we = min(wb + per_wave, lb1);
        const float4* X = static_cast<const float4*>(seg.rows);
        for (int64_t e0 = wb; e0 < we; e0 += R) {
            const bool valid = e0 + gr < we;
            const int64_t row = valid ? min<int64_t>(C[e0 + gr], seg.n_rows - 1) : 0;
            const int32_t doc = valid ? (seg.ord_to_doc ? seg.ord_to_doc[row] : (int32_t)row) : 0;
            const float xn = (!L2K && sim == SIM_COSINE && valid) ? seg.xnorm_f[row] : 0.0f;
            const float sc = settle_exact<L, V, L2K>(X + row * p.units, valid, p.units, t, qf, sim, qn, xn);
            wave_offer(valid ? make_key(sc, (uint32_t)(seg.doc_base + doc)) : 0ull, t == 0, lk, thr, lane, k);
        }
    }
    for (uint32_t bits = p.gtiles ? 0u : exact; bits; bits &= bits - 1u) {
        const int list = sl.x + __builtin_ctz(bits);
        const TileDev td = p.tiles[list >> 2];
        const SegDev seg = p.segs[td.seg];
        const uint64_t* abits = p.accept ? p.accept[td.seg] : nullptr;
        const int64_t trows = td.row_end - td.row_begin;
        const int64_t spw = ((trows + 4 * p.scan_R - 1) / (4 * p.scan_R)) * p.scan_R;
        const int64_t lb0 = min(td.row_begin + (list & 3) * spw, td.row_end);
        const int64_t lb1 = min(lb0 + spw, td.row_end);
        const int64_t rows = lb1 - lb0;
        const int64_t per_wave = ((rows + kSettleWaves * R - 1) / (kSettleWaves * R)) * R;
        const int64_t wb = lb0 + wave * per_wave;
        const int64_t we = min(wb + per_wave, lb1);
        const float4* X = static_cast<const float4*>(seg.rows);
        walk_rows<R>(wb, we, abits, seg.ord_to_doc, lane, gr, [&](const int64_t row, bool valid, bool known) {
            int32_t doc = 0;
            if (valid) {
                doc = seg.ord_to_doc ? seg.ord_to_doc[row] : (int32_t)row;
                if (abits && !known) valid = (abits[doc >> 6] >> (doc & 63)) & 1ull;
            }
            const float xn = (!L2K && sim == SIM_COSINE && valid) ? seg.xnorm_f[row] : 0.0f;
            const float sc = settle_exact<L, V, L2K>(X + row * p.units, valid, p.units, t, qf, sim, qn, xn);
            wave_offer(valid ? make_key(sc, (uint32_t)(seg.doc_base + doc)) : 0ull, t == 0, lk, thr, lane, k);
        });
    }
    // (d) the slice's top k → part
    s_lists[wave * 64 + lane] = lane < k ? lk : 0ull;
    __syncthreads();
    block_rank_topk<kSettleWaves>(s_lists, k, tid, s_top);
    __syncthreads();
    if (tid < k) p.part[((size_t)q * p.n_slices + g) * k + tid] = s_top[tid];
    if (p.trace && tid == 0) {
        p.trace[((size_t)q * p.n_slices + g) * 8 + 4] = wall_clock64();
        p.trace[((size_t)q * p.n_slices + g) * 8 + 5] = (unsigned long long)nc;
    }
}

// per (shard, query): the top k of the shard's slice lists → shard keys and counts.
// Selection without a serial insertion chain: t = the k-th best of 64 bucket maxima of the lists'
// first (best) keys — a lower bound of the k-th best key (distinct keys) — then only keys ≥ t
// (≈ k … 2k of them) are ranked against each other in LDS.
constexpr int kMergeCap = 2048;
__global__ __launch_bounds__(kSettleThreads) void sq8_settle_merge(SettleParams p) {
    __shared__ __attribute__((aligned(16))) uint64_t s_b[64];
    __shared__ __attribute__((aligned(16))) uint64_t s_surv[kMergeCap];
    __shared__ uint64_t s_top[64];
    __shared__ int s_ns;
    __shared__ uint64_t s_t;
    const int sh = blockIdx.x, q = blockIdx.y, S = p.n_shards, k = p.k;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform: scalar loop control
    const int g0 = p.shard_slice_begin[sh], g1 = p.shard_slice_begin[sh + 1];
    const uint64_t* __restrict__ src = p.part + ((size_t)q * p.n_slices + g0) * k;
    const int nl = g1 - g0, n = nl * k;
    if (tid == 0) { s_ns = 0; s_t = 0ull; }
    if (tid < 64) s_top[tid] = 0ull;
    if (n <= kSettleThreads) {
        // few keys (a shard of ≤ 25 slice lists at k = 10): rank them all directly, one per thread.
        // Keys are distinct (they carry the doc) or 0 = empty.
        const uint64_t key = tid < n ? src[tid] : 0ull;
        s_surv[tid] = key;
        __syncthreads();
        if (key) {
            int rank = 0;
            const int n2 = (n + 1) & ~1;   // s_surv[n] is a 0 key when n is odd
#pragma unroll 4
            for (int j = 0; j < n2; j += 2) {
                const ulonglong2 v2 = *reinterpret_cast<const ulonglong2*>(s_surv + j);
                rank += (v2.x > key) + (v2.y > key);
            }
            if (rank < k) s_top[rank] = key;
        }
        __syncthreads();
        if (wave == 0) {
            const uint64_t kk = lane < k ? s_top[lane] : 0ull;
            const size_t o = (size_t)q * S + sh;
            if (lane < k) p.shard_keys[o * k + lane] = kk;
            const int cnt = __popcll(__ballot(kk != 0ull));
            if (lane == 0) p.shard_counts[o] = cnt;
        }
        return;
    }
    // bucket maxima of the lists' first keys (list l → bucket l mod 64), one bucket per lane of wave 0
    // (no 64-bit LDS atomics: tools/mc_micro.hip measured them at several µs per block)
    if (tid < 64) {
        uint64_t m = 0ull;
        for (int l = tid; l < nl; l += 64) m = max(m, src[(size_t)l * k]);
        s_b[tid] = m;
    }
    __syncthreads();
    if (tid < 64) {
        const uint64_t v = s_b[tid];
        int rank = 0;
#pragma unroll
        for (int j = 0; j < 64; j += 2) {
            const ulonglong2 v2 = *reinterpret_cast<const ulonglong2*>(s_b + j);
            rank += (v2.x > v) + (v2.y > v);
        }
        // buckets are distinct keys or 0; with fewer than k non-empty buckets t stays 0
        if (rank == k - 1 && v) s_t = v;
    }
    __syncthreads();
    const uint64_t t = s_t;
    for (int e = tid; e < n; e += kSettleThreads) {
        const uint64_t key = src[e];
        if (key && key >= t) {
            const int slot = atomicAdd(&s_ns, 1);
            if (slot < kMergeCap) s_surv[slot] = key;
        }
    }
    __syncthreads();
    const int ns = s_ns;
    if (ns <= kMergeCap) {
        for (int i = tid; i < ns; i += kSettleThreads) {
            const uint64_t key = s_surv[i];
            int rank = 0;
            for (int j = 0; j < ns && rank < k; ++j) rank += s_surv[j] > key;
            if (rank < k) s_top[rank] = key;
        }
    } else if (wave == 0) {   // degenerate (> kMergeCap keys ≥ t): one wave inserts them all
        uint64_t lk = 0ull, thr = 0ull;
        for (int i0 = 0; i0 < n; i0 += 64) {
            const int i = i0 + lane;
            wave_offer(i < n ? src[i] : 0ull, true, lk, thr, lane, k);
        }
        if (lane < k) s_top[lane] = lk;
    }
    __syncthreads();
    if (wave == 0) {
        const uint64_t key = lane < k ? s_top[lane] : 0ull;
        const size_t o = (size_t)q * S + sh;
        if (lane < k) p.shard_keys[o * k + lane] = key;
        const int cnt = __popcll(__ballot(key != 0ull));
        if (lane == 0) p.shard_counts[o] = cnt;
    }
}

// ------------------------------------------------------------------------------------------------
// the settle of a wide batch, one workgroup per (shard, query):
//   (a) L = the k-th best of 64 bucket maxima of the lists' best lower bounds over ALL the shard's lists
//       (bucket = list mod 64: each maximum is a distinct row's lb, so L ≤ the shard's k-th best lb — the
//       per-slice settle's argument over one group of the shard's lists; over all of them L is no lower);
//   (b) the lists in chunks of 256: a list with no row (best lb 0) is skipped without reading its keys;
//       a full list whose 16th upper bound reaches L (it may have dropped a qualifying row) is re-scanned
//       exactly; the other lists' rows with ub ≥ L are re-scored exactly (scan_f32's arithmetic);
//   (c) the 16 waves' top k → shard_keys / shard_counts.
// Exactness is sq8_settle's: every row of the shard's top k has ub ≥ exact ≥ T ≥ L, so it is re-scored or
// lies in a re-scanned list.
// ------------------------------------------------------------------------------------------------
constexpr int kWideChunk = 256;   // lists per chunk of the list walk
// 16 waves per (shard, query): a wide batch has few of these workgroups (C2 b256: 256, one per CU), and
// the walk and the re-score are latency-bound chains, so more waves per workgroup hide more of them
constexpr int kWideSettleWaves = 16, kWideSettleThreads = kWideSettleWaves * 64;
template <int L, int V, bool L2K>
__global__ __launch_bounds__(kWideSettleThreads) void sq8_settle_wide(SettleParams p) {
    constexpr int R = 64 / L, UP = L * V;
    __shared__ uint32_t s_bm[kWideSettleWaves][64];
    __shared__ uint64_t s_keys[64];
    __shared__ uint32_t s_L;
    __shared__ uint32_t s_cand[kWideChunk * kKQ];
    __shared__ int32_t s_exact[kWideChunk];
    __shared__ int s_nc, s_ne;
    __shared__ uint64_t s_lists[kWideSettleWaves * 64];
    __shared__ uint64_t s_top[64];
    const int sh = blockIdx.x, q = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int t = lane & (L - 1), gr = lane / L;
    const int k = p.k, sim = p.sim;
    const int l0 = 4 * p.shard_tile_begin[sh], l1 = 4 * p.shard_tile_begin[sh + 1];
    const uint32_t* __restrict__ lm = p.list_lbmax + (size_t)q * p.n_lists;
    // (a) bucket maxima: thread t takes lists l0 + t + 1024j (bucket t mod 64, 16 threads per bucket)
    uint32_t mx = 0u;
    for (int l = l0 + tid; l < l1; l += kWideSettleThreads) mx = max(mx, lm[l]);
    s_bm[wave][lane] = mx;
    const float4* __restrict__ Q = reinterpret_cast<const float4*>(p.q) + (size_t)q * UP;
    float4 qf[V];
#pragma unroll
    for (int j = 0; j < V; ++j) qf[j] = Q[t + j * L];
    const float qn = (!L2K && sim == SIM_COSINE) ? p.qnorm[q] : 0.0f;
    __syncthreads();
    if (tid < 64) {
        uint32_t m = 0u;
#pragma unroll
        for (int w = 0; w < kWideSettleWaves; ++w) m = max(m, s_bm[w][tid]);
        s_keys[tid] = ((uint64_t)m << 32) | (uint32_t)tid;   // distinct
    }
    __syncthreads();
    if (tid < 64) {
        const uint64_t mkey = s_keys[tid];
        int rank = 0;
        for (int j = 0; j < 64; ++j) rank += s_keys[j] > mkey;
        if (rank == k - 1) s_L = (uint32_t)(mkey >> 32);   // (0 when fewer than k lists hold rows)
        if (tid == 0 && k > 64) s_L = 0u;
    }
    if (tid == 0) {
        s_nc = 0;
        s_ne = 0;
    }
    __syncthreads();
    const uint32_t Lb = s_L;
    uint64_t lk = 0ull, thr = 0ull;   // this wave's top k of re-scored rows
    unsigned long long n_res = 0, n_exact = 0;
    auto rescore = [&](uint32_t vrow, bool valid) {
        int sg = 0;
        for (int j = 1; j < p.n_segs; ++j)
            if ((int64_t)vrow >= p.seg_vrow[j]) sg = j;
        const SegDev seg = p.segs[sg];
        const int64_t ord = (int64_t)vrow - p.seg_vrow[sg];
        const int32_t doc = valid ? (seg.ord_to_doc ? seg.ord_to_doc[ord] : (int32_t)ord) : 0;
        const float xn = (!L2K && sim == SIM_COSINE && valid) ? seg.xnorm_f[ord] : 0.0f;
        const float sc = settle_exact<L, V, L2K>(static_cast<const float4*>(seg.rows) + ord * p.units, valid,
                                                 p.units, t, qf, sim, qn, xn);
        wave_offer(valid ? make_key(sc, (uint32_t)(seg.doc_base + doc)) : 0ull, t == 0, lk, thr, lane, k);
    };
    for (int c0 = l0; c0 < l1; c0 += kWideChunk) {
        const int c1 = min(c0 + kWideChunk, l1);
        // (b) 4 lists per wave-iteration, 16 lanes each: entry e = lane & 15 of list c0 + 4i + (lane >> 4);
        // kWideUnroll iterations' best bounds and keys are loaded together (one round trip, not two per
        // iteration: the walk was latency-bound, 39 µs per C2 b256 search), an empty list's (best lb 0)
        // keys masked to 0 after the load
        constexpr int kWideUnroll = 4;
        const int e = lane & 15;
        for (int i0 = wave; 4 * i0 < c1 - c0; i0 += kWideSettleWaves * kWideUnroll) {
            uint32_t lmv[kWideUnroll];
            uint64_t kv[kWideUnroll];
            bool in[kWideUnroll];
#pragma unroll
            for (int u = 0; u < kWideUnroll; ++u) {
                const int l = c0 + 4 * (i0 + u * kWideSettleWaves) + (lane >> 4);
                in[u] = l < c1;
                const int lc = in[u] ? l : c0;
                lmv[u] = lm[lc];
                kv[u] = p.cand[((size_t)q * p.n_lists + lc) * kKQ + e];
            }
#pragma unroll
            for (int u = 0; u < kWideUnroll; ++u) {
                const int l = c0 + 4 * (i0 + u * kWideSettleWaves) + (lane >> 4);
                const uint64_t key = (in[u] && lmv[u] != 0u) ? kv[u] : 0ull;
                const bool reach = key && (uint32_t)(key >> 32) >= Lb;
                const uint64_t full = __ballot(reach && e == kKQ - 1);   // the list's 16th key reaches L
                const bool exact = (full >> (lane | 15)) & 1ull;
                if (reach && e == kKQ - 1) s_exact[atomicAdd(&s_ne, 1)] = l;
                if (reach && !exact) s_cand[atomicAdd(&s_nc, 1)] = 0xFFFFFFFFu - (uint32_t)key;
            }
        }
        __syncthreads();
        const int nc = s_nc, ne = s_ne;
        n_res += nc;
        n_exact += ne;
        for (int i0 = wave * R; i0 < nc; i0 += kWideSettleWaves * R) {
            const int ci = i0 + gr;
            rescore(s_cand[ci < nc ? ci : 0], ci < nc);
        }
        // (b') lists that may have dropped a qualifying row: every row of the scan quarter, exactly
        for (int x = 0; x < ne; ++x) {
            const int list = s_exact[x];
            const TileDev td = p.tiles[list >> 2];
            const SegDev seg = p.segs[td.seg];
            const int64_t trows = td.row_end - td.row_begin;
            const int64_t spw = ((trows + 4 * p.scan_R - 1) / (4 * p.scan_R)) * p.scan_R;
            const int64_t lb0 = min(td.row_begin + (list & 3) * spw, td.row_end);
            const int64_t lb1 = min(lb0 + spw, td.row_end);
            const int64_t per_wave = ((lb1 - lb0 + kWideSettleWaves * R - 1) / (kWideSettleWaves * R)) * R;
            const int64_t wb = lb0 + wave * per_wave, we = min(wb + per_wave, lb1);
            const float4* X = static_cast<const float4*>(seg.rows);
            for (int64_t r0 = wb; r0 < we; r0 += R) {
                const int64_t row = r0 + gr;
                const bool valid = row < we;
                const int32_t doc = valid ? (seg.ord_to_doc ? seg.ord_to_doc[row] : (int32_t)row) : 0;
                const float xn = (!L2K && sim == SIM_COSINE && valid) ? seg.xnorm_f[row] : 0.0f;
                const float sc = settle_exact<L, V, L2K>(X + (valid ? row : 0) * p.units, valid, p.units, t, qf, sim, qn, xn);
                wave_offer(valid ? make_key(sc, (uint32_t)(seg.doc_base + doc)) : 0ull, t == 0, lk, thr, lane, k);
            }
        }
        __syncthreads();   // every wave is done with this chunk's candidates before the counters reset
        if (tid == 0) {
            s_nc = 0;
            s_ne = 0;
        }
        __syncthreads();
    }
    if (tid == 0) {
        if (n_exact) {
            if (atomicOr(&p.flags[q], 1) == 0) atomicAdd(&p.counters[0], 1ull);
            atomicAdd(&p.counters[2], n_exact);
        }
        if (n_res) atomicAdd(&p.counters[1], n_res);
    }
    // (c) the shard's top k
    s_lists[wave * 64 + lane] = lane < k ? lk : 0ull;
    if (tid < 64) s_top[tid] = 0ull;
    __syncthreads();
    block_rank_topk<kWideSettleWaves>(s_lists, k, tid, s_top);
    __syncthreads();
    if (wave == 0) {
        const uint64_t key = lane < k ? s_top[lane] : 0ull;
        const size_t o = (size_t)q * p.n_shards + sh;
        if (lane < k) p.shard_keys[o * k + lane] = key;
        const int cnt = __popcll(__ballot(key != 0ull));
        if (lane == 0) p.shard_counts[o] = cnt;
    }
}

using SettleFn = void (*)(SettleParams);
#define OSK_SETTLE_ROW(L, V) {sq8_settle<L, V, false>, sq8_settle<L, V, true>}
static const SettleFn kSettle[9][2] = {OSK_SETTLE_ROW(4, 2),  OSK_SETTLE_ROW(8, 2),  OSK_SETTLE_ROW(8, 4),
                                       OSK_SETTLE_ROW(16, 4), OSK_SETTLE_ROW(16, 8), OSK_SETTLE_ROW(16, 12),
                                       OSK_SETTLE_ROW(32, 8), OSK_SETTLE_ROW(64, 8), OSK_SETTLE_ROW(64, 16)};

// (the wide kernel takes rows of ≤ 768 dims, sq8_wide_supported: settle configs 0–5)
#define OSK_SETTLE_WIDE_ROW(L, V) {sq8_settle_wide<L, V, false>, sq8_settle_wide<L, V, true>}
static const SettleFn kSettleWide[6][2] = {OSK_SETTLE_WIDE_ROW(4, 2),  OSK_SETTLE_WIDE_ROW(8, 2),
                                           OSK_SETTLE_WIDE_ROW(8, 4),  OSK_SETTLE_WIDE_ROW(16, 4),
                                           OSK_SETTLE_WIDE_ROW(16, 8), OSK_SETTLE_WIDE_ROW(16, 12)};

hipError_t launch_sq8_settle_wide(int cfg, int nq, const SettleParams& p, hipStream_t s) {
    if (p.accept || p.gtiles || !p.shard_tile_begin || p.k < 1 || p.k > 64 || cfg < 0 || cfg > 5) return hipErrorInvalidValue;
    hipLaunchKernelGGL(kSettleWide[cfg][p.sim == SIM_EUCLIDEAN ? 1 : 0], dim3(p.n_shards, nq), dim3(kWideSettleThreads), 0,
                       s, p);
    return hipGetLastError();
}

hipError_t launch_sq8_settle(int cfg, int nq, const SettleParams& p, hipStream_t s) {
    hipLaunchKernelGGL(kSettle[cfg][p.sim == SIM_EUCLIDEAN ? 1 : 0], dim3(p.n_slices, nq), dim3(kSettleThreads), 0, s,
                       p);
    hipLaunchKernelGGL(sq8_settle_merge, dim3(p.n_shards, nq), dim3(kSettleThreads), 0, s, p);
    return hipGetLastError();
}

}  // namespace osk
