// osk_sq6.hip — the 6-bit first tier of the certified prefilter (single unfiltered queries over
// float32 fields of ≥ 512 dims).
//
// The int8 prefilter (osk_sq8.hip) streams 768 + 16 B per 768-dim row at 0.94 of the measured HBM read
// ceiling, so a single query can only get faster by reading fewer bytes.  Here each row is also kept as
// 6-bit codes (per-row symmetric scale s = max|x|/31, q ∈ [-31, 31]) plus the same 16-B bound terms
// {s, s·|q|, |x − s·q|, |x|²}: 576 + 16 B per 768-dim row, 0.755 of the int8 bytes.  The 6-bit interval
// is sq8_bounds' (its Cauchy–Schwarz bound holds for any quantiser) but ≈ 2.6× wider than the int8 one,
// too wide to build the settle's lists from directly (on isotropic 768-dim data ≈ 1.9 % of a C3 shard's
// rows reach the re-score and 8 % of the lists overflow).  So the 6-bit pass only filters, against a
// per-(query, shard) FLOOR, and the int8 copy re-bounds what passes:
//   sq6_pilot    the first 8 rows of every scan wave (2 % of the rows) on the int8 copy: their lower
//                bounds seed 64 floor buckets per shard (bucket = wave list mod 64, atomicMax);
//   sq6_scan     streams the 6-bit codes; a row whose 6-bit upper bound is below the floor T = the k-th
//                best of the 64 bucket maxima is dropped (T ≤ the shard's k-th best exact score, so it
//                cannot enter the top k); the rest (≈ 1.3–1.6 % at C3) go to the wave's candidate buffer,
//                and their 6-bit lower bounds raise the buckets as the pass goes (only while they can
//                still lift the floor: same-address atomics queue at L2);
//   sq6_rebound  one wave per scan wave's list: the candidates' int8 intervals, sq8_scan's quick test and
//                list insertion; writes the lists the settle reads (osk_sq8.hip sq8_settle, scan_R = 8).
// Results are bit-identical to the fp32 streaming scan.  Tiles are dispatched interleaved over shards
// (osk_view::d_tile_order) so every round of workgroups scans a slice of every shard and each shard's
// floor rises from the first round.  4-bit and 5-bit codes were simulated and rejected: their bounds
// pass ≈ 100 % and ≈ 18 % of isotropic 768-dim rows.  A segment whose first probe calls send more than
// sq6_probe_pct % of its rows to the re-bound (e.g. uniform EUCLIDEAN rows, whose 6-bit bounds do not
// separate) stops using the tier (osk_api.hip fold_probe).
//
// Code layout (per segment, "tiled"): blocks of 8 rows.  Lane t ∈ [0, 8) of a row owns the half-chunks
// hc = 8j + t (j < C), each 32 dims [32hc, 32hc + 32); C = ⌈dim / 256⌉.  A code q = 4h + l with
// h = q >> 2 ∈ [-8, 7] (signed nibble) and l = q & 3 ∈ [0, 3]:
//   hi slab j of a block: [8 rows][8 lanes][16 B] — dword m (< 4), nibble n: h of dim 32hc + 8m + n;
//   lo slab j:            [8 rows][8 lanes][8 B]  — dword w (< 2), nibble n: l of dim 32hc + 16w + n
//                                                   in bits 4n..4n+1 and l of dim 32hc + 16w + 8 + n in
//                                                   bits 4n+2..4n+3.
// Block bytes: C·(1024 + 512).  Every load instruction of a wave reads 1 KiB (hi) or 512 B (lo)
// contiguous.  The query is quantised to [-119, 119] (s_b = max|b|/119) and split b = 16·bh + bl into
// two signed nibbles (bl = ((b + 8) & 15) − 8, |bh| ≤ 7), stored per half-chunk as 8 dwords: bh of dims
// 8m..8m+7 (m < 4), then bl of the same dims.  The exact int32 dot is then
//   Σ q·b = 64·Σh·bh + 4·Σh·bl + 16·Σl·bh + Σl·bl,
// eight v_dot8_i32_i4 per hi dword pair and lo dword (the lo plane is spread to nibbles with one and,
// one shift + and: (w & 0x33333333) pairs with query dword 2w, ((w >> 2) & 0x33333333) with 2w + 1).
#include <hip/hip_ext.h>

#include <atomic>

#include "osk_device.h"
#include "osk_internal.h"
#include "osk_wave.h"

namespace osk {

int sq6_chunks(int dim) { return (dim + 255) / 256; }

// Worth a separate copy only when the 6-bit rows are clearly smaller than the int8 rows (dims are
// padded to 256 per lane set), within the instantiated C.
int sq6_supported(int dim) {
    const int C = sq6_chunks(dim);
    if (C < 2 || C > 6) return 0;   // C = 7, 8 spill past 128 VGPRs
    const int u8 = (dim + 15) / 16;
    return 192 * C * 10 <= 16 * u8 * 8 ? 1 : 0;   // 6-bit bytes ≤ 0.8 × int8 bytes
}

int64_t sq6_bytes(int64_t n_rows, int dim) {
    return std::max<int64_t>(1, (n_rows + 7) / 8) * (int64_t)sq6_chunks(dim) * 1536 +
           std::max<int64_t>(1, n_rows) * 16;
}

// ------------------------------------------------------------------------------------------------
// quantisation of a segment's rows (one wave per row; lane c < 8C owns half-chunk c).  aux as
// sq8_quantize's mode 0: {s, s·|q|, |x − s·q|, |x|²} in double, rounded up (|x|² to nearest).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void sq6_quantize(const float4* __restrict__ X, int64_t n, int units, int C,
                                                       char* __restrict__ out, float4* __restrict__ aux) {
    const int lane = threadIdx.x & 63;
    const int64_t wave_global = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) >> 6;
    const bool mine = lane < 8 * C;
    for (int64_t r = wave_global; r < n; r += n_waves) {
        const float4* xr = X + r * units;
        float xs[32];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int f = lane * 8 + i;
            const float4 x = (mine && f < units) ? xr[f] : make_float4(0.f, 0.f, 0.f, 0.f);
            xs[4 * i] = x.x;
            xs[4 * i + 1] = x.y;
            xs[4 * i + 2] = x.z;
            xs[4 * i + 3] = x.w;
        }
        float m = 0.0f;
#pragma unroll
        for (int e = 0; e < 32; ++e) m = fmaxf(m, fabsf(xs[e]));
        for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
        const float s = m / 31.0f;
        long long sq = 0;
        double se = 0.0, sx = 0.0;
        uint32_t hi[4] = {0u, 0u, 0u, 0u}, lo[2] = {0u, 0u};
#pragma unroll
        for (int e = 0; e < 32; ++e) {
            int qi = 0;
            if (s > 0.0f) qi = (int)fminf(fmaxf(rintf(xs[e] / s), -31.0f), 31.0f);
            sq += (long long)(qi * qi);
            const double rr = (double)xs[e] - (double)s * (double)qi;   // exact in double
            se += rr * rr;
            sx += (double)xs[e] * (double)xs[e];
            const uint32_t h = (uint32_t)(qi >> 2) & 15u, l = (uint32_t)qi & 3u;
            hi[e >> 3] |= h << (4 * (e & 7));
            // dim e = 16w + n (n < 8) → bits 4n; e = 16w + 8 + n → bits 4n + 2
            lo[e >> 4] |= l << (4 * (e & 7) + 2 * ((e >> 3) & 1));
        }
        if (mine) {
            const int t = lane & 7, j = lane >> 3, g = (int)(r & 7);
            char* blk = out + (r >> 3) * (int64_t)(1536 * C);
            *reinterpret_cast<uint4*>(blk + j * 1024 + (g * 8 + t) * 16) = make_uint4(hi[0], hi[1], hi[2], hi[3]);
            *reinterpret_cast<uint2*>(blk + C * 1024 + j * 512 + (g * 8 + t) * 8) = make_uint2(lo[0], lo[1]);
        }
        for (int o = 32; o >= 1; o >>= 1) {
            sq += __shfl_xor(sq, o);
            se += __shfl_xor(se, o);
            sx += __shfl_xor(sx, o);
        }
        if (lane == 0) {
            const double A = (double)s * sqrt((double)sq) * (1.0 + 1e-12);
            const double B = sqrt(se) * (1.0 + 1e-12);
            aux[r] = make_float4(s, f32_round_up(A), f32_round_up(B), (float)sx);
        }
    }
}

hipError_t launch_sq6_quantize(const float4* x, int64_t n, int units, int dim, void* out, float4* aux, hipStream_t s) {
    const int C = sq6_chunks(dim);
    if (C < 1 || C > 8 || 4 * units > 256 * C) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(out, 0, (size_t)std::max<int64_t>(1, (n + 7) / 8) * 1536 * C, s);
    if (e != hipSuccess || n <= 0) return e;
    int64_t blocks = (n + 3) / 4;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(sq6_quantize, dim3((unsigned)blocks), dim3(kBlock), 0, s, x, n, units, C,
                       static_cast<char*>(out), aux);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// the three kernels of a 6-bit search (one query).  A scan row is 8 lanes; a wave takes 8 rows (one
// block) per row group and U groups per iteration (≈ U·4.6 KiB in flight per wave at C = 3); the row
// split per wave is sq8_scan's with R = 8, and each wave's list is list = tile·4 + wave.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int2 load_i2_nt(const int2* p) {
    typedef int i2v __attribute__((ext_vector_type(2)));
    const i2v v = __builtin_nontemporal_load(reinterpret_cast<const i2v*>(p));
    return make_int2(v.x, v.y);
}

// The k-th largest of the 64 lanes' values (k ≤ 64): each lane ranks its value against every lane's
// (ties by lane), read with v_readlane — no LDS round trips, unlike a shuffle sort.
__device__ __forceinline__ uint32_t wave_kth_largest(uint32_t v, int lane, int k) {
    int rank = 0;
#pragma unroll 4   // (16 kept 16 compare masks live in SGPRs and spilled the callers' scalars)
    for (int j = 0; j < 64; ++j) {
        const uint32_t o = (uint32_t)__builtin_amdgcn_readlane((int)v, j);
        rank += (o > v) || (o == v && j < lane);
    }
    const uint64_t hit = __ballot(rank == k - 1);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)__builtin_ctzll(hit));
}

// A lower bound of the exact score of a row whose raw device-order value is ≥ lo (dot kinds) or whose d²
// is ≤ hi (EUCLIDEAN), for the floor only (never returned), in float arithmetic: COSINE takes |x|² from
// the bound terms (Σx² in double, rounded) instead of the device-order norm the exact score divides by,
// so the norm is widened by g2 (≥ the device order's relative rounding) on the side that lowers the
// score, v_rsq's 1-ulp error and the few float roundings are covered by 2^-18, and the result is lowered
// by 2^-18 more (Java's double cosine and float transform are within an ulp or two of it).
__device__ __forceinline__ float floor_lb_score(int sim, float lo, float hi, float qnd, float xn_aux, float g2) {
    if (sim == SIM_EUCLIDEAN) return score_f32_l2(hi) * (1.0f - 0x1p-18f);
    if (sim != SIM_COSINE) return score_f32(sim, lo, qnd, 0.0f) * (1.0f - 0x1p-18f);
    const float xn = lo >= 0.0f ? xn_aux * (1.0f + g2) : xn_aux * (1.0f - g2);
    float c = lo * __builtin_amdgcn_rsqf(qnd * xn);
    c = c >= 0.0f ? c * (1.0f - 0x1p-18f) : c * (1.0f + 0x1p-18f);
    return fmaxf((1.0f + c) * 0.5f, 0.0f) * (1.0f - 0x1p-18f);
}

// Sampled int8 lower bounds seed the floor before the streaming pass: each wave scores the first 4 rows
// of its range (the 6-bit pass's split) on the int8 copy (16 lanes per row, exact device-order norms)
// and raises its floor bucket (list mod 64) to the best of them.
template <int C>
__global__ __launch_bounds__(kBlock) void sq6_pilot(Sq8Params p) {
    constexpr int R = 8;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform: scalar loop control
    const int cg = lane >> 4, ct = lane & 15;
    const int tix = p.tile_order[blockIdx.x];
    const TileDev tile = p.tiles[tix];
    const SegDev seg = p.segs[tile.seg];
    const int4* __restrict__ X8 = p.rows8[tile.seg];
    const int sim = p.sim, u8 = p.units8;
    const int64_t rows = tile.row_end - tile.row_begin;
    const int64_t per_wave = ((rows + 4 * R - 1) / (4 * R)) * R;
    const int64_t wb = tile.row_begin + wave * per_wave;
    const int64_t we = min(wb + per_wave, tile.row_end);
    const float4 qc = p.qc[0];
    const float qnd = sim == SIM_COSINE ? p.qn_dev[0] : 0.0f;
    // the first 4 rows of the wave's range (1 % of the rows), 16 lanes each (u8 ≤ 16·C units: C per lane)
    constexpr int H = 1;
    int4 xv[H][C], qv[C];
    float4 ax[H];
    float xnd[H] = {0.0f};
    bool v[H];
#pragma unroll
    for (int i = 0; i < C; ++i) qv[i] = ct + 16 * i < u8 ? p.q8[ct + 16 * i] : make_int4(0, 0, 0, 0);
#pragma unroll
    for (int h = 0; h < H; ++h) {
        const int64_t r = wb + 4 * h + cg;
        v[h] = r < we;
        const int64_t rc = v[h] ? r : tile.row_begin;
        const int4* xr = X8 + rc * u8;
#pragma unroll
        for (int i = 0; i < C; ++i) xv[h][i] = ct + 16 * i < u8 ? xr[ct + 16 * i] : make_int4(0, 0, 0, 0);
        ax[h] = p.aux[tile.seg][rc];
        if (sim == SIM_COSINE) xnd[h] = seg.xnorm_f[rc];
    }
    uint32_t best = 0u;
#pragma unroll
    for (int h = 0; h < H; ++h) {
        int a8 = 0;
#pragma unroll
        for (int i = 0; i < C; ++i) {
            a8 = __builtin_amdgcn_sdot4(xv[h][i].x, qv[i].x, a8, false);
            a8 = __builtin_amdgcn_sdot4(xv[h][i].y, qv[i].y, a8, false);
            a8 = __builtin_amdgcn_sdot4(xv[h][i].z, qv[i].z, a8, false);
            a8 = __builtin_amdgcn_sdot4(xv[h][i].w, qv[i].w, a8, false);
        }
        a8 = lane_sum<16>(a8);
        float lo, hi;
        sq8_bounds(sim, (float)a8, ax[h], qc, p.gam, p.g2, lo, hi);
        const float lb = sim == SIM_EUCLIDEAN ? score_f32_l2(hi) : score_f32(sim, lo, qnd, xnd[h]);
        if (v[h]) best = max(best, float_to_sortable(lb));
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) best = max(best, (uint32_t)__shfl_xor((int)best, o));
    uint32_t* fb = p.floor + ((size_t)p.q0 * p.n_shards + tile.shard) * (kFloorBuckets + 1) * kFloorStride;
    if (lane == 0 && best) atomicMax(fb + ((tix * 4 + wave) & (kFloorBuckets - 1)) * kFloorStride, best);
}

// A candidate's 6-bit test in one float, for the re-bound's re-test against the final floor's quick
// threshold tq (cand6_keep): the bound side itself (EUCLIDEAN: keep unless v > tq; dot kinds: unless v < tq),
// COSINE the side over √|x|² rounded up (keep unless v < tq: never stricter than the real-valued
// side ≥ tq·√|x|², which the quick threshold's slack covers like the scan's own test; a zero row keeps).
__device__ __forceinline__ float cand6_value(int sim, float side6, float sx) {
    if (sim != SIM_COSINE) return side6;
    if (!(sx > 0.0f)) return __builtin_inff();
    const float v = side6 / sx;
    return v + fmaxf(fabsf(v) * 0x1p-22f, 0x1p-126f);   // (≥ 2 ulps up: covers the division's rounding)
}
__device__ __forceinline__ bool cand6_keep(int sim, float v, float tq) {
    return sim == SIM_EUCLIDEAN ? !(v > tq) : !(v < tq);
}

// The streaming pass: 6-bit dot of every row, the 6-bit bound's upper side against the shard's floor,
// and the rows that pass appended to the wave's candidate buffer (cand6[list][cap6]: {row, its 6-bit test
// value (cand6_value)}, count in cnt6;
// cnt6 > cap6 = overflowed) for the int8 re-bound pass.  A row dropped here has ub6 < T ≤ the shard's
// k-th best exact score: it cannot enter the top k.  The best 6-bit lower bound among a wave's passing
// rows raises its floor bucket as the pass goes (a distinct row per bucket, as for the pilot's).
template <int C, int U>
__global__ __launch_bounds__(kBlock, 4) void sq6_scan(Sq8Params p) {   // ≤ 128 VGPRs: 4 waves/SIMD
    constexpr int R = 8;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform: scalar loop control
    const int t = lane & 7, g = lane >> 3;
    const int tix = p.tile_order[blockIdx.x];
    const TileDev tile = p.tiles[tix];
    const char* __restrict__ X6 = reinterpret_cast<const char*>(p.rows6[tile.seg]);
    const float4* __restrict__ AX6 = p.aux6[tile.seg];
    const int sim = p.sim;
#ifdef OSK_TESTING
    const int ablate = p.ablate;   // A/B timing only (results wrong): 1 no candidates, 2 no floor refresh, 4 no
                                   // candidate stores, 8 no 6-bit lower bounds, 16 no dots (loads only)
#else
    constexpr int ablate = 0;
#endif

    // the query's nibbles of this lane's half-chunks: bh[4] then bl[4] per j
    int qh[C][4], ql[C][4];
#pragma unroll
    for (int j = 0; j < C; ++j) {
        const int4 a = p.q6[(8 * j + t) * 2], b = p.q6[(8 * j + t) * 2 + 1];
        qh[j][0] = a.x; qh[j][1] = a.y; qh[j][2] = a.z; qh[j][3] = a.w;
        ql[j][0] = b.x; ql[j][1] = b.y; ql[j][2] = b.z; ql[j][3] = b.w;
    }
    const float4 qc6 = p.qc6[0];
    const float qnd0 = sim == SIM_COSINE ? p.qn_dev[0] : 0.0f;
    const float sqn0 = sqrtf(qnd0);

    const int64_t rows = tile.row_end - tile.row_begin;
    const int64_t per_wave = ((rows + 4 * R - 1) / (4 * R)) * R;
    const int64_t wb = tile.row_begin + wave * per_wave;   // a multiple of 8: tiles start at multiples of 16
    const int64_t we = min(wb + per_wave, tile.row_end);

    const int list = tix * 4 + wave;
    uint32_t* fb = p.floor + ((size_t)p.q0 * p.n_shards + tile.shard) * (kFloorBuckets + 1) * kFloorStride;
    uint2* cbuf = p.cand6 + (size_t)list * p.cap6;
    uint64_t fkey = 0ull;
    uint32_t best = 0u;
    float tq0 = sq8_quick(sim, 0ull, 0.0f, 0.0f);
    int nc = 0, it = 0;
    uint32_t* cell = fb + kFloorBuckets * kFloorStride;   // the shard's floor: max of the k-th values computed
    auto set_floor = [&](uint32_t f32) {
        uint64_t f = (uint64_t)f32 << 32;
        if (!(key_score(f) > 0.0f)) f = 0ull;
        if (f > fkey) {
            fkey = f;
            tq0 = sq8_quick(sim, fkey, sqn0, p.cos_slack);
        }
    };
    // k-th best of the buckets now (the pilot's and earlier tiles' bounds) → the cell and this wave
    auto recompute = [&](bool write) {
        const uint32_t v = __hip_atomic_load(fb + lane * kFloorStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t kth = wave_kth_largest(v, lane, p.k);
        if (write && kth > (uint32_t)(fkey >> 32) && lane == 0) atomicMax(cell, kth);
        set_floor(kth);
    };
    // at the start every wave computes the k-th itself but only one wave in 64 writes the cell: all of a
    // round's waves start together, and thousands of atomics on one address would queue for 100+ µs
    if (!(ablate & 2)) recompute((list & (kFloorBuckets - 1)) == 0);
    // then the cell is re-read every iteration for the first four, every fourth later (one load, issued
    // a refresh ahead).  A wave publishes its best lower bound to its bucket once, at its end, for the
    // later rounds of workgroups: publishing and re-ranking inside the loop (same-address atomics queue at
    // L2, and the ranking's registers spilled the loop's scalars) left the re-bound count unchanged at C3
    // and cost ≈ 10 % of the pass (profiles/r03c/sq6_ablate_r3.jsonl)
    uint32_t cv = __hip_atomic_load(cell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

    for (int64_t r0 = wb; r0 < we; r0 += R * U, ++it) {
        if ((it < 4 || (it & 3) == 0) && !(ablate & 2)) {
            set_floor(cv);
            cv = __hip_atomic_load(cell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        int4 hv[U][C];
        int2 lv[U][C];
        // unconditional loads from a clamped in-range block (masked after): see sq8_scan
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t gb = r0 + u * R;   // wave-uniform, 8-aligned
            const char* blk = X6 + ((gb < we ? gb : wb) >> 3) * (int64_t)(1536 * C);
#pragma unroll
            for (int j = 0; j < C; ++j) {
                hv[u][j] = load_i4_nt(reinterpret_cast<const int4*>(blk + j * 1024) + lane);
                lv[u][j] = load_i2_nt(reinterpret_cast<const int2*>(blk + C * 1024 + j * 512) + lane);
            }
        }
        // the tests run once per iteration, lane (g, t < U) on group t's row g (the U groups' sums are
        // gathered to those lanes below): one bound term load, one test and at most one candidate block
        // per iteration instead of U — their latency sits between this wave's loads
        const int64_t row = r0 + (int64_t)t * R + g;
        const bool valid = t < U && row < we;
        const float4 ax = AX6[valid ? row : wb];
        // every group's dot first, then the bounds and tests: the four v_dot8 chains of a group are serial
        // dependencies, and with the tests (ballot, branch) between groups the compiler could not overlap
        // one group's chains with the next one's (36 % of the wave cycles were issue stalls)
        int accu[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (ablate & 16) {   // loads only: the words folded, no dots
                int x = 0;
#pragma unroll
                for (int j = 0; j < C; ++j) x ^= hv[u][j].x ^ hv[u][j].y ^ hv[u][j].z ^ hv[u][j].w ^ lv[u][j].x ^ lv[u][j].y;
                accu[u] = x & 1;
                continue;
            }
            int hh[2] = {0, 0}, hl[2] = {0, 0}, lh[2] = {0, 0}, ll[2] = {0, 0};   // two chains each
#pragma unroll
            for (int j = 0; j < C; ++j) {
                const int hw[4] = {hv[u][j].x, hv[u][j].y, hv[u][j].z, hv[u][j].w};
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    hh[m & 1] = __builtin_amdgcn_sdot8(hw[m], qh[j][m], hh[m & 1], false);
                    hl[m & 1] = __builtin_amdgcn_sdot8(hw[m], ql[j][m], hl[m & 1], false);
                }
                const int lw[2] = {lv[u][j].x, lv[u][j].y};
#pragma unroll
                for (int w = 0; w < 2; ++w) {
                    const int a = lw[w] & 0x33333333, b = (int)(((uint32_t)lw[w] >> 2) & 0x33333333u);
                    lh[0] = __builtin_amdgcn_sdot8(a, qh[j][2 * w], lh[0], false);
                    lh[1] = __builtin_amdgcn_sdot8(b, qh[j][2 * w + 1], lh[1], false);
                    ll[0] = __builtin_amdgcn_sdot8(a, ql[j][2 * w], ll[0], false);
                    ll[1] = __builtin_amdgcn_sdot8(b, ql[j][2 * w + 1], ll[1], false);
                }
            }
            accu[u] = 64 * (hh[0] + hh[1]) + 4 * (hl[0] + hl[1]) + 16 * (lh[0] + lh[1]) + (ll[0] + ll[1]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) accu[u] = lane_sum<8>(accu[u]);
        int acc = accu[0];
#pragma unroll
        for (int u = 1; u < U; ++u) acc = t == u ? accu[u] : acc;
        const uint64_t vm = __ballot(valid);
        if (!vm) continue;
        const float sx = sim == SIM_COSINE ? __builtin_amdgcn_sqrtf(ax.w) : 0.0f;   // (1 ulp ≪ the quick test's slack)
        const float side6 = sq8_bound_side(sim, (float)acc, ax, qc6, p.gam, p.g2);
        const bool pass6 = valid && sq8_pass(sim, side6, side6, tq0, sx);
        const uint64_t pm = __ballot(pass6);
        if (!pm || (ablate & 1)) continue;   // wave-uniform: rare once the floor has risen
        // the passing rows (one lane per row) → the candidate buffer, and their 6-bit lower bounds
        const int slot = nc + __popcll(pm & ((1ull << lane) - 1ull));
        if (pass6) {
            if (slot < p.cap6 && !(ablate & 4)) {   // the row and its 6-bit test inputs (the re-bound re-tests)
                cbuf[slot] = make_uint2((uint32_t)row, __float_as_uint(cand6_value(sim, side6, sx)));
            }
            if (!(ablate & 8)) {
                float lo, hi;
                sq8_bounds(sim, (float)acc, ax, qc6, p.gam, p.g2, lo, hi);
                best = max(best, float_to_sortable(floor_lb_score(sim, lo, hi, qnd0, ax.w, p.g2)));
            }
        }
        nc += __popcll(pm);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) best = max(best, (uint32_t)__shfl_xor((int)best, o));
    if (lane == 0) {
        if (best > (uint32_t)(fkey >> 32)) atomicMax(fb + (list & (kFloorBuckets - 1)) * kFloorStride, best);
        p.cnt6[(size_t)p.q0 * p.n_lists + list] = nc;   // (visited rows and the re-bound counter: sq6_rebound)
    }
}

// The int8 re-bound pass.  Each list's candidates are first re-tested at the 6-bit level against the
// shard's FINAL floor (the scan tested them against the floor as it stood when their tile ran, lower for
// the tiles scanned first; sq8_pass is monotone in the threshold and the final floor is as valid as any
// earlier one), and only the survivors are gathered from the int8 copy: their int8 interval (sq8_bounds,
// exact device-order norms), sq8_scan's quick test and the list insertion; the list, its lower bounds and
// its best lower bound are written as sq8_scan writes them.  A list whose candidates overflowed the buffer
// gets a 16th key above every threshold, so the settle re-scans its rows exactly (its entries are then not
// re-scored).
//
// Persistent waves (round 5): W waves walk the list table, each with the NEXT list's descriptor — its tile,
// candidate count, and its first 64 candidates with their 6-bit test inputs, one per lane — loaded before
// the current list's rows, so a list costs one dependent round trip (its survivors' rows and bound terms).
// Assignment (p.rb_stride): contiguous (wave gw: lists [gw·per, (gw+1)·per)) or strided (lists gw, gw + W,
// …).  The shards' floors (≤ 64 shards) and the per-segment counts (≤ 64 segments) live in LDS, and the
// workgroup's counters leave with one global atomic each: same-address atomics queue at L2 (≈ 4 ns apiece;
// one per wave, 4,096 of them, cost ≈ 16 µs per launch, profiles/r05e/).
template <int C>
__global__ __launch_bounds__(kBlock) void sq6_rebound(Sq8Params p) {
    constexpr int kMaxLds = 64;
    __shared__ uint32_t s_floor[kMaxLds];
    __shared__ unsigned long long s_vis[kMaxLds], s_reb[kMaxLds];
    __shared__ unsigned long long s_tot[4];   // the workgroup's re-bounds, gathered rows (testing: passes, max clocks)
    __shared__ uint32_t s_sel[4][kSq6Cap];    // each wave's surviving candidates of its current list
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int cg = lane >> 4, ct = lane & 15;
    const int W = gridDim.x * 4, gw = blockIdx.x * 4 + wave;
    const bool strided = p.rb_stride != 0;
    const int per = (p.n_lists + W - 1) / W;
    const int l0 = strided ? gw : min(gw * per, p.n_lists);
    const int l1 = strided ? p.n_lists : min(l0 + per, p.n_lists);
    const int dl = strided ? W : 1;
    const int sim = p.sim, u8 = p.units8;
    const bool floor_lds = p.n_shards <= kMaxLds, seg_lds = p.n_segs <= kMaxLds;
    const float4 qc = p.qc[0];
    const float qnd0 = sim == SIM_COSINE ? p.qn_dev[0] : 0.0f;
    const float sqn0 = sqrtf(qnd0);
    int4 qv8[C];   // this lane's units of the int8 query
#pragma unroll
    for (int i = 0; i < C; ++i) qv8[i] = ct + 16 * i < u8 ? p.q8[ct + 16 * i] : make_int4(0, 0, 0, 0);
    const size_t cnt_base = (size_t)p.q0 * p.n_lists;
    auto shard_floor = [&](int shard) -> uint32_t {   // the k-th best bucket maximum, or the floor cell
        const uint32_t* fb = p.floor + ((size_t)p.q0 * p.n_shards + shard) * (kFloorBuckets + 1) * kFloorStride;
        return max(wave_kth_largest(fb[lane * kFloorStride], lane, p.k), fb[kFloorBuckets * kFloorStride]);
    };
    if (floor_lds)
        for (int s = wave; s < p.n_shards; s += 4) {
            const uint32_t f = shard_floor(s);
            if (lane == 0) s_floor[s] = f;
        }
    if (seg_lds)
        for (int i = threadIdx.x; i < kMaxLds; i += kBlock) s_vis[i] = 0ull, s_reb[i] = 0ull;
    if (threadIdx.x < 4) s_tot[threadIdx.x] = 0ull;
    __syncthreads();
    struct Desc {
        TileDev tile;
        int nc;
        uint2 c64;      // candidate `lane` (if < nc): {row, its 6-bit test value}
    };
    auto load_desc = [&](int list, Desc& d) {
        const int l = list < l1 ? list : l0;   // (clamped: a valid address, unused)
        d.tile = p.tiles[l >> 2];
        d.nc = p.cnt6[cnt_base + l];
        d.c64 = p.cand6[(size_t)l * p.cap6 + lane];
    };
    int cur_shard = -1, cur_seg = -1;
    uint64_t fkey = 0ull;
    float tqf = 0.0f;   // the final floor's quick threshold (the 6-bit re-test)
    const int4* X8 = nullptr;
    const float4* AX8 = nullptr;
    const float* XN = nullptr;
    uint32_t vbase = 0;
    unsigned long long vis = 0, reb = 0, reb_seg = 0, gathered = 0;   // (current segment's) visited rows, re-bounds
#ifdef OSK_TESTING
    unsigned long long n_pass = 0;
    const long long t_begin = clock64();
#endif
    auto flush_seg = [&]() {   // the current segment's counts: LDS, or (> 64 segments) one global atomic each
        if (cur_seg < 0 || lane != 0) return;
        if (seg_lds) {
            if (vis) atomicAdd(&s_vis[cur_seg], vis);
            if (reb_seg) atomicAdd(&s_reb[cur_seg], reb_seg);
        } else {
            if (p.visited && p.q0 == 0 && vis) atomicAdd(&p.visited[cur_seg], vis);
            if (p.seg_rebound && reb_seg) atomicAdd(&p.seg_rebound[cur_seg], reb_seg);
        }
    };
    uint32_t* sel = s_sel[wave];
    Desc dn;
    if (l0 < l1) load_desc(l0, dn);
    for (int list = l0; list < l1; list += dl) {
        const Desc d = dn;
        if (list + dl < l1) load_desc(list + dl, dn);
        TileDev tile = d.tile;   // (every lane loaded the same descriptor: keep it in SGPRs)
        tile.seg = __builtin_amdgcn_readfirstlane(tile.seg);
        tile.shard = __builtin_amdgcn_readfirstlane(tile.shard);
        const int nc = __builtin_amdgcn_readfirstlane(d.nc);
        if (tile.seg != cur_seg) {   // (wave-uniform) the segment's pointers; flush its counts
            flush_seg();
            vis = 0;
            reb_seg = 0;
            cur_seg = tile.seg;
            X8 = p.rows8[tile.seg];
            AX8 = p.aux[tile.seg];
            XN = p.segs[tile.seg].xnorm_f;
            vbase = (uint32_t)p.seg_vrow[tile.seg];
        }
        if (tile.shard != cur_shard) {   // the shard's final floor
            cur_shard = tile.shard;
            fkey = (uint64_t)(floor_lds ? s_floor[tile.shard] : shard_floor(tile.shard)) << 32;
            if (!(key_score(fkey) > 0.0f)) fkey = 0ull;
            tqf = sq8_quick(sim, fkey, sqn0, p.cos_slack);
        }
        if ((list & 3) == 0) vis += (unsigned long long)(tile.row_end - tile.row_begin);   // (each tile once)
        reb += (unsigned long long)nc;
        reb_seg += (unsigned long long)nc;
        uint64_t lk0 = 0ull, thr0 = 0ull;
        uint32_t lp0 = 0u;
        if (nc <= p.cap6) {
            // the 6-bit re-test against the final floor, survivors compacted into sel (64 candidates per
            // round; the first 64 came with the descriptor)
            int ns = 0;
            for (int c0 = 0; c0 < nc; c0 += 64) {
                uint2 c = d.c64;
                if (c0 > 0 && c0 + lane < nc) c = p.cand6[(size_t)list * p.cap6 + c0 + lane];
                const uint32_t r = c.x;
                const bool keep = c0 + lane < nc && (!p.rb_retest || cand6_keep(sim, __uint_as_float(c.y), tqf));
                const uint64_t km = __ballot(keep);
                if (keep)
                    sel[ns + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(km >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)km, 0u))] = r;
                ns += __popcll(km);
            }
            gathered += (unsigned long long)ns;
            float tq0 = tqf;
            // 8 survivors per pass (two halves of 4 rows × 16 lanes), every load of a pass issued before any
            // is used
            for (int c0 = 0; c0 < ns; c0 += 8) {
#ifdef OSK_TESTING
                ++n_pass;
#endif
                bool v[2];
                uint32_t r[2];
#pragma unroll
                for (int h = 0; h < 2; ++h) {   // (a slot past the count reads row 0: a valid address, masked after)
                    v[h] = c0 + 4 * h + cg < ns;
                    r[h] = v[h] ? sel[c0 + 4 * h + cg] : 0u;
                }
                int4 xv[2][C];
                float4 ax[2];
                float xnd[2] = {0.0f, 0.0f};
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int4* xr = X8 + (int64_t)r[h] * u8;
#pragma unroll
                    for (int i = 0; i < C; ++i) xv[h][i] = ct + 16 * i < u8 ? xr[ct + 16 * i] : make_int4(0, 0, 0, 0);
                    ax[h] = AX8[r[h]];
                    if (sim == SIM_COSINE) xnd[h] = XN[r[h]];
                }
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    int a8 = 0;
#pragma unroll
                    for (int i = 0; i < C; ++i) {
                        const int4 qv = qv8[i];
                        a8 = __builtin_amdgcn_sdot4(xv[h][i].x, qv.x, a8, false);
                        a8 = __builtin_amdgcn_sdot4(xv[h][i].y, qv.y, a8, false);
                        a8 = __builtin_amdgcn_sdot4(xv[h][i].z, qv.z, a8, false);
                        a8 = __builtin_amdgcn_sdot4(xv[h][i].w, qv.w, a8, false);
                    }
                    a8 = lane_sum<16>(a8);
                    float lo, hi;
                    sq8_bounds(sim, (float)a8, ax[h], qc, p.gam, p.g2, lo, hi);
                    const float sx = sim == SIM_COSINE ? __builtin_amdgcn_sqrtf(ax[h].w) : 0.0f;
                    const bool pass = v[h] && sq8_pass(sim, lo, hi, tq0, sx);
                    if (__ballot(pass && ct == 0)) {
                        const float ub = sim == SIM_EUCLIDEAN ? score_f32_l2(lo) : score_f32(sim, hi, qnd0, xnd[h]);
                        const float lb = sim == SIM_EUCLIDEAN ? score_f32_l2(hi) : score_f32(sim, lo, qnd0, xnd[h]);
                        const uint64_t key = pass ? make_key(ub, vbase + r[h]) : 0ull;
                        wave_offer2(key, float_to_sortable(lb), pass && ct == 0, lk0, lp0, thr0, lane, kKQ);
                        tq0 = sq8_quick(sim, max(thr0, fkey), sqn0, p.cos_slack);
                    }
                }
            }
        } else if (lane == kKQ - 1) {
            lk0 = ~0ull;   // overflowed: above every threshold → the settle re-scans the list's rows exactly
            lp0 = 0u;
        }
        uint32_t m = (lane < kKQ && lk0 && lk0 != ~0ull) ? lp0 : 0u;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
        const size_t l = cnt_base + list;
        if (lane < kKQ) {
            p.cand[l * kKQ + lane] = lk0;
            p.cand_lb[l * kKQ + lane] = lp0;
        }
        if (lane == 0) p.list_lbmax[l] = m;
    }
    flush_seg();
    // the workgroup's totals: reduced in LDS, then one global atomic each per workgroup
    if (lane == 0) {
        atomicAdd(&s_tot[0], reb);
        atomicAdd(&s_tot[1], gathered);
#ifdef OSK_TESTING
        atomicAdd(&s_tot[2], n_pass);
        atomicMax(&s_tot[3], (unsigned long long)(clock64() - t_begin));
#endif
    }
    __syncthreads();
    if (threadIdx.x == 0 && p.counters) {
        if (s_tot[0]) atomicAdd(&p.counters[3], s_tot[0]);
        if (s_tot[1]) atomicAdd(&p.counters[11], s_tot[1]);   // rows gathered from the int8 copy
#ifdef OSK_TESTING
        atomicAdd(&p.counters[12], s_tot[2]);   // 8-row passes
        atomicMax(&p.counters[13], s_tot[3]);   // the slowest workgroup's clocks
#endif
    }
    if (seg_lds)
        for (int i = threadIdx.x; i < p.n_segs; i += kBlock) {
            if (p.visited && p.q0 == 0 && s_vis[i]) atomicAdd(&p.visited[i], s_vis[i]);
            if (p.seg_rebound && s_reb[i]) atomicAdd(&p.seg_rebound[i], s_reb[i]);
        }
}

// row groups per wave-iteration by C: ≈ 12–14 KiB of loads in flight per wave
using Sq6Fn = void (*)(Sq8Params);
static const Sq6Fn kSq6[5] = {sq6_scan<2, 4>, sq6_scan<3, 3>, sq6_scan<4, 2>, sq6_scan<5, 1>, sq6_scan<6, 1>};
static const Sq6Fn kSq6Pilot[5] = {sq6_pilot<2>, sq6_pilot<3>, sq6_pilot<4>, sq6_pilot<5>, sq6_pilot<6>};
static const Sq6Fn kSq6Rebound[5] = {sq6_rebound<2>, sq6_rebound<3>, sq6_rebound<4>, sq6_rebound<5>, sq6_rebound<6>};

// pilot → streaming pass → int8 re-bound pass; the profiling events bracket the streaming pass, the
// dominant kernel whose roofline bench.py reports (the pilot and the re-bound read ≈ 2-3 % of its bytes)
hipError_t launch_sq6_scan(const Sq8Params& p, int dim, hipStream_t s, hipEvent_t ev_start, hipEvent_t ev_stop) {
    const int C = sq6_chunks(dim);
    if (C < 2 || C > 6 || p.q_count != 1 || p.k < 1 || p.k > kKQ || !p.floor || !p.q6 || !p.cand6 || !p.cnt6 ||
        !p.tile_order || p.cap6 < 64 || p.cap6 > kSq6Cap)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(kSq6Pilot[C - 2], dim3(p.n_tiles), dim3(kBlock), 0, s, p);
    const Sq6Fn scan = kSq6[C - 2];
    if (ev_start || ev_stop)
        hipExtLaunchKernelGGL(scan, dim3(p.n_tiles), dim3(kBlock), 0, s, ev_start, ev_stop, 0, p);
    else
        hipLaunchKernelGGL(scan, dim3(p.n_tiles), dim3(kBlock), 0, s, p);
    // the re-bound: persistent waves, a few lists each — as many workgroups per CU as fit at once (the
    // kernel's registers decide: 4 at ≤ 128 VGPRs), so no wave waits for another's lists to finish
    const Sq6Fn rb = kSq6Rebound[C - 2];
    static std::atomic<int> s_fit[5];   // (zero-initialised; the same value from every thread)
    std::atomic<int>& fit_of = s_fit[C - 2];
    int fit = fit_of.load(std::memory_order_relaxed);
    if (fit == 0) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(rb), kBlock, 0) != hipSuccess ||
            n < 1)
            n = 1;
        fit = std::min(n, 8);
        fit_of.store(fit, std::memory_order_relaxed);
    }
    const int per_cu = p.rb_wg_per_cu > 0 ? p.rb_wg_per_cu : fit;
    const int rb_grid = std::max(1, std::min(p.n_tiles, per_cu * (p.wide_grid > 0 ? p.wide_grid : 256)));
    hipLaunchKernelGGL(rb, dim3(rb_grid), dim3(kBlock), 0, s, p);
    return hipGetLastError();
}

}  // namespace osk
