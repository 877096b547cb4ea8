// osk_mfma.hip — batched exact k-NN (batch ≥ 16): MFMA candidate pass + exact re-score + certificate.
//
// Why: at batch B the scan is B dot products per corpus byte; past ~4 queries the VALU streaming
// kernel stops being HBM-bound.  Here the contraction Q×Xᵀ runs on CDNA4 bf16 MFMA
// (v_mfma_f32_16x16x32_bf16) with every fp32 operand split into bf16 hi + lo parts and three
// products (hi·hi + hi·lo + lo·hi, ≈2^-16 relative), LDS-tiled (128 rows × 256 queries per
// workgroup, LDS-DMA double-buffered K-steps of 32 dims).
//
// Exactness: the MFMA scores are only used to pick k' = kKC candidates per (query, shard).  The
// candidates are re-scored with the streaming kernel's arithmetic (identical bits),
// and a per-(query, shard) certificate proves no non-candidate can enter the top k:
//     exact k-th score  >  U = T(approx score of the k'-th candidate, + the error bound)
// where the bound covers the split, the fp32 accumulation and the device-order rounding
// (|Σ approx − Σ device| ≤ c·|x|·|q|, c from Kpad).  A query whose certificate fails for any shard
// is recomputed by the exact streaming scan.  Results are therefore bit-identical to the
// streaming path (and to the ORDER_DEVICE oracle) — asserted by tests/test_gpu_parity.py.
#include "osk_internal.h"
#include "osk_wave.h"

namespace osk {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t bf16_rne_bits(float x) {
    uint32_t u = __float_as_uint(x);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return u >> 16;
}

// ------------------------------------------------------------------------------------------------
// fp32 rows (padded units) → fragment-ordered bf16 hi/lo copy.
// Block (rb, ks, part) is 1 KiB: lane l holds row rb·16 + (l&15), dims ks·32 + 8(l>>4) … +7.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void split_rows(const float4* __restrict__ X, int64_t n_rows,
                                                     int units, int KS, int64_t n_rb,
                                                     uint4* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t wave_global = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) >> 6;
    for (int64_t blk = wave_global; blk < n_rb * KS; blk += n_waves) {
        const int64_t rb = blk / KS;
        const int ks = (int)(blk % KS);
        const int64_t row = rb * 16 + (lane & 15);
        const int f0 = ks * 8 + 2 * (lane >> 4);
        float v[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
            if (row < n_rows && f0 + h < units) x = X[row * units + f0 + h];
            v[4 * h + 0] = x.x; v[4 * h + 1] = x.y; v[4 * h + 2] = x.z; v[4 * h + 3] = x.w;
        }
        uint32_t hi[8], lo[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            hi[j] = bf16_rne_bits(v[j]);
            const float r = v[j] - __uint_as_float(hi[j] << 16);
            lo[j] = bf16_rne_bits(r);
        }
        uint4 H = make_uint4(hi[0] | (hi[1] << 16), hi[2] | (hi[3] << 16), hi[4] | (hi[5] << 16), hi[6] | (hi[7] << 16));
        uint4 Lo = make_uint4(lo[0] | (lo[1] << 16), lo[2] | (lo[3] << 16), lo[4] | (lo[5] << 16), lo[6] | (lo[7] << 16));
        out[(blk * 2 + 0) * 64 + lane] = H;
        out[(blk * 2 + 1) * 64 + lane] = Lo;
    }
}

hipError_t launch_split_rows(const float4* rows, int64_t n_rows, int units, int KS, int64_t n_rb,
                             void* out, hipStream_t s) {
    int64_t blocks = (n_rb * KS + 3) / 4;
    if (blocks < 1) blocks = 1;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(split_rows, dim3((unsigned)blocks), dim3(kBlock), 0, s, rows, n_rows, units, KS,
                       n_rb, static_cast<uint4*>(out));
    return hipGetLastError();
}

// max over rows of |x|² (float bits compare as ints for non-negative floats)
__global__ __launch_bounds__(kBlock) void max_norm2(const float* __restrict__ xn, int64_t n,
                                                    unsigned* __restrict__ out) {
    float m = 0.0f;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
        m = fmaxf(m, xn[i]);
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) atomicMax(out, __float_as_uint(m));
}

// |x| per row (the cosine bound of the candidate epilogue)
__global__ __launch_bounds__(kBlock) void row_sqrt(const float* __restrict__ xn, int64_t n, float* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
        out[i] = sqrtf(xn[i]);
}

hipError_t launch_row_sqrt(const float* xn, int64_t n, float* out, hipStream_t s) {
    int64_t blocks = (n + kBlock - 1) / kBlock;
    if (blocks < 1) blocks = 1;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(row_sqrt, dim3((unsigned)blocks), dim3(kBlock), 0, s, xn, n, out);
    return hipGetLastError();
}

hipError_t launch_max_norm2(const float* xn, int64_t n, unsigned* out, hipStream_t s) {
    int64_t blocks = (n + kBlock - 1) / kBlock;
    if (blocks < 1) blocks = 1;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(max_norm2, dim3((unsigned)blocks), dim3(kBlock), 0, s, xn, n, out);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// candidate pass: 8 waves, 128 rows × 256 queries per tile, K-steps of 32 dims.
//
// Wave w owns queries w·32 … +31 of the block against all 128 rows of the tile (acc: 8 row
// blocks × 2 query blocks of 16×16).  Its query fragments (hi/lo, 4 KiB per K-step) are private:
// they stream from L2 straight into a register ring kDepth K-steps deep.  The corpus fragments
// (16 KiB per K-step, shared by all waves) stream by LDS-DMA into a (kDepth+1)-slot LDS ring.
// The (tile, K-step) sequence of a unit is one flat stream of steps, so the pipeline stays full
// across tile boundaries.
// ------------------------------------------------------------------------------------------------
constexpr int kMB = 512;                        // threads per workgroup
constexpr int kDepth = kKsAlign;                // K-steps in flight (KS is a multiple of it)
constexpr int kStageA = 16 * 1024;              // 8 row blocks × hi/lo × 1 KiB
constexpr int kRing = (kDepth + 1) * kStageA;   // 80 KiB
constexpr int kStagePitch = 260;                // fp32 per staged score row (bank-conflict-free writes)
constexpr int kOffStaged = kRing;               // 64 rows × 260 fp32 (half a tile) = 65 KiB
constexpr int kStaging = 64 * kStagePitch * 4;

// wait until at most `steps` K-steps of this wave's loads (6 VMEM ops each) are in flight
// (`steps` is a compile-time constant after unrolling; the switch folds away)
__device__ __forceinline__ void vm_wait_steps(int steps) {
    switch (steps) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    }
}

// LDS-DMA: 16 B (or 4 B) per lane from a per-lane global address to lds_base + lane·size.
// AUX = 2: non-temporal (the corpus copy streams through once and must not evict the queries,
// which every workgroup re-reads from L2 each tile).
template <int AUX = 0>
__device__ __forceinline__ void glds16(const void* g, char* lds_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)lds_base, 16, 0, AUX);
}
__device__ __forceinline__ void glds4(const void* g, char* lds_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)lds_base, 4, 0, 0);
}

__device__ __forceinline__ float approx_score(int sim, float d, float qn, float xn) {
    switch (sim) {
        case SIM_EUCLIDEAN: {
            const float d2 = fmaxf(xn + qn - 2.0f * d, 0.0f);
            return 1.0f / (1.0f + d2);
        }
        case SIM_DOT_PRODUCT: return (1.0f + d) * 0.5f;
        case SIM_COSINE: return (1.0f + d * rsqrtf(qn * xn)) * 0.5f;
        default: return d < 0.0f ? 1.0f / (1.0f - d) : d + 1.0f;
    }
}

// LDS beyond the ring and the staging: per-query survivor slots of the MAIN epilogue
constexpr int kSlots = 4;                              // survivors per query per tile before overflow
constexpr int kOffXn = kOffStaged + kStaging;          // f32 [2][|x|², |x|][128] of the tile (by tile parity)
constexpr int kOffThr = kOffXn + 2 * 256 * 4;          // u32 [256] sortable score thresholds
constexpr int kOffCnt = kOffThr + 256 * 4;             // i32 [256] survivor counts
constexpr int kOffSlot = kOffCnt + 256 * 4;            // u64 [256][kSlots] survivor keys
constexpr int kOffOvf = kOffSlot + 256 * kSlots * 8;   // i32 overflow flag
constexpr int kLdsTotal = kOffOvf + 16;
static_assert(kLdsTotal <= 160 * 1024, "LDS budget");

__device__ __forceinline__ void list_insert(uint64_t (&lst)[kKC], uint64_t key) {
    if (key > lst[kKC - 1]) {
        uint64_t cur = key;
#pragma unroll
        for (int i = 0; i < kKC; ++i) {
            const uint64_t a = lst[i];
            const bool gt = cur > a;
            lst[i] = gt ? cur : a;
            cur = gt ? a : cur;
        }
    }
}

// PILOT = true: only the first tile of each unit, every score staged (the lists it leaves are
// merged per (query, shard) into the thresholds of the main pass).
// SIM is compile-time: with the similarity a runtime value every unrolled scoring site carried all
// four transforms (260 IEEE divisions, 17k instructions in one kernel: more than the instruction cache
// holds, so the epilogue's rare paths missed it on every tile).
template <bool PILOT, int SIM>
__global__ __launch_bounds__(kMB) void mfma_cand(MfmaParams p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* staged = reinterpret_cast<float*>(smem + kOffStaged);
    uint32_t* s_thr = reinterpret_cast<uint32_t*>(smem + kOffThr);
    int* s_cnt = reinterpret_cast<int*>(smem + kOffCnt);
    uint64_t* s_slot = reinterpret_cast<uint64_t*>(smem + kOffSlot);
    int* s_ovf = reinterpret_cast<int*>(smem + kOffOvf);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform → scalar addressing
    const MfmaUnit unit = p.units[blockIdx.x];
    const SegDev seg = p.segs[unit.seg];
    const char* __restrict__ A = static_cast<const char*>(p.seg_split[unit.seg]);
    const int qblock = blockIdx.y;
    const int KS = p.KS;
    constexpr int sim = SIM;
    // this wave's two 16-query blocks, fragment-ordered [qb][ks][hi/lo][64 lanes][16 B]
    const char* __restrict__ Bw = static_cast<const char*>(p.qsplit) +
                                  (size_t)(qblock * 16 + wave * 2) * KS * 2048 + lane * 16;
    const size_t Bqb = (size_t)KS * 2048;   // bytes per query block
    const uint64_t* abits = p.accept ? p.accept[unit.seg] : nullptr;

    // thread-side selection state: thread ↔ (query q_sel of this block, row half h_sel)
    const int q_sel = tid & 255, h_sel = tid >> 8;
    uint64_t lst[kKC];
#pragma unroll
    for (int i = 0; i < kKC; ++i) lst[i] = 0ull;
    uint32_t nvis = 0;
    if (h_sel == 0) {
        // initial threshold: k'-th approx score of the pilot tiles of this (query, shard), else none
        uint32_t t0 = 0u;
        const int qg = qblock * 256 + q_sel;
        if (!PILOT && p.thr_keys && qg < p.nq) {
            const size_t o = (size_t)qg * p.n_shards + unit.shard;
            if (p.thr_counts[o] >= kKC) t0 = (uint32_t)(p.thr_keys[o * kKC + kKC - 1] >> 32);
        }
        s_thr[q_sel] = t0;
        s_cnt[q_sel] = 0;
    }
    if (tid == 0) s_ovf[0] = 0;

    // this lane's queries / norms in the MFMA layout: q_local = wave·32 + j·16 + (lane & 15)
    float qn_l[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int qg = qblock * 256 + wave * 32 + j * 16 + (lane & 15);
        qn_l[j] = qg < p.nq_pad ? p.qnorm[qg] : 1.0f;
    }

    const int64_t tile_last = PILOT ? unit.tile_begin : unit.tile_end - 1;
    const int lane16 = lane * 16;
    // corpus fragments of (tile, k-step ks) → ring slot `slot` (this wave's 2 of the 16 chunks)
    auto issue_a = [&](int64_t tile, int ks, int slot) {
        if (p.ablate & 4) return;
        const char* src = A + ((size_t)tile * 8 * KS + ks) * 2048 + lane16;
        char* dst = smem + slot * kStageA;
#pragma unroll
        for (int c2 = 0; c2 < 2; ++c2) {
            const int c = wave * 2 + c2;               // chunk = (row block c >> 1, hi/lo c & 1)
            glds16<2>(src + ((size_t)(c >> 1) * KS * 2 + (c & 1)) * 1024, dst + c * 1024);
        }
        if (ks == 0 && wave < 4) {   // the tile's |x|² and |x| ride along with its first K-step
            const int64_t row = min(tile * 128 + (wave & 1) * 64 + lane, seg.n_rows - 1);
            glds4((wave < 2 ? seg.xnorm_f : p.xsqrt[unit.seg]) + row,
                  smem + kOffXn + (int)(tile & 1) * 1024 + wave * 256);
        }
    };
    bf16x8 bq[kDepth][4];   // register ring: [slot][qb0 hi, qb0 lo, qb1 hi, qb1 lo]
    auto issue_b = [&](int ks, bf16x8 (&r)[4]) {
        if (p.ablate & 2) return;
        const char* src = Bw + (size_t)ks * 2048;
        r[0] = *reinterpret_cast<const bf16x8*>(src);
        r[1] = *reinterpret_cast<const bf16x8*>(src + 1024);
        r[2] = *reinterpret_cast<const bf16x8*>(src + Bqb);
        r[3] = *reinterpret_cast<const bf16x8*>(src + Bqb + 1024);
    };
#pragma unroll
    for (int u = 0; u < kDepth; ++u) {
        if (p.ablate & 2) {
#pragma unroll
            for (int x = 0; x < 4; ++x) bq[u][x] = bf16x8{};
        }
        issue_a(unit.tile_begin, u, u);
        issue_b(u, bq[u]);
    }

    f32x4 acc[8][2];
    int slot = 0;   // ring slot of the current step; step + kDepth goes to slot − 1 (mod kDepth + 1)
    for (int64_t tile = unit.tile_begin; tile <= tile_last; ++tile) {
        const int64_t tile_rb0 = tile * 8;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

        for (int ks0 = 0; ks0 < KS; ks0 += kDepth) {
            // the step kDepth ahead: same tile, or (KS multiple of kDepth) the next tile's k-step u
            const bool wrap = ks0 + kDepth >= KS;
            const int64_t tile_n = wrap ? tile + 1 : tile;
            const int ks_n0 = wrap ? 0 : ks0 + kDepth;
            const bool more = tile_n <= tile_last;
#pragma unroll
            for (int u = 0; u < kDepth; ++u) {
                // own DMA + query loads of this step done (later steps stay in flight), then every
                // wave's; past the barrier no wave still reads the previous step's slot
                vm_wait_steps(more ? kDepth - 1 : kDepth - 1 - u);
                __builtin_amdgcn_s_barrier();
                const char* sA = smem + slot * kStageA + lane16;
                const int slot_n = slot == 0 ? kDepth : slot - 1;
                if (more) issue_a(tile_n, ks_n0 + u, slot_n);
                const bf16x8 b0h = bq[u][0], b0l = bq[u][1], b1h = bq[u][2], b1l = bq[u][3];
#pragma unroll
                for (int i = 0; i < 8; i += 2) {
                    const bf16x8 ah0 = *reinterpret_cast<const bf16x8*>(sA + (i * 2 + 0) * 1024);
                    const bf16x8 al0 = *reinterpret_cast<const bf16x8*>(sA + (i * 2 + 1) * 1024);
                    const bf16x8 ah1 = *reinterpret_cast<const bf16x8*>(sA + (i * 2 + 2) * 1024);
                    const bf16x8 al1 = *reinterpret_cast<const bf16x8*>(sA + (i * 2 + 3) * 1024);
                    // three sweeps over 4 accumulators: consecutive MFMAs never share one
                    acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah0, b0h, acc[i][0], 0, 0, 0);
                    acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah0, b1h, acc[i][1], 0, 0, 0);
                    acc[i + 1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah1, b0h, acc[i + 1][0], 0, 0, 0);
                    acc[i + 1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah1, b1h, acc[i + 1][1], 0, 0, 0);
                    acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah0, b0l, acc[i][0], 0, 0, 0);
                    acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah0, b1l, acc[i][1], 0, 0, 0);
                    acc[i + 1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah1, b0l, acc[i + 1][0], 0, 0, 0);
                    acc[i + 1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah1, b1l, acc[i + 1][1], 0, 0, 0);
                    acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al0, b0h, acc[i][0], 0, 0, 0);
                    acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al0, b1h, acc[i][1], 0, 0, 0);
                    acc[i + 1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al1, b0h, acc[i + 1][0], 0, 0, 0);
                    acc[i + 1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al1, b1h, acc[i + 1][1], 0, 0, 0);
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this step's slot reads retired
                if (more) issue_b(ks_n0 + u, bq[u]);
                slot = slot == kDepth ? 0 : slot + 1;
            }
        }

        // visited: accepted rows of the tile, counted once (query block 0, one thread per row)
        if (!PILOT && p.visited && qblock == 0 && tid < 128) {
            const int64_t row = tile_rb0 * 16 + tid;
            bool ok = row < seg.n_rows;
            if (ok && abits) {
                const int32_t doc = seg.ord_to_doc ? seg.ord_to_doc[row] : (int32_t)row;
                ok = (abits[doc >> 6] >> (doc & 63)) & 1ull;
            }
            nvis += ok ? 1u : 0u;
        }
        if (p.ablate & 1) {   // A/B: no epilogue at all (the accumulators stay live)
            float sink = 0.f;
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) sink += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
            if (sink == 12345.678f) lst[0] = 1;
            continue;
        }

        // ---- epilogue (uses only the staging / slot LDS: the ring keeps streaming) ----
        const float* xs = reinterpret_cast<const float*>(smem + kOffXn + (int)(tile & 1) * 1024);
        const float* xr = xs + 128;   // |x|
        // MAIN: every accumulator is scored in registers and compared with its query's threshold
        // (pilot k'-th score, raised as the lists fill); the few survivors go to kSlots LDS slots
        // per query and the query's owner thread merges them into its list.  A tile where some
        // query has more survivors than slots takes the full path below instead (its
        // accumulators are still live).
        // PILOT and overflow: the scores are staged in LDS half a tile at a time and every
        // (query, row quarter) thread offers its 32 rows of the half to its list.
        bool full = PILOT || (p.ablate & 8);
        if (!full) {
            // Per query a bound equivalent to "approx score ≥ threshold" in the dot domain, loosened by
            // 2^-16·max(1, |t|) (far above the rounding of either form), evaluated branch-free as
            //   α·d − β·v_row ≥ γ_q:
            //   COSINE      α = 1, β = cq_q, v = |x|, γ = 0              (d ≥ cq·|x|)
            //   DOT / MIP   α = 1, β = 0, γ = cq_q                       (d ≥ cq)
            //   EUCLIDEAN   α = 2, β = 1 − 2^-18, v = |x|², γ = |q|² − D − 2^-18·(|q|² + D), D = 1/tm − 1
            //               (1/(1 + max(|x|² + |q|² − 2d, 0)) ≥ tm ⟸ 2d − |x|² ≥ |q|² − D; the 2^-18 terms
            //               cover the float rounding of both sides, 2|d| ≤ |x|² + |q|²)
            // Only a row block (8 pairs per lane) with a passing lane in the wave runs the exact approx
            // score and the real test; the per-pair branches of that path cost 0.36 of the 0.66 ms of a C2
            // b256 search when every pair took them (EUCLIDEAN had no quick test).
            uint32_t thr_l[2];
            float be[2], ga[2];
            const bool cosine = sim == SIM_COSINE, l2 = sim == SIM_EUCLIDEAN;
            const float al = l2 ? 2.0f : 1.0f;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                thr_l[j] = s_thr[wave * 32 + j * 16 + (lane & 15)];
                const float t = sortable_to_float(thr_l[j]);
                // EUCLIDEAN scores 1/(1 + d²) are tiny at large d² (≈ 3e-6 on C2's SIFT-like rows): an
                // absolute 2^-16 slack made tm negative and let every pair through to the exact test
                // (half of all (row, query) pairs: 0.37 of 0.71 ms at C2 b256), so its slack is relative
                const float tm = l2 ? t * (1.0f - 0x1p-16f) : t - 0x1p-16f * fmaxf(1.0f, fabsf(t));
                float c = -__builtin_inff();
                if (thr_l[j] != 0u) {
                    if (sim == SIM_COSINE) c = (2.0f * tm - 1.0f) * sqrtf(qn_l[j]);
                    else if (sim == SIM_DOT_PRODUCT) c = 2.0f * tm - 1.0f;
                    else if (sim == SIM_MIP && tm > 0.0f) c = tm >= 1.0f ? tm - 1.0f : 1.0f - 1.0f / tm;
                    else if (l2 && tm > 0.0f) {
                        const float D = 1.0f / tm - 1.0f, qn = qn_l[j];
                        c = (qn - D) - 0x1p-18f * (fabsf(qn) + fabsf(D));
                    }
                }
                // padded query columns (batch not a multiple of 256) have no threshold: without this
                // every one of their accumulators would pass, overflow the slots and send every
                // tile down the full path (C2 b128: 1.18 ms against 0.65 at b256)
                const int qg = qblock * 256 + wave * 32 + j * 16 + (lane & 15);
                c = qg < p.nq ? c : __builtin_inff();
                if (cosine) {   // d − c·|x| ≥ 0; ±∞ (no threshold / padded column): always / never
                    const bool fin = c > -__builtin_inff() && c < __builtin_inff();
                    be[j] = fin ? c : 0.0f;
                    ga[j] = fin ? 0.0f : c;
                } else {
                    be[j] = l2 ? 1.0f - 0x1p-18f : 0.0f;
                    ga[j] = c;
                }
            }
            const float* vrow = cosine ? xr : xs;
            uint32_t mh[2] = {0u, 0u};   // pass masks per half tile: bit (i & 3)·8 + r·2 + j
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (p.ablate & 32) break;   // A/B: no quick tests
                const int rl0 = i * 16 + (lane >> 4) * 4;
                const float4 v4 = (cosine || l2) ? *reinterpret_cast<const float4*>(vrow + rl0)
                                                 : make_float4(0.f, 0.f, 0.f, 0.f);
                const float vr[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const float lhs = fmaf(al, acc[i][j][r], -be[j] * vr[r]);
                        mh[i >> 2] |= !(lhs < ga[j]) ? (1u << ((i & 3) * 8 + r * 2 + j)) : 0u;   // (NaN passes)
                    }
            }
            // the pairs that pass: this wave stages its own 32 query columns of the half tile in LDS (no
            // other wave touches them, so no barrier) and each lane walks its own passing pairs in a
            // rolled loop — one copy of the exact test and the slot insertion instead of 64 unrolled
            // ones (the kernel outgrew the instruction cache)
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                if (p.ablate & 128) {   // A/B: quick tests only (results wrong)
                    if (mh[half] == 0xFFFFFFFFu) s_ovf[1] = 1;
                    continue;
                }
                if (!__ballot(mh[half] != 0u)) continue;   // wave-uniform

#pragma unroll
                for (int i = half * 4; i < half * 4 + 4; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int j = 0; j < 2; ++j)
                            staged[(i * 16 + (lane >> 4) * 4 + r - half * 64) * kStagePitch + wave * 32 + j * 16 + (lane & 15)] =
                                acc[i][j][r];
                for (uint32_t m = mh[half]; m; m &= m - 1u) {
                    const int e = __builtin_ctz(m);
                    const int i = half * 4 + (e >> 3), r = (e >> 1) & 3, j = e & 1;
                    const int row_local = i * 16 + (lane >> 4) * 4 + r;
                    const int ql = wave * 32 + j * 16 + (lane & 15);
                    const int64_t row = tile_rb0 * 16 + row_local;
                    if (row >= seg.n_rows) continue;
                    const float d = staged[(row_local - half * 64) * kStagePitch + ql];
                    const float sc = approx_score(sim, d, j ? qn_l[1] : qn_l[0], xs[row_local]);
                    if (float_to_sortable(sc) < (j ? thr_l[1] : thr_l[0])) continue;
                    if (abits) {
                        const int32_t doc = seg.ord_to_doc ? seg.ord_to_doc[row] : (int32_t)row;
                        if (!((abits[doc >> 6] >> (doc & 63)) & 1ull)) continue;
                    }
                    const int slot = atomicAdd(&s_cnt[ql], 1);
                    if (slot < kSlots) s_slot[ql * kSlots + slot] = make_key(sc, (uint32_t)(unit.vrow_base + row));
                    else s_ovf[0] = 1;
                }
            }
            if (p.ablate & 64) continue;   // A/B: no merge (results wrong)
            __syncthreads();
            full = s_ovf[0] != 0;   // uniform
            if (h_sel == 0) {
                if (!full) {
                    const int n = min(s_cnt[q_sel], kSlots);
                    for (int e = 0; e < n; ++e) list_insert(lst, s_slot[q_sel * kSlots + e]);
                    if (lst[kKC - 1]) atomicMax(&s_thr[q_sel], (uint32_t)(lst[kKC - 1] >> 32));
                }
                s_cnt[q_sel] = 0;
            }
            __syncthreads();        // every thread has read s_ovf
            if (tid == 0) s_ovf[0] = 0;
        }
        if (full) {
            if (!PILOT && p.full_tiles && tid == 0) atomicAdd(p.full_tiles, 1ull);
#pragma unroll
            for (int half = 0; half < 2; ++half) {
#pragma unroll
                for (int i = half * 4; i < half * 4 + 4; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int row_local = i * 16 + (lane >> 4) * 4 + r;
                        const int64_t row = tile_rb0 * 16 + row_local;
                        const bool rv = row < seg.n_rows;
                        const float xn = rv ? xs[row_local] : 1.0f;
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            const int ql = wave * 32 + j * 16 + (lane & 15);
                            staged[(row_local - half * 64) * kStagePitch + ql] =
                                rv && qblock * 256 + ql < p.nq ? approx_score(sim, acc[i][j][r], qn_l[j], xn)
                                                               : -__builtin_inff();
                        }
                    }
                __syncthreads();
#pragma unroll 2
                for (int rr = 0; rr < 32; ++rr) {
                    const int row_half = h_sel * 32 + rr;
                    const int64_t ord = tile_rb0 * 16 + half * 64 + row_half;
                    const float s = staged[row_half * kStagePitch + q_sel];
                    if (!(s > -__builtin_inff())) continue;
                    if (abits) {
                        const int32_t doc = seg.ord_to_doc ? seg.ord_to_doc[ord] : (int32_t)ord;
                        if (!((abits[doc >> 6] >> (doc & 63)) & 1ull)) continue;
                    }
                    list_insert(lst, make_key(s, (uint32_t)(unit.vrow_base + ord)));
                }
                __syncthreads();
            }
            if (!PILOT && lst[kKC - 1]) atomicMax(&s_thr[q_sel], (uint32_t)(lst[kKC - 1] >> 32));
            __syncthreads();
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may outlive the workgroup

    const int qg = qblock * 256 + q_sel;
    if (qg < p.nq) {
        uint64_t* o = p.cand + ((size_t)qg * p.n_units * 2 + (size_t)blockIdx.x * 2 + h_sel) * kKC;
#pragma unroll
        for (int i = 0; i < kKC; ++i) o[i] = lst[i];
    }
    if (!PILOT && p.visited && qblock == 0 && tid < 128 && nvis)
        atomicAdd(&p.visited[unit.seg], (unsigned long long)nvis);
}

using MfmaCandFn = void (*)(MfmaParams);
static const MfmaCandFn kMfmaCand[2][4] = {
    {mfma_cand<false, 0>, mfma_cand<false, 1>, mfma_cand<false, 2>, mfma_cand<false, 3>},
    {mfma_cand<true, 0>, mfma_cand<true, 1>, mfma_cand<true, 2>, mfma_cand<true, 3>}};

hipError_t launch_mfma_cand(const MfmaParams& p, int n_qblocks, bool pilot, hipStream_t s) {
    if (p.KS % kDepth != 0 || p.sim < 0 || p.sim > 3) return hipErrorInvalidValue;
    static bool attr_set = false;
    if (!attr_set) {
        for (int pl = 0; pl < 2; ++pl)
            for (int sm = 0; sm < 4; ++sm) {
                const hipError_t e = hipFuncSetAttribute((const void*)kMfmaCand[pl][sm],
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, kLdsTotal);
                if (e != hipSuccess) return e;
            }
        attr_set = true;
    }
    hipLaunchKernelGGL(kMfmaCand[pilot ? 1 : 0][p.sim], dim3(p.n_units, n_qblocks), dim3(kMB), kLdsTotal, s, p);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// exact re-score of the k' candidates of one (shard, query) + certificate (one wave each)
// ------------------------------------------------------------------------------------------------
template <int L, int V, bool L2K>
__global__ __launch_bounds__(64) void rescore(RescoreParams p) {
    constexpr int R = 64 / L;
    constexpr int UP = L * V;
    const int s = blockIdx.x, q = blockIdx.y, S = p.n_shards;
    const int lane = threadIdx.x, t = lane & (L - 1), g = lane / L;
    const size_t o = (size_t)q * S + s;
    const uint64_t akey = lane < kKC ? p.akeys[o * kKC + lane] : 0ull;
    const int nc = __popcll(__ballot(akey != 0ull));
    const float4* __restrict__ Q = reinterpret_cast<const float4*>(p.q) + (size_t)q * UP;
    float4 qf[V];
#pragma unroll
    for (int j = 0; j < V; ++j) qf[j] = Q[t + j * L];
    const float qn = p.qnorm_dev ? p.qnorm_dev[q] : 0.0f;
    const int k = p.k, sim = p.sim;
    uint64_t lk = 0ull, thr = 0ull;
    const uint32_t alo = (uint32_t)akey;
    for (int i0 = 0; i0 < nc; i0 += R) {
        const int ci = i0 + g;
        const bool valid = ci < nc;
        const uint32_t vrow = 0xFFFFFFFFu - (uint32_t)__shfl((int)alo, valid ? ci : 0);
        int sg = 0;
        for (int j = 1; j < p.n_segs; ++j)
            if ((int64_t)vrow >= p.seg_vrow_begin[j]) sg = j;
        const SegDev seg = p.segs[sg];
        const int64_t ord = (int64_t)vrow - p.seg_vrow_begin[sg];
        const int32_t doc = seg.ord_to_doc ? seg.ord_to_doc[ord] : (int32_t)ord;
        const float4* xr = static_cast<const float4*>(seg.rows) + ord * p.units;
        float ax = 0.f, ay = 0.f, az = 0.f, aw = 0.f;
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const int f = t + j * L;
            const float4 x = (valid && f < p.units) ? xr[f] : make_float4(0.f, 0.f, 0.f, 0.f);
            if constexpr (L2K) {
                const float dx = x.x - qf[j].x, dy = x.y - qf[j].y, dz = x.z - qf[j].z, dw = x.w - qf[j].w;
                ax = fmaf(dx, dx, ax); ay = fmaf(dy, dy, ay); az = fmaf(dz, dz, az); aw = fmaf(dw, dw, aw);
            } else {
                ax = fmaf(x.x, qf[j].x, ax); ay = fmaf(x.y, qf[j].y, ay);
                az = fmaf(x.z, qf[j].z, az); aw = fmaf(x.w, qf[j].w, aw);
            }
        }
        float sum = (ax + ay) + (az + aw);
        sum = lane_sum<L>(sum);
        float sc;
        if constexpr (L2K) sc = score_f32_l2(sum);
        else sc = score_f32(sim, sum, qn, (sim == SIM_COSINE && valid) ? seg.xnorm_f[ord] : 0.0f);
        const uint64_t key = valid ? make_key(sc, (uint32_t)(seg.doc_base + doc)) : 0ull;
        // wave_offer (inline: the helpers live in osk_kernels.hip)
        uint64_t m = __ballot(t == 0 && key > thr);
        while (m) {
            const int src = __builtin_ctzll(m);
            const uint64_t K = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(key >> 32), src) << 32) |
                               (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)key, src);
            const uint64_t better = __ballot(lane < k && lk > K);
            const int pos = __popcll(better);
            const uint64_t up = ((uint64_t)(uint32_t)__shfl_up((int)(lk >> 32), 1) << 32) |
                                (uint32_t)__shfl_up((int)(uint32_t)lk, 1);
            lk = lane < pos ? lk : (lane == pos ? K : up);
            thr = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(lk >> 32), k - 1) << 32) |
                  (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)lk, k - 1);
            m &= ~(1ull << src);
            m &= __ballot(t == 0 && key > thr);
        }
    }
    if (lane < k) p.shard_keys[o * k + lane] = lk;
    const int cnt = __popcll(__ballot(lane < k && lk != 0ull));
    // cross-lane reads with every lane active (bpermute from an inactive lane returns 0)
    const uint64_t a_last = __shfl(akey, kKC - 1);
    const uint64_t e_kth = __shfl(lk, k - 1);
    if (lane == 0) {
        p.shard_counts[o] = cnt;
        if (nc == kKC) {   // the candidate list is full: prove no non-candidate beats the k-th hit
            const double sa = (double)key_score(a_last);
            const double qabs = sqrt((double)fmaxf(p.qnorm_dev ? qn : p.qnorm_approx[q], 0.0f));
            const double xmax = sqrt((double)p.shard_maxnorm2[s]);
            const double e_dot = p.c * xmax * qabs;
            double U;
            switch (sim) {
                case SIM_DOT_PRODUCT: U = sa + 0.5 * e_dot; break;
                case SIM_COSINE: U = sa + 0.5 * p.c; break;
                case SIM_MIP: U = sa + e_dot; break;
                default: {
                    const double e_d2 = 2.0 * e_dot + 1e-6 * (xmax * xmax + qabs * qabs);
                    const double inv = 1.0 / sa - e_d2;
                    U = inv <= 1.0 ? 1.0 : 1.0 / inv;
                }
            }
            U += 1e-6 * fabs(U) + 1e-12;
            const bool ok = cnt == k && (double)key_score(e_kth) > U;
            if (!ok) atomicOr(&p.flags[q], 1);
        }
    }
}

using RescoreFn = void (*)(RescoreParams);
#define OSK_RS_ROW(L, V) {rescore<L, V, false>, rescore<L, V, true>}
static const RescoreFn kRescore[9][2] = {OSK_RS_ROW(4, 2),  OSK_RS_ROW(8, 2),  OSK_RS_ROW(8, 4),
                                         OSK_RS_ROW(16, 4), OSK_RS_ROW(16, 8), OSK_RS_ROW(16, 12),
                                         OSK_RS_ROW(32, 8), OSK_RS_ROW(64, 8), OSK_RS_ROW(64, 16)};

hipError_t launch_rescore(int cfg, int nq, const RescoreParams& p, hipStream_t s) {
    hipLaunchKernelGGL(kRescore[cfg][p.sim == SIM_EUCLIDEAN ? 1 : 0], dim3(p.n_shards, nq), dim3(64), 0, s, p);
    return hipGetLastError();
}

}  // namespace osk
