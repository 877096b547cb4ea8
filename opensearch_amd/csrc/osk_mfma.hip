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

hipError_t launch_max_norm2(const float* xn, int64_t n, unsigned* out, hipStream_t s) {
    int64_t blocks = (n + kBlock - 1) / kBlock;
    if (blocks < 1) blocks = 1;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(max_norm2, dim3((unsigned)blocks), dim3(kBlock), 0, s, xn, n, out);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// candidate pass: 8 waves, 128 rows × 256 queries per tile, K-steps of 32 dims.
// ------------------------------------------------------------------------------------------------
constexpr int kMB = 512;                       // threads per workgroup
constexpr int kStageA = 16 * 1024;             // 8 row blocks × hi/lo × 1 KiB
constexpr int kStageB = 32 * 1024;             // 16 query blocks × hi/lo × 1 KiB
constexpr int kStage = kStageA + kStageB;      // 48 KiB
constexpr int kStagePitch = 260;               // fp32 per staged score row (bank-conflict-free writes)
constexpr int kStaging = 128 * kStagePitch * 4; // 130 KiB of epilogue score staging (aliases the ring)
constexpr int kLds = 3 * kStage > kStaging ? 3 * kStage : kStaging;   // 144 KiB: 3-slot ring

__device__ __forceinline__ void glds16(const void* g, char* lds_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
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

__global__ __launch_bounds__(kMB) void mfma_cand(MfmaParams p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform → scalar addressing
    const int wr = wave & 1, wq = wave >> 1;
    const MfmaUnit unit = p.units[blockIdx.x];
    const SegDev seg = p.segs[unit.seg];
    const char* __restrict__ A = static_cast<const char*>(p.seg_split[unit.seg]);
    const int qblock = blockIdx.y;
    const char* __restrict__ Bq = static_cast<const char*>(p.qsplit) + (size_t)qblock * 16 * p.KS * 2 * 1024;
    const int KS = p.KS, sim = p.sim;
    const uint64_t* abits = p.accept ? p.accept[unit.seg] : nullptr;

    // thread-side selection state: thread ↔ (query q_sel of this block, row half h_sel)
    const int q_sel = tid & 255, h_sel = tid >> 8;
    uint64_t lst[kKC];
#pragma unroll
    for (int i = 0; i < kKC; ++i) lst[i] = 0ull;
    uint32_t nvis = 0;

    // this lane's queries / norms in the MFMA layout: q_local = wq·64 + qb·16 + (lane & 15)
    float qn_l[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int qg = qblock * 256 + wq * 64 + j * 16 + (lane & 15);
        qn_l[j] = qg < p.nq_pad ? p.qnorm[qg] : 1.0f;
    }

    // Each wave moves 6 of the 48 1-KiB chunks of a stage.  Chunk c of k-step ks lives at a
    // wave-uniform byte offset; only lane·16 varies per lane.
    const int lane16 = lane * 16;
    auto issue = [&](const char* tileA, int ks, int buf) {
        char* base = smem + buf * kStage;
#pragma unroll
        for (int c6 = 0; c6 < 6; ++c6) {
            const int c = wave * 6 + c6;   // uniform
            const char* src;
            char* dst;
            if (c < 16) {
                const int rb = c >> 1, part = c & 1;
                src = tileA + (size_t)((rb * KS + ks) * 2 + part) * 1024;
                dst = base + c * 1024;
            } else {
                const int c2 = c - 16, qb = c2 >> 1, part = c2 & 1;
                src = Bq + (size_t)((qb * KS + ks) * 2 + part) * 1024;
                dst = base + kStageA + c2 * 1024;
            }
            if (!(p.ablate & (c < 16 ? 4 : 2))) glds16(src + lane16, dst);
        }
    };

    for (int64_t tile = unit.tile_begin; tile < unit.tile_end; ++tile) {
        const int64_t tile_rb0 = tile * 8;
        f32x4 acc[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

        // 3-slot ring, two K-steps in flight: slot (ks+2)%3 was last read in iteration ks−1, whose
        // closing barrier every wave has passed before this iteration issues into it.
        const char* tileA = A + (size_t)tile_rb0 * KS * 2048;
        issue(tileA, 0, 0);
        if (KS > 1) issue(tileA, 1, 1);
        int buf = 0;
        for (int ks = 0; ks < KS; ++ks) {
            if (ks + 2 < KS) {
                const int nb = buf == 0 ? 2 : buf - 1;   // (ks + 2) % 3
                issue(tileA, ks + 2, nb);
                asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
            } else if (ks + 1 < KS) {
                asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __builtin_amdgcn_s_barrier();
            const char* sA = smem + buf * kStage;
            const char* sB = sA + kStageA;
            bf16x8 bh[4], bl[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int qb = wq * 4 + j;
                bh[j] = *reinterpret_cast<const bf16x8*>(sB + (qb * 2 + 0) * 1024 + lane * 16);
                bl[j] = *reinterpret_cast<const bf16x8*>(sB + (qb * 2 + 1) * 1024 + lane * 16);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int rb = wr * 4 + i;
                const bf16x8 ah = *reinterpret_cast<const bf16x8*>(sA + (rb * 2 + 0) * 1024 + lane * 16);
                const bf16x8 al = *reinterpret_cast<const bf16x8*>(sA + (rb * 2 + 1) * 1024 + lane * 16);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[j], acc[i][j], 0, 0, 0);
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();   // every wave is done reading buf: it may be refilled
            buf = buf == 2 ? 0 : buf + 1;
        }
        __syncthreads();

        // epilogue: approx scores → staged [128 rows][256 queries] (the accumulators die here) →
        // thread (q_sel, h_sel) offers rows h_sel·64 … +63 of its query to its top-k' list
        float* staged = reinterpret_cast<float*>(smem);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row_local = wr * 64 + i * 16 + (lane >> 4) * 4 + r;
                const int64_t row = tile_rb0 * 16 + row_local;
                const bool rv = row < seg.n_rows;
                const float xn = rv ? seg.xnorm_f[row] : 1.0f;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int ql = wq * 64 + j * 16 + (lane & 15);
                    staged[row_local * kStagePitch + ql] =
                        rv ? approx_score(sim, acc[i][j][r], qn_l[j], xn) : -__builtin_inff();
                }
            }
        __syncthreads();
        const int sel_rows = (p.ablate & 1) ? 0 : 64;
#pragma unroll 2
        for (int rr = 0; rr < sel_rows; ++rr) {
            const int row_local = h_sel * 64 + rr;
            const int64_t ord = tile_rb0 * 16 + row_local;
            const float s = staged[row_local * kStagePitch + q_sel];
            if (!(s > -__builtin_inff())) continue;
            if (abits) {
                const int32_t doc = seg.ord_to_doc ? seg.ord_to_doc[ord] : (int32_t)ord;
                if (!((abits[doc >> 6] >> (doc & 63)) & 1ull)) continue;
            }
            if (q_sel == 0) ++nvis;
            const uint64_t key = make_key(s, (uint32_t)(unit.vrow_base + ord));
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
        __syncthreads();
    }

    const int qg = qblock * 256 + q_sel;
    if (qg < p.nq) {
        uint64_t* o = p.cand + ((size_t)qg * p.n_units * 2 + (size_t)blockIdx.x * 2 + h_sel) * kKC;
#pragma unroll
        for (int i = 0; i < kKC; ++i) o[i] = lst[i];
    }
    if (p.visited && qblock == 0 && q_sel == 0) atomicAdd(&p.visited[unit.seg], (unsigned long long)nvis);
}

hipError_t launch_mfma_cand(const MfmaParams& p, int n_qblocks, hipStream_t s) {
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)mfma_cand, hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    hipLaunchKernelGGL(mfma_cand, dim3(p.n_units, n_qblocks), dim3(kMB), kLds, s, p);
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
#pragma unroll
        for (int m = 1; m < L; m <<= 1) sum += __shfl_xor(sum, m);
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
