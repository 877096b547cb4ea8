// osk_device.h — device helpers shared by the prefilter (osk_sq8.hip) and the large-k select path
// (osk_select.hip): the certified bound of an int8 dot, the exact fp32 score in the streaming scan's
// lane order, and global-address-space loads.
#pragma once
#include "osk_internal.h"
#include "osk_wave.h"

namespace osk {

__device__ __forceinline__ float f32_round_up(double d) {   // d ≥ 0: smallest float ≥ d
    float f = (float)d;
    if ((double)f < d) f = __uint_as_float(__float_as_uint(f) + 1u);
    return f;
}

// ------------------------------------------------------------------------------------------------
// bounds
// ------------------------------------------------------------------------------------------------
// [lo, hi] ∋ the raw value the fp32 streaming scan computes for (row, query): its dot product
// (DOT_PRODUCT / COSINE / MAXIMUM_INNER_PRODUCT) or its squared distance (EUCLIDEAN).
//   x·b = s_x·s_b·I + e,  |e| ≤ s_x|q_x|·|δ_b| + |δ_x|·(s_b|q_b| + |δ_b|) = ax.y·qc.y + ax.z·qc.z
//   dot:  |dot_dev − x·b| ≤ γ_n·|x||b| ≤ gam·(|x|² + |b|²)
//   d²:   d² = |x|² + |b|² − 2x·b,  |d²_dev − d²| ≤ g2·d²
// Every float operation below rounds by ≤ 2^-24 relative; the 2^-20 slack covers all of them.
__device__ __forceinline__ void sq8_bounds(int sim, float I, float4 ax, float4 qc, float gam, float g2,
                                           float& lo, float& hi) {
    const float approx = I * (ax.x * qc.x);
    const float eq = fmaf(ax.y, qc.y, ax.z * qc.z);
    if (sim == SIM_EUCLIDEAN) {
        const float base = ax.w + qc.w;
        const float sl = 0x1p-20f * (base + 2.0f * (fabsf(approx) + eq));
        const float d2lo = base - 2.0f * (approx + eq) - sl;
        const float d2hi = base - 2.0f * (approx - eq) + sl;
        lo = fmaxf(d2lo, 0.0f) * (1.0f - g2);
        hi = d2hi * (1.0f + g2);
    } else {
        const float e = eq + gam * (ax.w + qc.w);
        const float sl = 0x1p-20f * (fabsf(approx) + e);
        hi = approx + e + sl;
        lo = approx - e - sl;
    }
}

// The one side of sq8_bounds the quick test reads (EUCLIDEAN: the d² lower bound; else the dot upper
// bound), bit-identical to sq8_bounds' value of it: hot loops need not compute the other side.
__device__ __forceinline__ float sq8_bound_side(int sim, float I, float4 ax, float4 qc, float gam, float g2) {
    const float approx = I * (ax.x * qc.x);
    const float eq = fmaf(ax.y, qc.y, ax.z * qc.z);
    if (sim == SIM_EUCLIDEAN) {
        const float base = ax.w + qc.w;
        const float sl = 0x1p-20f * (base + 2.0f * (fabsf(approx) + eq));
        const float d2lo = base - 2.0f * (approx + eq) - sl;
        return fmaxf(d2lo, 0.0f) * (1.0f - g2);
    }
    const float e = eq + gam * (ax.w + qc.w);
    const float sl = 0x1p-20f * (fabsf(approx) + e);
    return approx + e + sl;
}

// Quick-reject threshold of a wave list whose worst upper-bound key is `thr` (0 = list not full):
// a row whose bound fails sq8_pass has upper-bound score ≤ the list's worst score, so it cannot
// enter the list (the precise test below decides the rest).
//   EUCLIDEAN: d² threshold; COSINE: dot threshold per |x|; others: dot threshold.
__device__ __forceinline__ float sq8_quick(int sim, uint64_t thr, float sqn, float cos_slack) {
    if (thr == 0ull) return sim == SIM_EUCLIDEAN ? __builtin_inff() : -__builtin_inff();
    const float t = key_score(thr);
    switch (sim) {
        case SIM_EUCLIDEAN: {
            const float tm = t * (1.0f - 0x1p-16f);
            return tm > 0.0f ? 1.0f / tm - 1.0f : __builtin_inff();
        }
        case SIM_MIP: {
            const float tm = t * (1.0f - 0x1p-16f);
            if (!(tm > 0.0f)) return -__builtin_inff();
            return tm >= 1.0f ? tm - 1.0f : 1.0f - 1.0f / tm;
        }
        case SIM_DOT_PRODUCT: {
            const float tm = t - 0x1p-16f * fabsf(t) - 0x1p-20f;
            return 2.0f * tm - 1.0f;
        }
        default: {   // COSINE
            const float tm = t - 0x1p-16f * fabsf(t) - 0x1p-20f;
            return (2.0f * tm - 1.0f - cos_slack) * sqn;
        }
    }
}
__device__ __forceinline__ bool sq8_pass(int sim, float lo, float hi, float tq, float sx) {
    if (sim == SIM_EUCLIDEAN) return !(lo > tq);
    if (sim == SIM_COSINE) return !(hi < tq * sx);
    return !(hi < tq);
}

// A workgroup's visited rows, added with ONE global atomic per workgroup: per-wave atomics on a
// segment's counter queue at L2 behind each other and hold the kernel's last waves (every thread of the
// workgroup must call this: it has barriers).
__device__ __forceinline__ void add_visited_wg(unsigned long long* visited, uint32_t nvis) {
    __shared__ uint32_t s_vis;
    if (threadIdx.x == 0) s_vis = 0u;
    __syncthreads();
    if ((threadIdx.x & 63) == 0 && nvis) atomicAdd(&s_vis, nvis);
    __syncthreads();
    if (threadIdx.x == 0 && s_vis) atomicAdd(visited, (unsigned long long)s_vis);
}

// Global-address-space loads (global_load, not flat_load): a flat load also counts in lgkmcnt, so
// the first LDS read after it would wait for every row load in flight, prefetched ones included.
__device__ __forceinline__ int4 load_i4_g(const int4* p, bool nt) {
    typedef int i4v __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) const i4v gi4v;
    const gi4v* g = (const gi4v*)p;
    const i4v v = nt ? __builtin_nontemporal_load(g) : *g;
    return make_int4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float4 load_f4_g(const float4* p) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) const f4v gf4v;
    const f4v v = *(const gf4v*)p;
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ int4 load_i4_nt(const int4* p) {
    typedef int i4v __attribute__((ext_vector_type(4)));
    const i4v v = __builtin_nontemporal_load(reinterpret_cast<const i4v*>(p));
    return make_int4(v.x, v.y, v.z, v.w);
}

// LDS-DMA (global_load_lds_dwordx4) from a per-lane source into a wave-uniform LDS base (+ lane·16 B).
// Written as asm so the compiler keeps no bookkeeping for it (its own LDS-DMA tracking puts vmcnt(0)
// before every LDS read of the buffer): completion is counted by hand (vm_wait), and only the issuing
// wave reads what it loaded.  M0 is saved and restored inside the statement (compiler-reserved).
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_byte) {
    lds_byte = __builtin_amdgcn_readfirstlane(lds_byte);   // wave-uniform by construction; make it an SGPR
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_byte)
                 : "memory");
}
// N such DMAs in one statement (M0 saved once): the k-th from gbase + voff + k·GS (GS·(N−1) ≤ 4095: the
// instruction's immediate offset; gbase wave-uniform, in SGPRs) into LDS at lds[k].  The immediate offset
// moves the LDS destination too (M0 + offset + lane·16: tools/glds_offset_probe.hip), so M0 = lds[k] − k·GS,
// which must not go below 0: lds[k] ≥ k·GS (an M0 that wraps does not land — osk_testing_glds_probe; every
// caller's destinations grow by ≥ GS per DMA from the ring's base).
template <int N, int GS>
__device__ __forceinline__ void glds16_run(const void* gbase, uint32_t voff, const uint32_t (&ldsk)[N]) {
    static_assert((N == 1 || N == 2 || N == 4) && GS * (N - 1) <= 4095, "glds16_run: 1, 2 or 4 DMAs");
    uint32_t lds[N];
#pragma unroll
    for (int k = 0; k < N; ++k) lds[k] = ldsk[k] - (uint32_t)(k * GS);
    const uint64_t sb = (uint64_t)gbase;
    unsigned keep;
    if constexpr (N == 1) {
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 offset:0 nt\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(voff), "s"(sb), "s"(lds[0])
                     : "memory");
    } else if constexpr (N == 2) {
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 offset:0 nt\n\t"
                     "s_mov_b32 m0, %4\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 offset:%5 nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(voff), "s"(sb), "s"(lds[0]), "s"(lds[1]), "n"(GS)
                     : "memory");
    } else {
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 offset:0 nt\n\t"
                     "s_mov_b32 m0, %4\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 offset:%7 nt\n\t"
                     "s_mov_b32 m0, %5\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 offset:%8 nt\n\t"
                     "s_mov_b32 m0, %6\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 offset:%9 nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(voff), "s"(sb), "s"(lds[0]), "s"(lds[1]), "s"(lds[2]), "s"(lds[3]), "n"(GS), "n"(2 * GS),
                       "n"(3 * GS)
                     : "memory");
    }
}
template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// (kept in the scan's lane layout: L lanes per row, V float4 per lane, 4 fma chains, pairwise tree)
// exact score of one row (the streaming scan's arithmetic: same lane layout and fma order)
template <int L, int V, bool L2K>
__device__ __forceinline__ float settle_exact(const float4* xr, bool valid, int units, int t,
                                              const float4 (&qf)[V], int sim, float qn, float xn) {
    float4 xv[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
        const int f = t + j * L;
        xv[j] = (valid && f < units) ? xr[f] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float ax = 0.f, ay = 0.f, az = 0.f, aw = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j) {
        const float4 x = xv[j];
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
    if constexpr (L2K) return score_f32_l2(sum);
    else return score_f32(sim, sum, qn, xn);
}

// The exchange header check of the coordinator reduce (one wave, lane = 0..63): 1 when some rank's
// header words differ from rank 0's — the ranks did not issue the same call (osk_comm.hip).  The first
// mismatch is recorded in x.err: [1, rank 0's call sequence number, the rank, its sequence number].
// The flag is sticky: once an earlier call of the communicator has set it, every later reduce reports a
// mismatch too (count −1), without the host refusing the call before its collective (osk_comm.hip).
__device__ __forceinline__ int xchg_header_check(const XLayout& x, int n_ranks, size_t rank_words, int lane) {
    if (x.err && __hip_atomic_load(&x.err[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return 1;
    const int pairs = (n_ranks - 1) * kXHdrWords;
    int bad_pair = 0x7FFFFFFF;
    for (int e = lane; e < pairs; e += 64) {
        const int r = 1 + e / kXHdrWords, w = e % kXHdrWords;
        if (x.hdr[(size_t)r * rank_words + w] != x.hdr[w]) bad_pair = min(bad_pair, e);
    }
    // a refusing rank (every rank may refuse alike: the headers then agree) — rank 0's refusal counts as a
    // mismatch at rank 1 (its header word 0), another rank's at its own
    for (int r = lane; r < n_ranks; r += 64)
        if (x.hdr[(size_t)r * rank_words] != kXMagic) bad_pair = min(bad_pair, max(r - 1, 0) * kXHdrWords);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) bad_pair = min(bad_pair, __shfl_xor(bad_pair, o));
    if (bad_pair == 0x7FFFFFFF) return 0;
    if (lane == 0 && x.err) {
        const int r = 1 + bad_pair / kXHdrWords;
        x.err[1] = (int64_t)x.hdr[1];
        x.err[2] = r;
        x.err[3] = (int64_t)x.hdr[(size_t)r * rank_words + 1];
        __threadfence_system();
        x.err[0] = 1;
    }
    return 1;
}

}  // namespace osk
