// osk_wave.h — wavefront-level top-k helpers shared by the scan, prefilter and merge kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace osk {

// ------------------------------------------------------------------------------------------------
// wavefront helpers
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, l);
    uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl_up1_64(uint64_t v) {
    int lo = __shfl_up((int)(uint32_t)v, 1);
    int hi = __shfl_up((int)(uint32_t)(v >> 32), 1);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

// Sum of v over each aligned group of L lanes (L a power of two ≤ 64), every lane of the group receiving
// it.  The steps are the xor butterfly's (partners at distance 1, 2, 4, … in that order), so fp32 sums
// have exactly its bits; distances 1 and 2 are DPP quad permutes and 4 and 8 DPP row mirrors (after the
// first steps every lane of a quad / 8-lane half holds the same partial, so the mirrored partner's value
// is the xor partner's), fused into the add: __shfl_xor compiles to ds_bpermute, an LDS round trip per
// step on the scans' critical path.  16 and 32 stay shuffles.
template <int CTRL>
__device__ __forceinline__ int dpp_mov(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
template <int L>
__device__ __forceinline__ int lane_sum(int v) {
    if constexpr (L >= 2) v += dpp_mov<0xB1>(v);    // quad_perm [1,0,3,2]
    if constexpr (L >= 4) v += dpp_mov<0x4E>(v);    // quad_perm [2,3,0,1]
    if constexpr (L >= 8) v += dpp_mov<0x141>(v);   // row_half_mirror
    if constexpr (L >= 16) v += dpp_mov<0x140>(v);  // row_mirror
    if constexpr (L >= 32) v += __shfl_xor(v, 16);
    if constexpr (L >= 64) v += __shfl_xor(v, 32);
    return v;
}
template <int L>
__device__ __forceinline__ float lane_sum(float v) {
    if constexpr (L >= 2) v += __int_as_float(dpp_mov<0xB1>(__float_as_int(v)));
    if constexpr (L >= 4) v += __int_as_float(dpp_mov<0x4E>(__float_as_int(v)));
    if constexpr (L >= 8) v += __int_as_float(dpp_mov<0x141>(__float_as_int(v)));
    if constexpr (L >= 16) v += __int_as_float(dpp_mov<0x140>(__float_as_int(v)));
    if constexpr (L >= 32) v += __shfl_xor(v, 16);
    if constexpr (L >= 64) v += __shfl_xor(v, 32);
    return v;
}

// Insert key K (known to beat thr = lk[k-1]) into the wave's sorted-descending list held in
// lanes 0..k-1 of lk.  Entries better than K form a prefix; K goes to lane `pos`, the tail
// shifts down one lane and the old k-th entry falls off.
__device__ __forceinline__ void wave_insert(uint64_t& lk, uint64_t& thr, uint64_t K, int lane,
                                            int k) {
    const uint64_t better = __ballot(lane < k && lk > K);
    const int pos = __popcll(better);
    const uint64_t up = shfl_up1_64(lk);
    lk = lane < pos ? lk : (lane == pos ? K : up);
    thr = readlane64(lk, k - 1);
}

// Offer each lane's key where `offer` holds; wave-uniform loop over the (few) lanes that beat thr.
__device__ __forceinline__ void wave_offer(uint64_t key, bool offer, uint64_t& lk, uint64_t& thr,
                                           int lane, int k) {
    uint64_t m = __ballot(offer && key > thr);
    while (m) {
        const int src = __builtin_ctzll(m);
        const uint64_t K = readlane64(key, src);
        wave_insert(lk, thr, K, lane, k);
        m &= ~(1ull << src);
        m &= __ballot(offer && key > thr);
    }
}

// wave_offer with a 32-bit payload riding along each list entry (the prefilter's lower bound).
__device__ __forceinline__ void wave_offer2(uint64_t key, uint32_t pay, bool offer, uint64_t& lk,
                                            uint32_t& lp, uint64_t& thr, int lane, int k) {
    uint64_t m = __ballot(offer && key > thr);
    while (m) {
        const int src = __builtin_ctzll(m);
        const uint64_t K = readlane64(key, src);
        const uint32_t P = (uint32_t)__builtin_amdgcn_readlane((int)pay, src);
        const uint64_t better = __ballot(lane < k && lk > K);
        const int pos = __popcll(better);
        const uint64_t up = shfl_up1_64(lk);
        const uint32_t upp = (uint32_t)__shfl_up((int)lp, 1);
        lk = lane < pos ? lk : (lane == pos ? K : up);
        lp = lane < pos ? lp : (lane == pos ? P : upp);
        thr = readlane64(lk, k - 1);
        m &= ~(1ull << src);
        m &= __ballot(offer && key > thr);
    }
}

// Walk a wave's rows [wb, we) in groups of R (lane group g ↔ one row) and call
// body(row, in_range, accepted_known).  Filter pushdown: with an accept bitset over a dense field
// (doc == ord) the rows are taken 64 at a time, the accepted ones are compacted to the front of
// the wave with one ds_permute, and only they are visited — at 1 % selectivity a wave touches ~1 %
// of the rows instead of every row.  Otherwise every row is visited and the body checks accept.
template <int R, class F>
__device__ __forceinline__ void walk_rows(int64_t wb, int64_t we, const uint64_t* abits,
                                          const int32_t* ord_to_doc, int lane, int g, F&& body) {
    if (abits && !ord_to_doc) {
        for (int64_t w0 = wb; w0 < we; w0 += 64) {
            const int64_t word = w0 >> 6;
            const int sh = (int)(w0 & 63);
            uint64_t m = abits[word] >> sh;
            if (sh && (word + 1) * 64 < we) m |= abits[word + 1] << (64 - sh);
            if (we - w0 < 64) m &= (1ull << (we - w0)) - 1ull;
            const int n = __popcll(m);
            if (n == 0) continue;
            // rank of each lane's bit among the set (or the unset) bits → a permutation that puts
            // the positions of the n accepted rows into lanes 0..n-1
            const bool bit = (m >> lane) & 1ull;
            const int below = __popcll(m & ((1ull << lane) - 1ull));
            const int dst = bit ? below : n + (lane - below);
            const int pos = __builtin_amdgcn_ds_permute(dst << 2, lane);
            for (int i0 = 0; i0 < n; i0 += R) {
                const int idx = i0 + g;
                const int pr = __shfl(pos, idx < 64 ? idx : 0);
                body(w0 + pr, idx < n, true);
            }
        }
    } else {
        for (int64_t r0 = wb; r0 < we; r0 += R) body(r0 + g, r0 + g < we, false);
    }
}

// Top-k of NW wave lists in LDS (lists[w·64 + i], i < k, best first, 0 = empty; non-zero keys are
// distinct): thread t < NW·k ranks its key against all NW·k keys and writes it to out[rank] when
// rank < k.  Every thread works at once (a serial fold of NW lists by one wave costs ~NW·k insertion
// rounds); out[] slots past the number of keys keep what the caller put there (zeros).
template <int NW>
__device__ __forceinline__ void block_rank_topk(const uint64_t* lists, int k, int tid, uint64_t* out) {
    if (tid < NW * k) {
        const int w = tid / k, i = tid - w * k;
        const uint64_t key = lists[w * 64 + i];
        if (key) {
            int rank = 0;
            for (int w2 = 0; w2 < NW; ++w2) {
                const uint64_t* l2 = lists + w2 * 64;
                for (int i2 = 0; i2 < k; ++i2) rank += l2[i2] > key;
            }
            if (rank < k) out[rank] = key;
        }
    }
}

// Fold the lists of waves 1..3 (in LDS) into wave 0's list.
__device__ __forceinline__ void block_fold(const uint64_t* lists /*[4][64]*/, uint64_t& lk,
                                           uint64_t& thr, int lane, int k) {
    for (int w = 1; w < 4; ++w) {
        const uint64_t key = lane < k ? lists[w * 64 + lane] : 0ull;
        wave_offer(key, true, lk, thr, lane, k);
    }
}

}  // namespace osk
