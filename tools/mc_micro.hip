// Micro-benchmark: where does a one-query coordinator merge (8 shards × k=10) spend its ~10 µs?
// Phase timestamps (s_memrealtime, 100 MHz) of a copy of merge_coord's structure, plus the launch
// latency of an empty kernel and of a kernel with the same 48 KB of static LDS.
// Build: hipcc --offload-arch=gfx950 -O3 -Iopensearch_amd/csrc tools/mc_micro.hip -o tools/mc_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#include "osk_common.h"

constexpr int kB = 256;
constexpr int kMax = 4096;

__global__ void empty_k(int* p) { if (threadIdx.x == 1000) p[0] = 1; }

__global__ __launch_bounds__(kB) void lds_k(int* p) {
    __shared__ uint32_t a[3 * kMax];
    a[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (a[(threadIdx.x + 1) & 255] == 1000) p[0] = 1;
}

template <bool TRACE>
__global__ __launch_bounds__(kB) void mc(const uint64_t* __restrict__ keys, const int32_t* __restrict__ sidx_g, int S,
                                         int k, int from, int size, float* scores, int32_t* docs, int32_t* shard_out,
                                         int32_t* count, int64_t* total, float* maxs, uint64_t* tr) {
    __shared__ __attribute__((aligned(16))) uint32_t s_su[kMax];
    __shared__ __attribute__((aligned(16))) int32_t s_sidx[kMax];
    __shared__ __attribute__((aligned(16))) int32_t s_doc[kMax];
    __shared__ int s_n;
    __shared__ unsigned long long s_total;
    __shared__ uint32_t s_max;
    const int tid = threadIdx.x;
    if (TRACE && tid == 0) tr[0] = wall_clock64();
    const int topn = min(k, from + size);
    const int n_slots = S * topn;
    const int n4 = (n_slots + 3) & ~3;
    if (tid == 0) { s_n = 0; s_total = 0ull; s_max = 0u; }
    __syncthreads();
    int mine = 0;
    for (int slot = tid; slot < n4; slot += kB) {
        const int s = slot / topn, i = slot - s * topn;
        const bool real = slot < n_slots;
        const uint64_t key = real ? keys[(size_t)s * k + i] : 0ull;
        const int32_t si = real ? sidx_g[s] : 0;
        const bool hit = real && key != 0ull;
        s_su[slot] = hit ? (uint32_t)(key >> 32) : 0u;
        s_doc[slot] = hit ? osk::key_doc(key) : INT32_MAX;
        s_sidx[slot] = hit ? si : INT32_MAX;
        mine += hit;
        if (hit && i == 0) atomicMax(&s_max, (uint32_t)(key >> 32));
    }
    if (TRACE && tid == 0) tr[1] = wall_clock64();
    if (mine) { atomicAdd(&s_n, mine); atomicAdd(&s_total, (unsigned long long)mine); }
    __syncthreads();
    if (TRACE && tid == 0) tr[2] = wall_clock64();
    for (int i = tid; i < n_slots; i += kB) {
        const uint32_t su = s_su[i];
        if (su == 0u && s_sidx[i] == INT32_MAX) continue;
        const int32_t si = s_sidx[i], d = s_doc[i];
        int rank = 0;
#pragma unroll 4
        for (int j = 0; j < n4; j += 4) {
            const uint4 u4 = *reinterpret_cast<const uint4*>(s_su + j);
            const int4 s4 = *reinterpret_cast<const int4*>(s_sidx + j);
            const int4 d4 = *reinterpret_cast<const int4*>(s_doc + j);
            rank += (u4.x > su) || (u4.x == su && (s4.x < si || (s4.x == si && d4.x < d)));
            rank += (u4.y > su) || (u4.y == su && (s4.y < si || (s4.y == si && d4.y < d)));
            rank += (u4.z > su) || (u4.z == su && (s4.z < si || (s4.z == si && d4.z < d)));
            rank += (u4.w > su) || (u4.w == su && (s4.w < si || (s4.w == si && d4.w < d)));
        }
        if (rank >= from && rank < from + size) {
            scores[rank - from] = osk::sortable_to_float(su);
            docs[rank - from] = d;
            shard_out[rank - from] = si;
        }
    }
    if (TRACE && tid == 0) tr[3] = wall_clock64();
    __syncthreads();
    if (tid == 0) {
        count[0] = min(size, s_n);
        total[0] = (int64_t)s_total;
        maxs[0] = osk::sortable_to_float(s_max);
    }
    if (TRACE && tid == 0) tr[4] = wall_clock64();
}

// variant: no LDS atomics (hit count by __syncthreads_count, max score = the rank-0 hit), and the
// rank loop reads only the 32-bit scores (ties, rare, take the detailed (shardIndex, doc) compare)
template <bool TRACE>
__global__ __launch_bounds__(kB) void mc2(const uint64_t* __restrict__ keys, const int32_t* __restrict__ sidx_g, int S,
                                          int k, int from, int size, float* scores, int32_t* docs, int32_t* shard_out,
                                          int32_t* count, int64_t* total, float* maxs, uint64_t* tr) {
    __shared__ __attribute__((aligned(16))) uint32_t s_su[kMax];
    __shared__ __attribute__((aligned(16))) int32_t s_sidx[kMax];
    __shared__ __attribute__((aligned(16))) int32_t s_doc[kMax];
    const int tid = threadIdx.x;
    if (TRACE && tid == 0) tr[0] = wall_clock64();
    const int topn = min(k, from + size);
    const int n_slots = S * topn;
    const int n4 = (n_slots + 3) & ~3;
    int mine = 0;
    for (int slot = tid; slot < n4; slot += kB) {
        const int s = slot / topn, i = slot - s * topn;
        const bool real = slot < n_slots;
        const uint64_t key = real ? keys[(size_t)s * k + i] : 0ull;
        const int32_t si = real ? sidx_g[s] : 0;
        const bool hit = real && key != 0ull;
        s_su[slot] = hit ? (uint32_t)(key >> 32) : 0u;
        s_doc[slot] = hit ? osk::key_doc(key) : INT32_MAX;
        s_sidx[slot] = hit ? si : INT32_MAX;
        mine += hit;
    }
    if (TRACE && tid == 0) tr[1] = wall_clock64();
    const int n = __syncthreads_count(mine);   // (≤ 1 slot per thread when n_slots ≤ 256)
    if (TRACE && tid == 0) tr[2] = wall_clock64();
    for (int i = tid; i < n_slots; i += kB) {
        const uint32_t su = s_su[i];
        if (su == 0u && s_sidx[i] == INT32_MAX) continue;
        const int32_t si = s_sidx[i], d = s_doc[i];
        int rank = 0, eq = 0;
#pragma unroll 4
        for (int j = 0; j < n4; j += 4) {
            const uint4 u4 = *reinterpret_cast<const uint4*>(s_su + j);
            rank += (u4.x > su) + (u4.y > su) + (u4.z > su) + (u4.w > su);
            eq += (u4.x == su) + (u4.y == su) + (u4.z == su) + (u4.w == su);
        }
        if (eq > 1) {   // equal scores: (shardIndex asc, doc asc)
            for (int j = 0; j < n_slots; ++j)
                rank += s_su[j] == su && (s_sidx[j] < si || (s_sidx[j] == si && s_doc[j] < d));
        }
        if (rank >= from && rank < from + size) {
            scores[rank - from] = osk::sortable_to_float(su);
            docs[rank - from] = d;
            shard_out[rank - from] = si;
        }
        if (rank == 0) maxs[0] = osk::sortable_to_float(su);
    }
    if (TRACE && tid == 0) tr[3] = wall_clock64();
    if (tid == 0) {
        count[0] = max(0, min(size, n - from));
        total[0] = n;
    }
    if (TRACE && tid == 0) tr[4] = wall_clock64();
}

int main() {
    const int S = 8, K = 10;
    std::vector<uint64_t> hk(S * K);
    for (int s = 0; s < S; ++s)
        for (int i = 0; i < K; ++i) hk[s * K + i] = ((uint64_t)(0xC0000000u - 1000u * i - s) << 32) | (0xFFFFFFFFu - (s * 100 + i));
    std::vector<int32_t> hs(S);
    for (int s = 0; s < S; ++s) hs[s] = s;
    uint64_t *dk, *tr; int32_t *ds, *docs, *sh, *cnt; float *sc, *mx; int64_t* tot; int* dummy;
    hipMalloc(&dk, 8 * S * K); hipMalloc(&ds, 4 * S); hipMalloc(&tr, 8 * 64);
    hipMalloc(&sc, 64); hipMalloc(&docs, 64); hipMalloc(&sh, 64); hipMalloc(&cnt, 4); hipMalloc(&tot, 8);
    hipMalloc(&mx, 4); hipMalloc(&dummy, 4);
    hipMemcpy(dk, hk.data(), 8 * S * K, hipMemcpyHostToDevice);
    hipMemcpy(ds, hs.data(), 4 * S, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    auto timeit = [&](const char* name, auto launch) {
        for (int i = 0; i < 50; ++i) launch();
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int i = 0; i < 1000; ++i) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("%-28s %8.2f us/launch (back-to-back)\n", name, ms);
    };
    timeit("empty kernel", [&] { hipLaunchKernelGGL(empty_k, dim3(1), dim3(kB), 0, 0, dummy); });
    timeit("48 KB static LDS kernel", [&] { hipLaunchKernelGGL(lds_k, dim3(1), dim3(kB), 0, 0, dummy); });
    timeit("merge_coord copy", [&] { hipLaunchKernelGGL(mc<false>, dim3(1), dim3(kB), 0, 0, dk, ds, S, K, 0, 10, sc, docs, sh, cnt, tot, mx, tr); });
    timeit("merge_coord v2", [&] { hipLaunchKernelGGL(mc2<false>, dim3(1), dim3(kB), 0, 0, dk, ds, S, K, 0, 10, sc, docs, sh, cnt, tot, mx, tr); });
    for (int v = 0; v < 2; ++v) {
    if (v == 0) hipLaunchKernelGGL(mc<true>, dim3(1), dim3(kB), 0, 0, dk, ds, S, K, 0, 10, sc, docs, sh, cnt, tot, mx, tr);
    else hipLaunchKernelGGL(mc2<true>, dim3(1), dim3(kB), 0, 0, dk, ds, S, K, 0, 10, sc, docs, sh, cnt, tot, mx, tr);
    hipDeviceSynchronize();
    uint64_t t[5];
    hipMemcpy(t, tr, 40, hipMemcpyDeviceToHost);
    printf("phases (10 ns ticks): loads %lu, atomics+sync %lu, rank+store %lu, tail %lu\n",
           (unsigned long)(t[1] - t[0]), (unsigned long)(t[2] - t[1]), (unsigned long)(t[3] - t[2]), (unsigned long)(t[4] - t[3]));
    std::vector<float> hsc(10); std::vector<int32_t> hd(10);
    hipMemcpy(hsc.data(), sc, 40, hipMemcpyDeviceToHost);
    hipMemcpy(hd.data(), docs, 40, hipMemcpyDeviceToHost);
    printf("top: %d %d %d\n", hd[0], hd[1], hd[2]);
    }
    return 0;
}
