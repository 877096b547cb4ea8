// lds_ring.hip — streaming rate of the wide prefilter's load structure (osk_sq8w.hip), in isolation:
// persistent workgroups of 4 waves, each step = 4 groups of (KS 1-KiB LDS-DMA pieces + one 272-B piece), one
// piece set per wave, an NS-deep ring, a counted vmcnt wait and a workgroup barrier per step, no compute.
// Prints TB/s for ring depths, workgroups per CU and the variants that isolate the barrier and the
// per-lane source permutation.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/lds_ring tools/lds_ring.hip && tools/lds_ring
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_byte) {
    lds_byte = __builtin_amdgcn_readfirstlane(lds_byte);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_byte)
                 : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// MODE bit 1: no barrier; bit 2: lane-linear sources (no permutation); bit 4: no aux piece
// WORK: dependent VALU fma per step after the barrier (the compute a real step does); WAVES: 4 or 8 (8: waves
// 4–7 issue no DMA and only compute)
template <int KS, int NS, int MODE, int WORK = 0, int WAVES = 4>
__global__ __launch_bounds__(WAVES * 64, 1) void ring(const int4* __restrict__ rows, const int4* __restrict__ aux,
                                                      int64_t n_steps_total, int* __restrict__ sink) {
    constexpr int GB = KS * 1024 + 17 * 16, SLOT = 4 * GB, OPS = KS + ((MODE & 4) ? 0 : 1);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, wave_id = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wave = wave_id & 3;
    const bool loader = wave_id < 4;
    float f = (float)lane;
    const int64_t per = (n_steps_total + gridDim.x - 1) / gridDim.x;
    const int64_t s0 = (int64_t)blockIdx.x * per, s1 = s0 + per < n_steps_total ? s0 + per : n_steps_total;
    const int total = (int)(s1 > s0 ? s1 - s0 : 0);
    const uint32_t ring_lds = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(__attribute__((address_space(3))) char*)smem);
    const int perm = (MODE & 2) ? lane : (lane & 15) * 4 + (lane >> 4);
    auto issue = [&](int st, int slot) {
        if (!loader) return;
        const int64_t g = (s0 + st) * 4 + wave;   // this wave's 16-row group
        const int4* src = rows + g * (KS * 64);
        const uint32_t dst = ring_lds + (uint32_t)(slot * SLOT + wave * GB);
#pragma unroll
        for (int s = 0; s < KS; ++s) glds16(src + s * 64 + perm, dst + s * 1024);
        if (!(MODE & 4) && lane <= 16) glds16(aux + g * 17 + lane, dst + KS * 1024);
    };
    int acc = 0;
    for (int st = 0; st < NS - 1 && st < total; ++st) issue(st, st);
    int s_issue = (NS - 1) % NS, s_read = 0;
    for (int i = 0; i < total; ++i) {
        if (i + NS - 1 <= total)
            vm_wait<(NS - 2) * OPS>();
        else
            vm_wait<0>();
        if (!(MODE & 1)) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (i + NS - 1 < total) {
            issue(i + NS - 1, s_issue);
            s_issue = s_issue + 1 == NS ? 0 : s_issue + 1;
        }
        const int* sl = reinterpret_cast<const int*>(smem + s_read * SLOT);
        s_read = s_read + 1 == NS ? 0 : s_read + 1;
        acc ^= sl[lane * 4 + wave];   // touch the slot
#pragma unroll 16
        for (int w = 0; w < WORK; ++w) f = fmaf(f, 1.0000001f, 0.5f);
    }
    vm_wait<0>();
    if (acc == 0x12345678 || f == 1.2345f) sink[threadIdx.x] = acc;
}

template <int KS, int NS, int MODE, int WORK = 0, int WAVES = 4>
double run(const int4* rows, const int4* aux, int64_t n_steps, int blocks, int per_cu, int* sink) {
    const size_t lds = (size_t)NS * 4 * (KS * 1024 + 17 * 16);
    if (lds * per_cu > 160 * 1024) return -1.0;
    auto fn = ring<KS, NS, MODE, WORK, WAVES>;
    CHECK(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(fn, dim3(blocks), dim3(WAVES * 64), lds, 0, rows, aux, n_steps, sink);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a, 0));
    const int reps = 5;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(fn, dim3(blocks), dim3(WAVES * 64), lds, 0, rows, aux, n_steps, sink);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double bytes = (double)n_steps * 4 * (KS * 1024 + ((MODE & 4) ? 0 : 272)) * reps;
    return bytes / (ms * 1e-3) / 1e12;
}

int main() {
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const int64_t n_steps = 1 << 20;   // 4M groups of 16 rows: 8.6 GB of KS = 2 pieces
    int4 *rows = nullptr, *aux = nullptr;
    int* sink = nullptr;
    CHECK(hipMalloc(&rows, (size_t)n_steps * 4 * 2 * 1024 + 4096));
    CHECK(hipMalloc(&aux, (size_t)n_steps * 4 * 17 * 16 + 4096));
    CHECK(hipMalloc(&sink, 4096));
    CHECK(hipMemset(rows, 1, (size_t)n_steps * 4 * 2 * 1024));
    CHECK(hipMemset(aux, 1, (size_t)n_steps * 4 * 17 * 16));
    std::printf("{\"cus\": %d, \"results\": [\n", cus);
    bool first = true;
    auto pr = [&](const char* name, int per_cu, double tbps) {
        std::printf("%s {\"variant\": \"%s\", \"wg_per_cu\": %d, \"TBps\": %.3f}", first ? "" : ",\n", name, per_cu, tbps);
        first = false;
    };
    pr("NS8_work100", 1, run<2, 8, 0, 100>(rows, aux, n_steps, cus, 1, sink));
    pr("NS8_work300", 1, run<2, 8, 0, 300>(rows, aux, n_steps, cus, 1, sink));
    pr("NS8_work600", 1, run<2, 8, 0, 600>(rows, aux, n_steps, cus, 1, sink));
    pr("NS8_work300_8waves", 1, run<2, 8, 0, 300, 8>(rows, aux, n_steps, cus, 1, sink));
    pr("NS8_work600_8waves", 1, run<2, 8, 0, 600, 8>(rows, aux, n_steps, cus, 1, sink));
    for (int per_cu : {1}) {
        const int blocks = cus * per_cu;
        pr("NS2", per_cu, run<2, 2, 0>(rows, aux, n_steps, blocks, per_cu, sink));
        pr("NS4", per_cu, run<2, 4, 0>(rows, aux, n_steps, blocks, per_cu, sink));
        pr("NS8", per_cu, run<2, 8, 0>(rows, aux, n_steps, blocks, per_cu, sink));
        pr("NS8_nobarrier", per_cu, run<2, 8, 1>(rows, aux, n_steps, blocks, per_cu, sink));
        pr("NS8_linear", per_cu, run<2, 8, 2>(rows, aux, n_steps, blocks, per_cu, sink));
        pr("NS8_noaux", per_cu, run<2, 8, 4>(rows, aux, n_steps, blocks, per_cu, sink));
        pr("NS8_linear_noaux_nobarrier", per_cu, run<2, 8, 7>(rows, aux, n_steps, blocks, per_cu, sink));
    }
    std::printf("\n]}\n");
    return 0;
}
