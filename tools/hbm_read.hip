// hbm_read.hip — the practical HBM read ceiling of this MI355X for a streaming scan, measured the way
// the scan kernels read: 16-byte loads per lane, several loads in flight per wave, optionally
// non-temporal, a grid of whole rounds of resident workgroups, an 8 GB buffer (far beyond the 256 MB
// MALL).  The roofline's `frac` prices kernels against the 8 TB/s spec; this gives the ceiling a pure
// read stream actually reaches, for comparison.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/hbm_read tools/hbm_read.hip && tools/hbm_read [GiB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

// Each workgroup reads one contiguous chunk; every wave-instruction reads 64 × 16 B = 1 KiB
// contiguous; U loads in flight per lane.  The xor-sum is written once per thread so nothing is
// optimised away.
template <int U, bool NT>
__global__ __launch_bounds__(256) void read_stream(const int4* __restrict__ src, int64_t n_units,
                                                   int64_t chunk, int* __restrict__ sink) {
    typedef int i4v __attribute__((ext_vector_type(4)));
    const int64_t begin = (int64_t)blockIdx.x * chunk;
    const int64_t end = begin + chunk < n_units ? begin + chunk : n_units;
    i4v acc = {0, 0, 0, 0};
    const __attribute__((address_space(1))) i4v* g = (const __attribute__((address_space(1))) i4v*)src;
    for (int64_t i = begin + threadIdx.x; i < end; i += (int64_t)256 * U) {
        i4v v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + (int64_t)u * 256;
            const int64_t jj = j < end ? j : begin;
            v[u] = NT ? __builtin_nontemporal_load(g + jj) : g[jj];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u];
    }
    const int x = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (x == 0x12345678) sink[threadIdx.x] = x;   // practically never: keeps the loads live
}

// The 6-bit tier's load shape (osk_sq6.hip): blocks of 1536 B read as one 16-B-per-lane instruction (1 KiB)
// and one 8-B-per-lane instruction (512 B), U blocks per wave-iteration, non-temporal — against the pure
// 16-B stream, to tell whether the 8-B half of the pattern costs bandwidth.
template <int U>
__global__ __launch_bounds__(256) void read_mixed(const char* __restrict__ src, int64_t n_blocks, int64_t chunk,
                                                  int* __restrict__ sink) {
    typedef int i4v __attribute__((ext_vector_type(4)));
    typedef int i2v __attribute__((ext_vector_type(2)));
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t begin = (int64_t)blockIdx.x * chunk;
    const int64_t end = begin + chunk < n_blocks ? begin + chunk : n_blocks;
    i4v acc = {0, 0, 0, 0};
    for (int64_t b = begin + wave; b < end; b += (int64_t)4 * U) {
        i4v h[U];
        i2v l[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = b + (int64_t)u * 4;
            const int64_t jj = j < end ? j : begin;
            const char* blk = src + jj * 1536;
            h[u] = __builtin_nontemporal_load(reinterpret_cast<const i4v*>(blk) + lane);
            l[u] = __builtin_nontemporal_load(reinterpret_cast<const i2v*>(blk + 1024) + lane);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            acc ^= h[u];
            acc.x ^= l[u].x;
            acc.y ^= l[u].y;
        }
    }
    const int x = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (x == 0x12345678) sink[threadIdx.x] = x;
}

template <int U>
double run_mixed(const char* src, int64_t bytes, int blocks, int* sink, int reps) {
    const int64_t n_blocks = bytes / 1536;
    const int64_t chunk = (n_blocks + blocks - 1) / blocks;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL((read_mixed<U>), dim3(blocks), dim3(256), 0, 0, src, n_blocks, chunk, sink);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((read_mixed<U>), dim3(blocks), dim3(256), 0, 0, src, n_blocks, chunk, sink);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return (double)n_blocks * 1536.0 * reps / (ms * 1e-3) / 1e12;   // TB/s
}

template <int U, bool NT>
double run(const int4* src, int64_t n_units, int blocks, int* sink, int reps) {
    const int64_t chunk = (n_units + blocks - 1) / blocks;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL((read_stream<U, NT>), dim3(blocks), dim3(256), 0, 0, src, n_units, chunk, sink);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((read_stream<U, NT>), dim3(blocks), dim3(256), 0, 0, src, n_units, chunk, sink);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return (double)n_units * 16.0 * reps / (ms * 1e-3) / 1e12;   // TB/s
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? std::atof(argv[1]) : 8.0;
    const int64_t n_units = (int64_t)(gib * (1ull << 30)) / 16;
    int4* src = nullptr;
    int* sink = nullptr;
    CHECK(hipMalloc(&src, n_units * 16));
    CHECK(hipMalloc(&sink, 256 * sizeof(int)));
    CHECK(hipMemset(src, 1, n_units * 16));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    std::printf("{\"device\": \"%s\", \"cus\": %d, \"bytes\": %lld, \"results\": [\n", prop.gcnArchName, cus,
                (long long)(n_units * 16));
    const int reps = 10;
    bool first = true;
    for (int per_cu : {4, 8, 16, 24}) {
        const int blocks = cus * per_cu;
        const double r[6] = {run<2, false>(src, n_units, blocks, sink, reps), run<4, false>(src, n_units, blocks, sink, reps),
                             run<8, false>(src, n_units, blocks, sink, reps), run<2, true>(src, n_units, blocks, sink, reps),
                             run<4, true>(src, n_units, blocks, sink, reps), run<8, true>(src, n_units, blocks, sink, reps)};
        const int us[3] = {2, 4, 8};
        for (int i = 0; i < 6; ++i) {
            std::printf("%s {\"blocks_per_cu\": %d, \"loads_in_flight\": %d, \"nt\": %s, \"TBps\": %.3f}", first ? "" : ",\n",
                        per_cu, us[i % 3], i >= 3 ? "true" : "false", r[i]);
            first = false;
        }
    }
    std::printf("\n], \"mixed_16B_8B\": [\n");
    first = true;
    for (int per_cu : {4, 8}) {
        const int blocks = cus * per_cu;
        const double r[3] = {run_mixed<2>(reinterpret_cast<const char*>(src), n_units * 16, blocks, sink, reps),
                             run_mixed<3>(reinterpret_cast<const char*>(src), n_units * 16, blocks, sink, reps),
                             run_mixed<4>(reinterpret_cast<const char*>(src), n_units * 16, blocks, sink, reps)};
        for (int i = 0; i < 3; ++i) {
            std::printf("%s {\"blocks_per_cu\": %d, \"blocks_in_flight_per_wave\": %d, \"TBps\": %.3f}",
                        first ? "" : ",\n", per_cu, i + 2, r[i]);
            first = false;
        }
    }
    std::printf("\n]}\n");
    CHECK(hipFree(src));
    CHECK(hipFree(sink));
    return 0;
}
