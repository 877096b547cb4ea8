// Where does an LDS-DMA with an immediate offset write?  global_load_lds_dwordx4 v, s[base] offset:1024 with
// M0 = 0: the global source is base + v + 1024; the probe reports whether the LDS destination is M0 + lane·16
// or M0 + 1024 + lane·16 (both inside the 8 KiB it allocates).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void probe(const int4* src, int* out) {
    __shared__ __attribute__((aligned(16))) int4 lds[512];
    for (int i = threadIdx.x; i < 512; i += 64) lds[i] = make_int4(-1, -1, -1, -1);
    __syncthreads();
    const uint32_t voff = threadIdx.x * 16u;
    const uint64_t sb = (uint64_t)src;
    const uint32_t m0v = (uint32_t)(size_t)(__attribute__((address_space(3))) char*)lds;
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 offset:1024 nt\n\t"
                 "s_mov_b32 m0, %0\n\ts_waitcnt vmcnt(0)"
                 : "=&s"(keep) : "v"(voff), "s"(sb), "s"(m0v) : "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        out[0] = lds[0].x;    // M0 + lane·16: lane 0's value
        out[1] = lds[64].x;   // M0 + 1024 + lane·16: lane 0's value
    }
}
int main() {
    int4 h[128];
    for (int i = 0; i < 128; ++i) h[i] = make_int4(i, i, i, i);
    int4* d; int* o; int ho[2];
    hipMalloc(&d, sizeof(h)); hipMalloc(&o, 8);
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, o);
    hipMemcpy(ho, o, 8, hipMemcpyDeviceToHost);
    // the source of lane 0 is unit 64 (base + 1024 B)
    printf("lds[0].x = %d, lds[64].x = %d -> %s\n", ho[0], ho[1],
           ho[1] == 64 ? "offset applies to the LDS address too" : ho[0] == 64 ? "LDS address = M0 + lane*16" : "?");
    return 0;
}
