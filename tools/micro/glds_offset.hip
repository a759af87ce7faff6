// Micro-test: does global_load_lds_dwordx4's instruction offset also move the LDS destination?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const unsigned* src, unsigned* out) {
    __shared__ __attribute__((aligned(16))) unsigned sm[2048];
    for (int i = threadIdx.x; i < 2048; i += 64) sm[i] = 0xdeadbeef;
    __syncthreads();
    unsigned voff = threadIdx.x * 16;                     // bytes
    unsigned lds0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) unsigned*)sm);
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2 offset:1024\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep) : "v"(voff), "s"(src), "s"(__builtin_amdgcn_readfirstlane(lds0)) : "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 2048; i += 64) out[i] = sm[i];
}
int main() {
    unsigned h[4096], *d, *o;
    for (int i = 0; i < 4096; ++i) h[i] = i;
    hipMalloc(&d, sizeof(h)); hipMalloc(&o, 2048 * 4);
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, 1, 64, 0, 0, d, o);
    unsigned r[2048];
    hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
    int first = -1;
    for (int i = 0; i < 2048; ++i) if (r[i] != 0xdeadbeef) { first = i; break; }
    printf("first written LDS dword %d holds src dword %u; dword 256 holds %u\n", first, first >= 0 ? r[first] : 0, r[256]);
    return 0;
}
