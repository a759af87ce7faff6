// vit_fused.hip — fused residual add + LayerNorm (+ bf16 cast) and QuickGELU for the
// DreamSim-architecture ViT forward (include/imgrec_vit.h).  In the unfused forward each block
// runs, around its four bf16 matrix products, an fp32 residual add, an fp32 LayerNorm and a bf16
// cast of the LayerNorm output twice, and QuickGELU as three bf16 elementwise kernels
// (profiles/r02/dreamsim_pipeline_kernel_stats.csv: ~33 % of the forward).  Here each is one pass:
// a wave per row holds the row in registers (dim <= 1024: 16 values per lane), adds the bf16
// delta, writes the new residual, reduces mean and variance with wave sums and writes the
// normalised row as bf16 — the bytes of one read and two writes instead of six passes.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "../../include/imgrec_vit.h"

namespace {

__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ uint16_t f32_to_bf16(float x) {          // round to nearest even
    const uint32_t u = __float_as_uint(x);
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int PER>
__global__ void __launch_bounds__(256)
add_ln_kernel(float* __restrict__ x, const uint16_t* __restrict__ delta, const float* __restrict__ g,
              const float* __restrict__ b, uint16_t* __restrict__ y, int64_t rows, int dim, float eps) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    float* xr = x + row * dim;
    float v[PER];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int c = lane + 64 * i;
        float t = 0.f;
        if (c < dim) {
            t = xr[c];
            if (delta) {
                t += bf16_to_f32(delta[row * dim + c]);
                xr[c] = t;
            }
        }
        v[i] = t;
        s += t;
    }
    const float mean = wave_sum(s) / (float)dim;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int c = lane + 64 * i;
        const float d = c < dim ? v[i] - mean : 0.f;
        q = fmaf(d, d, q);
    }
    const float rstd = rsqrtf(wave_sum(q) / (float)dim + eps);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int c = lane + 64 * i;
        if (c < dim) y[row * dim + c] = f32_to_bf16(fmaf((v[i] - mean) * rstd, g[c], b[c]));
    }
}

__global__ void __launch_bounds__(256) quick_gelu_kernel(uint16_t* __restrict__ h, int64_t n) {
    const int64_t i8 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
    if (i8 + 8 <= n) {
        uint4 w = *reinterpret_cast<const uint4*>(h + i8);
        uint32_t p[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float a = __uint_as_float(p[j] << 16), c = __uint_as_float(p[j] & 0xffff0000u);
            const uint32_t lo = f32_to_bf16(a / (1.f + __expf(-1.702f * a)));
            const uint32_t hi = f32_to_bf16(c / (1.f + __expf(-1.702f * c)));
            p[j] = lo | (hi << 16);
        }
        *reinterpret_cast<uint4*>(h + i8) = make_uint4(p[0], p[1], p[2], p[3]);
    } else {
        for (int64_t i = i8; i < n; ++i) {
            const float a = bf16_to_f32(h[i]);
            h[i] = f32_to_bf16(a / (1.f + __expf(-1.702f * a)));
        }
    }
}

// nn.GELU (erf form) in place: 16 bf16 per thread (two 16-B loads in flight), fp32 inside.
__device__ __forceinline__ uint32_t gelu2(uint32_t p) {
    const float a = __uint_as_float(p << 16), c = __uint_as_float(p & 0xffff0000u);
    const uint32_t lo = f32_to_bf16(0.5f * a * (1.f + erff(a * 0.70710678118654752f)));
    const uint32_t hi = f32_to_bf16(0.5f * c * (1.f + erff(c * 0.70710678118654752f)));
    return lo | (hi << 16);
}

__global__ void __launch_bounds__(256) gelu_kernel(uint16_t* __restrict__ h, int64_t n) {
    const int64_t i16 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16;
    if (i16 + 16 <= n) {
        uint4 w0 = *reinterpret_cast<const uint4*>(h + i16);
        uint4 w1 = *reinterpret_cast<const uint4*>(h + i16 + 8);
        w0 = make_uint4(gelu2(w0.x), gelu2(w0.y), gelu2(w0.z), gelu2(w0.w));
        w1 = make_uint4(gelu2(w1.x), gelu2(w1.y), gelu2(w1.z), gelu2(w1.w));
        *reinterpret_cast<uint4*>(h + i16) = w0;
        *reinterpret_cast<uint4*>(h + i16 + 8) = w1;
    } else {
        for (int64_t i = i16; i < n; ++i) {
            const float a = bf16_to_f32(h[i]);
            h[i] = f32_to_bf16(0.5f * a * (1.f + erff(a * 0.70710678118654752f)));
        }
    }
}

}  // namespace

extern "C" int vit_gelu_bf16(uint16_t* h, int64_t n, void* stream) {
    if (n < 0 || (n > 0 && !h) || ((uintptr_t)h & 15)) return -1;
    if (n == 0) return 0;
    const int64_t threads = (n + 15) / 16;
    hipLaunchKernelGGL(gelu_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, h, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int vit_add_layernorm_bf16(float* x, const uint16_t* delta, const float* gamma,
                                      const float* beta, uint16_t* y, int64_t rows, int dim,
                                      float eps, void* stream) {
    if (rows < 0 || dim <= 0 || dim > 1024 || !x || !gamma || !beta || !y) return -1;
    if (rows == 0) return 0;
    const dim3 grid((unsigned)((rows + 3) / 4)), block(256);
    const hipStream_t st = (hipStream_t)stream;
    if (dim <= 256)
        hipLaunchKernelGGL(add_ln_kernel<4>, grid, block, 0, st, x, delta, gamma, beta, y, rows, dim, eps);
    else if (dim <= 512)
        hipLaunchKernelGGL(add_ln_kernel<8>, grid, block, 0, st, x, delta, gamma, beta, y, rows, dim, eps);
    else if (dim <= 768)
        hipLaunchKernelGGL(add_ln_kernel<12>, grid, block, 0, st, x, delta, gamma, beta, y, rows, dim, eps);
    else
        hipLaunchKernelGGL(add_ln_kernel<16>, grid, block, 0, st, x, delta, gamma, beta, y, rows, dim, eps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int vit_quick_gelu_bf16(uint16_t* h, int64_t n, void* stream) {
    if (n < 0 || (n > 0 && !h) || ((uintptr_t)h & 15)) return -1;
    if (n == 0) return 0;
    const int64_t threads = (n + 7) / 8;
    hipLaunchKernelGGL(quick_gelu_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, h, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
