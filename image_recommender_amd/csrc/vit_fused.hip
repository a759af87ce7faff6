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

// The same for dim = 256 * CH (ViT-B: 768): each lane owns CH chunks of 4 CONTIGUOUS elements,
// so every access is one 16-B (fp32) or 8-B (bf16) vector per lane — 1 KiB / 512 B per wave
// instruction instead of the 256 B / 128 B of the lane-strided form (round 3: 221 us per call
// at 100,864 x 768 rows = 4.2 TB/s for that form, profiles/r03/).
template <int CH>
__global__ void __launch_bounds__(256)
add_ln_vec_kernel(float* __restrict__ x, const uint16_t* __restrict__ delta, const float* __restrict__ g,
                  const float* __restrict__ b, uint16_t* __restrict__ y, int64_t rows, float eps) {
    constexpr int dim = 256 * CH;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    float4* xr = reinterpret_cast<float4*>(x + row * dim);
    float4 v[CH];
    uint2 dl[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
        v[i] = xr[lane + 64 * i];
        if (delta) dl[i] = reinterpret_cast<const uint2*>(delta + row * dim)[lane + 64 * i];
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
        if (delta) {
            v[i].x += __uint_as_float(dl[i].x << 16);
            v[i].y += __uint_as_float(dl[i].x & 0xffff0000u);
            v[i].z += __uint_as_float(dl[i].y << 16);
            v[i].w += __uint_as_float(dl[i].y & 0xffff0000u);
            // (a non-temporal form of this store measured the same in the forward:
            // profiles/r05/vit_gemm/store_policy_forward/ab_vit_ln_residual_nt.jsonl)
            xr[lane + 64 * i] = v[i];
        }
        s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    }
    const float mean = wave_sum(s) / (float)dim;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
        const float d0 = v[i].x - mean, d1 = v[i].y - mean, d2 = v[i].z - mean, d3 = v[i].w - mean;
        q = fmaf(d0, d0, q); q = fmaf(d1, d1, q); q = fmaf(d2, d2, q); q = fmaf(d3, d3, q);
    }
    const float rstd = rsqrtf(wave_sum(q) / (float)dim + eps);
    uint2* yr = reinterpret_cast<uint2*>(y + row * dim);
#pragma unroll
    for (int i = 0; i < CH; ++i) {
        const float4 gg = reinterpret_cast<const float4*>(g)[lane + 64 * i];
        const float4 bb = reinterpret_cast<const float4*>(b)[lane + 64 * i];
        const uint32_t o0 = f32_to_bf16(fmaf((v[i].x - mean) * rstd, gg.x, bb.x));
        const uint32_t o1 = f32_to_bf16(fmaf((v[i].y - mean) * rstd, gg.y, bb.y));
        const uint32_t o2 = f32_to_bf16(fmaf((v[i].z - mean) * rstd, gg.z, bb.z));
        const uint32_t o3 = f32_to_bf16(fmaf((v[i].w - mean) * rstd, gg.w, bb.w));
        yr[lane + 64 * i] = make_uint2(o0 | (o1 << 16), o2 | (o3 << 16));
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

// Patch extraction of the input normalisation + stride-p patch conv as a GEMM: image (B, 3, H, W)
// fp32 in [0, 1] -> ((x - mean[c]) / std[c]) as bf16 patches (B, (H/p)(W/p), 3 p p), each patch
// laid out (c, kh, kw) like the conv weight.  One thread per 8 consecutive patch elements (half a
// patch row for p = 16): two 16-B loads, one 16-B store.
__global__ void __launch_bounds__(256)
patchify_kernel(const float* __restrict__ img, int64_t B, int H, int W, int p,
                const float* __restrict__ mean, const float* __restrict__ std_,
                uint16_t* __restrict__ out) {
    const int gw = W / p, np = (H / p) * gw, pe = 3 * p * p;
    const int64_t i8 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
    if (i8 >= B * (int64_t)np * pe) return;
    const int e = (int)(i8 % pe);
    const int64_t bp = i8 / pe;
    const int pi = (int)(bp % np);
    const int64_t bi = bp / np;
    const int c = e / (p * p), kh = (e / p) % p, kw = e % p;
    const int ph = pi / gw, pw = pi % gw;
    const float* src = img + ((bi * 3 + c) * H + (int64_t)(ph * p + kh)) * W + pw * p + kw;
    const float4 a = *reinterpret_cast<const float4*>(src);
    const float4 b = *reinterpret_cast<const float4*>(src + 4);
    const float m = mean[c], sd = std_[c];
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
        w[j] = (uint32_t)f32_to_bf16((v[2 * j] - m) / sd) | ((uint32_t)f32_to_bf16((v[2 * j + 1] - m) / sd) << 16);
    *reinterpret_cast<uint4*>(out + i8) = make_uint4(w[0], w[1], w[2], w[3]);
}

// Token rows of a tower: out (B, np + 1, C) fp32 = [cls + pos[0] ; bf16 patch embeddings + pos[1:]]
// (torch.cat([cls, x.float()], 1) + pos in one pass); four elements per thread.
__global__ void __launch_bounds__(256)
tokens_kernel(const uint16_t* __restrict__ pe, const float* __restrict__ cls,
              const float* __restrict__ pos, int64_t B, int np, int C, float* __restrict__ out) {
    const int64_t i4 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    const int64_t per = (int64_t)(np + 1) * C;
    if (i4 >= B * per) return;
    const int64_t bi = i4 / per;
    const int64_t rc = i4 - bi * per;
    const int r = (int)(rc / C), c = (int)(rc % C);
    const float4 ps = *reinterpret_cast<const float4*>(pos + rc);
    float4 o;
    if (r == 0) {
        const float4 cl = *reinterpret_cast<const float4*>(cls + c);
        o = make_float4(cl.x + ps.x, cl.y + ps.y, cl.z + ps.z, cl.w + ps.w);
    } else {
        const uint2 h = *reinterpret_cast<const uint2*>(pe + (bi * np + (r - 1)) * (int64_t)C + c);
        o = make_float4(__uint_as_float(h.x << 16) + ps.x, __uint_as_float(h.x & 0xffff0000u) + ps.y,
                        __uint_as_float(h.y << 16) + ps.z, __uint_as_float(h.y & 0xffff0000u) + ps.w);
    }
    *reinterpret_cast<float4*>(out + i4) = o;
}

}  // namespace

extern "C" int vit_patchify_bf16(const float* img, int64_t batch, int height, int width, int patch,
                                 const float* mean, const float* std_, uint16_t* out, void* stream) {
    if (batch < 0 || patch <= 0 || patch % 8 != 0 || height % patch != 0 || width % patch != 0 ||
        !img || !mean || !std_ || !out || ((uintptr_t)img & 15) || ((uintptr_t)out & 15))
        return -1;
    const int64_t n = batch * (int64_t)(height / patch) * (width / patch) * 3 * patch * patch;
    if (n == 0) return 0;
    const int64_t threads = n / 8;
    hipLaunchKernelGGL(patchify_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, img, batch, height, width, patch, mean, std_, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int vit_tokens_f32(const uint16_t* patch_emb, const float* cls, const float* pos,
                              int64_t batch, int npatch, int dim, float* out, void* stream) {
    if (batch < 0 || npatch < 0 || dim <= 0 || dim % 4 != 0 || !patch_emb || !cls || !pos || !out ||
        (((uintptr_t)cls | (uintptr_t)pos | (uintptr_t)out) & 15) || ((uintptr_t)patch_emb & 7))
        return -1;
    const int64_t n = batch * (int64_t)(npatch + 1) * dim;
    if (n == 0) return 0;
    hipLaunchKernelGGL(tokens_kernel, dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, patch_emb, cls, pos, batch, npatch, dim, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

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
    const bool aligned = (((uintptr_t)x | (uintptr_t)gamma | (uintptr_t)beta) & 15) == 0 &&
                         (((uintptr_t)delta | (uintptr_t)y) & 7) == 0;
    if (aligned && dim % 256 == 0) {
        switch (dim / 256) {
            case 1: hipLaunchKernelGGL(add_ln_vec_kernel<1>, grid, block, 0, st, x, delta, gamma, beta, y, rows, eps); break;
            case 2: hipLaunchKernelGGL(add_ln_vec_kernel<2>, grid, block, 0, st, x, delta, gamma, beta, y, rows, eps); break;
            case 3: hipLaunchKernelGGL(add_ln_vec_kernel<3>, grid, block, 0, st, x, delta, gamma, beta, y, rows, eps); break;
            default: hipLaunchKernelGGL(add_ln_vec_kernel<4>, grid, block, 0, st, x, delta, gamma, beta, y, rows, eps); break;
        }
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
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
