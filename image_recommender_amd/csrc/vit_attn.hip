// vit_attn.hip — multi-head self-attention of the DreamSim-architecture ViT forward, one HIP
// kernel on v_mfma_f32_16x16x32_bf16 (include/imgrec_vit.h vit_attention_bf16).
//
// The reference's towers (dreamsim ensemble: DINO / CLIP / OpenCLIP ViT-B/16,
// /root/reference/vector_scripts/create_dreamsim_vector.py:38-48, 51-93) run softmax(q k^T / 8) v
// over 197 tokens x 12 heads of 64 dims.  torch's SDPA on that shape reads q / k / v through the
// (B, N, 3, H, 64) qkv GEMM output's strides and pads the 197-token rows to its 128 / 256 blocks:
// 351 us per call at batch 512 (profiles/r03/dreamsim_kernel_stats_gelu_lt.csv), 0.07 of the
// bf16 peak.  The whole 197 x 197 score matrix of one (image, head) fits in registers, so here
// one workgroup per (image, head) does it in one pass, with no online-softmax rescaling:
//
// * K and V (<= 256 tokens x 64 bf16 each) go to LDS once, 128-B rows with 16-B chunk c stored
//   at c ^ (row & 7): the ds_read_b128 K-fragment reads and the ds_read_b64_tr_b16 V-fragment
//   reads are both conflict-free on that image;
// * wave w takes 16-query blocks w, w + 4, ...; S^T = K Q^T, 16 keys x 16 queries per MFMA, so a
//   lane holds, for ONE query (lane & 15), 4 keys of every 16-key block: the row max and the row
//   sum are in-lane reductions plus two permlane swaps over the four lane quarters;
// * O^T = V^T P^T: the exponentiated scores ARE the B operand (converted to bf16 in place, the
//   k order permuted to the accumulator's row order), V^T comes from the transposed LDS read in
//   the same k order; each lane ends with 4 hd values of its query, scaled by 1 / row sum.
//
// Reads qkv (B, N, 3, H, 64) bf16 as the qkv Linear writes it and writes out (B, N, H * 64) bf16
// as the output projection reads it: no permute or transpose copies around the kernel.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "../../include/imgrec_vit.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int kHD = 64;          // head dim
constexpr int kRowB = kHD * 2;   // bytes per K / V row in LDS
constexpr int kWaves = 4;

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}

// byte offset of the 16-B chunk c of row r in the swizzled K / V image
__device__ __forceinline__ int img_off(int r, int c) { return r * kRowB + 16 * (c ^ (r & 7)); }

__device__ __forceinline__ float quarter_max(float x) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
    const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
}
__device__ __forceinline__ float quarter_sum(float x) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}

// Transposed 4 x 16 read (T10): lane 4q + p of each 16-lane group supplies row q, columns
// 4p .. 4p + 3; lane i receives column i of the 4 rows (the builtin: the compiler counts it in
// lgkmcnt like any LDS read).  Every lane of the wave must execute it (EXEC all ones).
__device__ __forceinline__ bf16x4 read_tr(const char* p) {
    const auto v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(uintptr_t)lds_addr(p));
    return __builtin_bit_cast(bf16x4, v);
}

// NKB = 16-token blocks (keys and queries); the kernel serves ntok <= 16 NKB tokens.
template <int NKB>
__global__ void __launch_bounds__(kWaves * 64) __attribute__((amdgpu_waves_per_eu(3)))
attn_kernel(const uint16_t* __restrict__ qkv, int ntok, int heads, float scale_log2,
            uint16_t* __restrict__ out) {
    constexpr int kNKS = (NKB + 1) / 2;            // 32-key steps of P V
    constexpr int kRows = NKB * 16;
    __shared__ __attribute__((aligned(16))) char smem[2 * kRows * kRowB];
    char* const sk = smem;
    char* const sv = smem + kRows * kRowB;

    const int bh = blockIdx.x;
    const int b = bh / heads, h = bh - b * heads;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lc = lane & 15, lq = lane >> 4;
    const int64_t tok_stride = (int64_t)3 * heads * kHD;            // elements per token row
    const uint16_t* const base = qkv + (int64_t)b * ntok * tok_stride + (int64_t)h * kHD;
    const int64_t koff = (int64_t)heads * kHD, voff = 2 * koff;

    // ---- K and V of this (image, head) into LDS, stored swizzled; rows >= ntok are zero.  Every
    // load of both is issued before the first LDS store (K's stores waiting on K's loads before V's
    // loads went out cost one more HBM round trip per workgroup)
    {
        constexpr int kChunks = kRows * 8;
        constexpr int kPer = (kChunks + kWaves * 64 - 1) / (kWaves * 64);
        uint4 rr[2][kPer];
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const int64_t moff = m == 0 ? koff : voff;
#pragma unroll
            for (int j = 0; j < kPer; ++j) {
                const int i = tid + j * kWaves * 64, r = i >> 3, c = i & 7;
                // rows past the last token load the last token's row (in bounds) and store zeros
                rr[m][j] = *reinterpret_cast<const uint4*>(base + (int64_t)min(r, ntok - 1) * tok_stride + 8 * c + moff);
                if (r >= ntok) rr[m][j] = make_uint4(0u, 0u, 0u, 0u);
            }
        }
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            char* const dst = m == 0 ? sk : sv;
#pragma unroll
            for (int j = 0; j < kPer; ++j) {
                const int i = tid + j * kWaves * 64, r = i >> 3, c = i & 7;
                if (i < kChunks) *reinterpret_cast<uint4*>(dst + img_off(r, c)) = rr[m][j];
            }
        }
    }

    // Q fragments of a query block: lane (lc, lq) holds dims 8 lq .. + 7 (k-step 0) and
    // 32 + 8 lq .. + 7 (k-step 1) of query 16 qb + lc
    auto load_q = [&](int qb, uint4 (&qf)[2]) {
        const int tq = 16 * qb + lc;
        qf[0] = qf[1] = make_uint4(0u, 0u, 0u, 0u);
        if (tq < ntok) {
            const uint16_t* src = base + (int64_t)tq * tok_stride + 8 * lq;
            qf[0] = *reinterpret_cast<const uint4*>(src);
            qf[1] = *reinterpret_cast<const uint4*>(src + 32);
        }
    };
    uint4 qf[2];
    if (wave < NKB) load_q(wave, qf);
    __syncthreads();

    // K fragment of key block kb, k-step c: row 16 kb + lc, logical chunk 4 c + lq
    const int kfo[2] = {img_off(lc, lq), img_off(lc, 4 + lq)};
    // V^T fragment of 32-key step ks, half e (keys 32 ks + 16 e + 4 lq + q), hd block hb:
    // lane 4q + p of its group reads row 32 ks + 16 e + 4 lq + q, columns 16 hb + 4 p .. + 3
    const int q4 = lc >> 2, p4 = lc & 3;

    for (int qb = wave; qb < NKB; qb += kWaves) {
        // S^T block kb: lane holds keys 16 kb + 4 lq + i (i = 0..3) of query 16 qb + lc.
        // Fragments of block kb + 1 are read under block kb's two MFMAs (the scheduling barrier
        // keeps the compiler from hoisting all 2 NKB reads: 4 NKB more registers would not fit
        // three waves per SIMD)
        float s[NKB][4];
        uint4 a[2][2];
        a[0][0] = *reinterpret_cast<const uint4*>(sk + kfo[0]);
        a[0][1] = *reinterpret_cast<const uint4*>(sk + kfo[1]);
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
            if (kb + 1 < NKB) {
                const char* kp = sk + (kb + 1) * 16 * kRowB;
                a[(kb + 1) & 1][0] = *reinterpret_cast<const uint4*>(kp + kfo[0]);
                a[(kb + 1) & 1][1] = *reinterpret_cast<const uint4*>(kp + kfo[1]);
            }
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[kb & 1][0]),
                                                          __builtin_bit_cast(bf16x8, qf[0]), acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[kb & 1][1]),
                                                          __builtin_bit_cast(bf16x8, qf[1]), acc, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 4; ++i) s[kb][i] = acc[i];
            __builtin_amdgcn_sched_barrier(0);
        }
        const int t = 16 * qb + lc;
        // the next block's Q under this block's softmax and P V
        if (qb + kWaves < NKB) load_q(qb + kWaves, qf);

        // softmax numerator exp2((s - max) * scale * log2 e); only the last key block can hold
        // keys >= ntok: -inf there, so exp2 gives 0
        const int kpad = 16 * (NKB - 1) + 4 * lq;
#pragma unroll
        for (int i = 0; i < 4; ++i) s[NKB - 1][i] = kpad + i < ntok ? s[NKB - 1][i] : -INFINITY;
        float m = -INFINITY;
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int i = 0; i < 4; ++i) m = fmaxf(m, s[kb][i]);
        m = quarter_max(m) * scale_log2;
        float sum = 0.f;
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float p = __builtin_amdgcn_exp2f(fmaf(s[kb][i], scale_log2, -m));
                s[kb][i] = p;
                sum += p;
            }
        const float inv = 1.f / quarter_sum(sum);

        // O^T = V^T P^T over 32-key steps: B element e of lane (lc, lq) = P of key
        // 32 ks + 4 lq + e (e < 4) / 32 ks + 16 + 4 lq + (e - 4)
        f32x4 o[4];
#pragma unroll
        for (int hb = 0; hb < 4; ++hb) o[hb] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < kNKS; ++ks) {
            bf16x8 pb;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                pb[i] = (__bf16)s[2 * ks][i];
                pb[4 + i] = 2 * ks + 1 < NKB ? (__bf16)s[2 * ks + 1][i] : (__bf16)0.f;
            }
            const int r0 = 32 * ks + 4 * lq + q4;
#pragma unroll
            for (int hb = 0; hb < 4; ++hb) {
                const int c = 2 * hb + (p4 >> 1), half = 8 * (p4 & 1);
                const bf16x4 lo = read_tr(sv + img_off(r0, c) + half);
                // a 32-key step past the last key block reads nothing (P is 0 there)
                const bf16x4 hi = 2 * ks + 1 < NKB ? read_tr(sv + img_off(r0 + 16, c) + half)
                                                   : (bf16x4){(__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
                const bf16x8 va = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                o[hb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pb, o[hb], 0, 0, 0);
            }
        }
        // lane holds hd 16 hb + 4 lq + i of query t
        if (t < ntok) {
            uint16_t* dst = out + ((int64_t)b * ntok + t) * heads * kHD + (int64_t)h * kHD + 4 * lq;
#pragma unroll
            for (int hb = 0; hb < 4; ++hb) {
                const bf16x4 v = {(__bf16)(o[hb][0] * inv), (__bf16)(o[hb][1] * inv),
                                  (__bf16)(o[hb][2] * inv), (__bf16)(o[hb][3] * inv)};
                *reinterpret_cast<bf16x4*>(dst + 16 * hb) = v;
            }
        }
    }
}

}  // namespace

extern "C" int vit_attention_bf16(const uint16_t* qkv, int64_t batch, int ntok, int heads,
                                  int head_dim, float scale, uint16_t* out, void* stream) {
    if (batch < 0 || ntok <= 0 || ntok > 256 || heads <= 0 || head_dim != kHD || !qkv || !out ||
        (((uintptr_t)qkv | (uintptr_t)out) & 15) || batch * heads > 0x7fffffff)
        return -1;
    if (batch == 0) return 0;
    const dim3 grid((unsigned)(batch * heads)), block(kWaves * 64);
    const hipStream_t st = (hipStream_t)stream;
    const float sl2 = scale * 1.4426950408889634f;
    switch ((ntok + 15) / 16) {
#define IMGREC_ATTN(N) case N: hipLaunchKernelGGL(attn_kernel<N>, grid, block, 0, st, qkv, ntok, heads, sl2, out); break;
        IMGREC_ATTN(1) IMGREC_ATTN(2) IMGREC_ATTN(3) IMGREC_ATTN(4) IMGREC_ATTN(5) IMGREC_ATTN(6)
        IMGREC_ATTN(7) IMGREC_ATTN(8) IMGREC_ATTN(9) IMGREC_ATTN(10) IMGREC_ATTN(11) IMGREC_ATTN(12)
        IMGREC_ATTN(13) IMGREC_ATTN(14) IMGREC_ATTN(15) IMGREC_ATTN(16)
#undef IMGREC_ATTN
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
