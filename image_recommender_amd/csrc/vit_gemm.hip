// vit_gemm.hip — the bf16 matrix products of the DreamSim-architecture ViT forward,
// Y = act(X W^T + b), as one 256 x 256-tile kernel on v_mfma_f32_16x16x32_bf16 (gfx950)
// (include/imgrec_vit.h vit_linear_bf16).
//
// The reference embeds images with dreamsim's ensemble of three ViT-B/16 towers
// (/root/reference/vector_scripts/create_dreamsim_vector.py:38-48, 51-93, `model.embed`); at
// batch 512 each of its 36 blocks runs four GEMMs over M = 100,864 token rows (qkv 768 -> 2304,
// proj 768 -> 768, fc1 768 -> 3072 + GELU, fc2 3072 -> 768).  hipBLASLt runs them at 0.39 of the
// dense bf16 peak (its MT256x256x64 MI16x16 kernel, 72 % of the forward:
// profiles/r03/dreamsim_hip_attn/kernel_stats.csv), while the k-NN candidate kernel's main loop
// (knn_b16w.hip) sustains 0.53 of the peak on the same MFMA form.  This is that main loop with a
// GEMM epilogue:
//
// * roles: the token rows X (M x K, the large operand) are the streamed "corpus" — 256-row tiles,
//   each workgroup walking the tiles of its token split s, s + nsplit, ...; the weight rows W
//   (N x K, nn.Linear's layout, 2-5 MB) are the workgroup's fixed block of 256 output features,
//   re-staged per stage from L2.  The workgroups sharing a token split sit on one XCD (the
//   bijective XCD map of knn_b16w.hip), so a token tile comes from HBM about once per XCD;
// * 64-deep stages of both 256-row operands (32 KiB each) through a two-slot LDS ring by LDS-DMA,
//   XOR-swizzled rows, fragments read one ds_read_b128 per MFMA gap, one barrier per stage; waves
//   0-3 move the token tile, 4-7 the weight tile (their issue deferred into the next stage);
// * the MFMA takes the WEIGHT fragment as its A operand and the token fragment as B, so a lane's
//   accumulator holds four consecutive output features of one token (row = 4 (lane >> 4) + reg,
//   col = lane & 15): the epilogue adds the bias, applies the activation in fp32, rounds to bf16,
//   pairs lane quarters by v_permlane16_swap and stores 16 contiguous bytes per (token, 8
//   features) — 16 stores per lane per tile;
// * 8 waves along the features (32 each) x all 256 tokens of the tile: 16 token blocks x 2
//   feature blocks of 16 x 16, 128 accumulator registers per lane.
// Requirements (checked by the launcher): K a multiple of 64, N a multiple of 256, 16-B aligned
// operands; any M (the last tile's rows past M are staged from row M - 1 and never stored).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include <type_traits>

#include "../../include/imgrec_vit.h"
#include "lds_dma.h"

namespace imgrec {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int kNW = 8;                    // waves, all along the features
constexpr int kBM = 256;                  // token rows per tile
constexpr int kBN = 256;                  // output features per workgroup
constexpr int kFW = kBN / kNW;            // 32 features per wave
constexpr int kRB = kBM / 16;             // 16-token blocks per tile
constexpr int kBKW = 32;                  // 32-bit words (2 bf16) per staged row: 64-deep stages
constexpr int kRowB = kBKW * 4;           // bytes per staged row
constexpr int kCPR = kBKW / 4;            // 16-B chunks per staged row
constexpr int kRPP = 64 / kCPR;           // rows per one-KiB DMA piece
constexpr int kRPB = 64 / kBKW;           // rows per 256-B bank row
constexpr int kSA = kBM * kRowB;          // token stage bytes
constexpr int kSB = kBN * kRowB;          // weight stage bytes
constexpr int kStage = kSA + kSB;
constexpr int kLPW = (kBM + kBN) / kRPP / kNW;   // DMA pieces per wave per stage
constexpr int kLDS = 2 * kStage;          // two-slot ring
constexpr int kDeferQ = 3;                // weight waves issue after this quad of the next stage
// Measurement builds only (tools/vit_gemm_tiles.py): 1 = the epilogue computed but its stores
// skipped (data-dependent predicate, never true in practice), 2 = no epilogue at all (one
// checksum store per tile)
#ifndef IMGREC_VIT_EPI_EXP
#define IMGREC_VIT_EPI_EXP 0
#endif
// The output stores are non-temporal (IMGREC_VIT_NT_STORE, default on) and the stage after a
// full tile's epilogue waits for its own DMA only (IMGREC_VIT_STORE_WAIT, default on: vmcnt(16) —
// the lane's 16 output stores stay in flight; the weight waves issue the DMA they would defer into
// that stage before the epilogue instead).  Every CU ends its tiles at the same moment, so a tile
// end is a 32 MB burst of output stores; waiting for it at the next stage and leaving the lines
// dirty in the L2 the operand stream runs through cost up to a third of the K = 768 GEMMs
// (stores skipped: qkv 0.364 -> 0.271 ms).  Measured at batch 512 (profiles/r05/vit_gemm/), each
// GEMM alone: qkv 0.357 -> 0.315 ms, proj 0.138 -> 0.110, fc1 + GELU 0.494 -> 0.456, fc2 0.416 ->
// 0.407; inside the forward the gain mostly does not survive (the next kernel reads an output
// that was streamed past the MALL; per kernel in the forward the qkv GEMM even got slower,
// forward_kernels/): batch 512 on one box 7,620 images/s (round-4 stores) -> 7,640 (non-temporal
// from 192 MB: qkv and fc1) -> 7,690 (from 512 MB: fc1's 620 MB output only, the default)
// (store_policy_forward/).
// Output store policy (IMGREC_VIT_NT_STORE): 0 plain, 1 non-temporal, 2 non-temporal only when
// the output exceeds kNtMinBytes (IMGREC_VIT_NT_MIN_MB).
#ifndef IMGREC_VIT_NT_STORE
#define IMGREC_VIT_NT_STORE 2
#endif
#ifndef IMGREC_VIT_NT_MIN_MB
#define IMGREC_VIT_NT_MIN_MB 512
#endif
constexpr int64_t kNtMinBytes = (int64_t)IMGREC_VIT_NT_MIN_MB << 20;
#ifndef IMGREC_VIT_STORE_WAIT
#define IMGREC_VIT_STORE_WAIT 1
#endif
static_assert(kBKW == 32 && kCPR == 8 && kRPP == 8 && kRPB == 2, "stage geometry");
static_assert(kLPW == 8, "pieces go out in two dma4x groups");
static_assert(kLDS <= 160 * 1024, "LDS budget");

// The sigmoid forms divide by v_rcp_f32 (1 ulp) instead of the IEEE division sequence (scale,
// Newton steps, fixup: ~10 VALU per element — most of fc1's epilogue); the result is rounded to
// bf16 (2^-9) right after, so the ulp never shows.
template <int ACT>
__device__ __forceinline__ float activate(float x) {
    if constexpr (ACT == VIT_ACT_GELU_ERF) return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
    if constexpr (ACT == VIT_ACT_GELU_TANH) {
        // 0.5 x (1 + tanh(u)) = x / (1 + exp(-2u)), u = sqrt(2/pi) (x + 0.044715 x^3)
        const float u = 0.7978845608028654f * fmaf(0.044715f * x * x, x, x);
        return x * __builtin_amdgcn_rcpf(1.f + __expf(-2.f * u));
    }
    if constexpr (ACT == VIT_ACT_QUICK_GELU) return x * __builtin_amdgcn_rcpf(1.f + __expf(-1.702f * x));
    return x;
}

template <int ACT, bool NT>
__global__ void __launch_bounds__(512, 2)
vit_gemm_kernel(const uint32_t* __restrict__ xw, const uint32_t* __restrict__ ww,
                const float* __restrict__ bias, uint16_t* __restrict__ y, int M, int dw, int N,
                int nsplit, int nqb) {
    __shared__ __attribute__((aligned(16))) char smem[kLDS];

    // XCD-aware bijective block -> (feature block, token split) map (knn_b16w.hip): the G
    // feature-block workgroups of a token split get consecutive ids on one XCD
    const int nwg = gridDim.x, wg = blockIdx.x;
    const int xcd = wg & 7, qq = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (wg >> 3);
    const int G = (nqb % 4 == 0) ? 4 : nqb;
    const int qbg = wgid / (nsplit * G), rem = wgid - qbg * (nsplit * G);
    const int split = rem / G;
    const int qb = qbg * G + rem % G;
    const int ntile = (M + kBM - 1) / kBM;
    const int cnt = split < ntile ? (ntile - split + nsplit - 1) / nsplit : 0;
    auto row0_of = [&](int t) { return (split + t * nsplit) * kBM; };
    auto valid_of = [&](int t) { return min(kBM, M - row0_of(t)); };

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lc = lane & 15, lq = lane >> 4;

    // ---- DMA: waves 0-3 the token tile, 4-7 the weight tile
    const bool isA = wave < 4;
    if (!isA) __builtin_amdgcn_s_setprio(1);
    const int pbase = (isA ? wave : wave - 4) * kLPW;
    const int prow = lane / kCPR, pchk = lane % kCPR;
    uint32_t vpar[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int r = (pbase + e) * kRPP + prow;
        vpar[e] = (uint32_t)r * (uint32_t)(dw * 4) + 16u * (uint32_t)(pchk ^ ((r / kRPB) % kCPR));
    }
    const uint32_t kPS = (uint32_t)(kRPP * dw * 4);
    auto voff_of = [&](int j) { return vpar[j & 1] + (uint32_t)(j & ~1) * kPS - 1024u * (uint32_t)(j & 3); };
    const uint32_t smem0 = lds_u32(smem);
    const uint32_t pdst = (uint32_t)((isA ? 0 : kSA) + pbase * 1024);

    const int fsw = (lc / kRPB) % kCPR;
    int aoff[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) aoff[c] = lc * kRowB + 16 * ((4 * c + lq) ^ fsw);
    const int boff = kSA + wave * kFW * kRowB;

    const int nst = dw / kBKW;
    const int total = cnt * nst;
    const uint32_t* wblk = ww + (size_t)qb * kBN * dw;

    // issue cursor: stage c_is of tile c_it
    int c_it = 0, c_is = 0;
    const uint32_t* c_tile = isA ? xw + (size_t)row0_of(0) * dw : wblk;
    int c_valid = isA ? valid_of(0) : kBM;
    auto issue = [&](int g) __attribute__((always_inline)) {
        const uint32_t* src = c_tile + c_is * kBKW;
        const uint32_t dst = smem0 + (uint32_t)((g & 1) * kStage) + pdst;
        if (!isA || c_valid == kBM) {
#pragma unroll
            for (int h = 0; h < kLPW / 4; ++h)
                dma4x(src, dst + 4096u * h, voff_of(4 * h), voff_of(4 * h + 1), voff_of(4 * h + 2),
                      voff_of(4 * h + 3));
        } else {
            // the split's last, partial tile: pieces past M are skipped, rows past M inside the
            // last live piece are staged from row M - 1 (never stored)
#pragma unroll
            for (int j = 0; j < kLPW; ++j) {
                const int r0 = (pbase + j) * kRPP;
                if (r0 < c_valid) {
                    const int r = r0 + prow, rs = min(r, c_valid - 1);
                    const uint32_t v = (uint32_t)rs * (uint32_t)(dw * 4) +
                                       16u * (uint32_t)(pchk ^ ((r / kRPB) % kCPR)) - 1024u * (uint32_t)(j & 3);
                    dma1_at(j, src, dst + 4096u * (j / 4), v);
                }
            }
        }
        if (++c_is == nst) {
            c_is = 0;
            ++c_it;
            if (isA && c_it < cnt) {
                c_tile = xw + (size_t)row0_of(c_it) * dw;
                c_valid = valid_of(c_it);
            }
        }
    };

    // quad q of a stage: k-step q >> 2, token blocks 4 (q & 3) .. + 3
    auto read_a = [&](const char* sb, int q, u32x4 (&fa)[4]) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            fa[j] = *reinterpret_cast<const u32x4*>(sb + aoff[q >> 2] + (4 * (q & 3) + j) * 16 * kRowB);
    };
    auto read_b = [&](const char* sb, int c, u32x4 (&fb)[2]) __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < 2; ++h) fb[h] = *reinterpret_cast<const u32x4*>(sb + aoff[c] + boff + h * 16 * kRowB);
    };
    // weight fragment as the MFMA's A operand: acc[token block][feature block] holds
    // D[feature 4 lq + reg][token lc]
    auto mfma_quad = [&](f32x4 (&acc)[kRB][2], const u32x4 (&fa)[4], const u32x4 (&fb)[2], int q) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                acc[4 * (q & 3) + j][h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                    __builtin_bit_cast(bf16x8, fb[h]), __builtin_bit_cast(bf16x8, fa[j]), acc[4 * (q & 3) + j][h], 0, 0, 0);
    };

    // bias of this lane's 8 output features (feature blocks h = 0, 1; 4 consecutive each)
    const int fcol = qb * kBN + wave * kFW + 4 * lq;
    f32x4 bv[2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
        bv[h] = bias ? *reinterpret_cast<const f32x4*>(bias + fcol + 16 * h) : (f32x4){0.f, 0.f, 0.f, 0.f};

    u32x4 fa[2][4], fb[2][2];
    int g = 0;
    int pend = -1;
    if (total > 0) {
        issue(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier_lds();
        if (total > 1) issue(1);
        read_a(smem, 0, fa[0]);
        read_b(smem, 0, fb[0]);
    }
    bool prev_full = false;            // the previous tile's epilogue issued all 16 stores
    for (int t = 0; t < cnt; ++t) {
        f32x4 acc[kRB][2];
#pragma unroll
        for (int rb = 0; rb < kRB; ++rb)
#pragma unroll
            for (int h = 0; h < 2; ++h) acc[rb][h] = (f32x4){0.f, 0.f, 0.f, 0.f};
        const int row0 = row0_of(t);
        const int valid = valid_of(t);
        // live quad rows (64 tokens each): a partial last tile runs the MFMAs of its live rows only
        const int nlive = (valid + 63) >> 6;
        auto stage_loop = [&](auto nr_tag) __attribute__((always_inline)) {
            constexpr int NR = decltype(nr_tag)::value, L = 2 * NR;
            for (int s = 0; s < nst; ++s, ++g) {
                const char* sb = smem + (g & 1) * kStage;
#pragma unroll
                for (int i = 0; i + 1 < L; ++i) {
                    read_a(sb, 4 * ((i + 1) / NR) + (i + 1) % NR, fa[(i + 1) & 1]);
                    if (i == NR - 1) read_b(sb, 1, fb[1]);
                    mfma_quad(acc, fa[i & 1], fb[i / NR], 4 * (i / NR) + i % NR);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
                    }
                    if (i == NR - 1) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                    } else {
                        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    if (i == (kDeferQ < L - 2 ? kDeferQ : L - 2) && pend >= 0) {
                        __builtin_amdgcn_sched_barrier(0);
                        issue(pend);
                        pend = -1;
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
                // vmcnt(16): the youngest 16 vector-memory ops of a lane are the previous tile's 16
                // output stores (one per 16-token block), so the stage's own DMA has landed.  Any
                // epilogue that stores differently (the IMGREC_VIT_EPI_EXP measurement builds)
                // waits for everything.
                static_assert(kRB == 16, "vmcnt(16) counts one output store per 16-token block");
                if (IMGREC_VIT_STORE_WAIT && IMGREC_VIT_EPI_EXP == 0 && s == 0 && prev_full)
                    asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)" ::: "memory");
                else
                    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
                barrier_lds();
                __builtin_amdgcn_sched_barrier(0);
                if (s + 1 < nst) {
                    const char* nb = smem + ((g + 1) & 1) * kStage;
                    read_a(nb, 0, fa[0]);
                    read_b(nb, 0, fb[0]);
                }
                if (g + 2 < total) {
                    // (IMGREC_VIT_STORE_WAIT: a tile's last stage issues for the weight waves too,
                    // so the next tile's first stage waits on no DMA issued after the stores)
                    if (isA || (IMGREC_VIT_STORE_WAIT && s + 1 == nst)) issue(g + 2);
                    else pend = g + 2;
                }
                mfma_quad(acc, fa[1], fb[1], 4 + NR - 1);
            }
        };
        if (nlive >= 4) stage_loop(std::integral_constant<int, 4>{});
        else if (nlive == 3) stage_loop(std::integral_constant<int, 3>{});
        else if (nlive == 2) stage_loop(std::integral_constant<int, 2>{});
        else stage_loop(std::integral_constant<int, 1>{});

        // ---- epilogue: bias, activation, bf16; then one 16-B store per (token, 8 features): a
        // lane holds features 4 lq .. + 3 of both feature blocks h = 0, 1 (16 apart), and a
        // v_permlane16_swap per dword pairs lane quarters lq, lq + 1 (cdna_hip_programming.md T21,
        // the 16-lane form): even quarters end with h = 0's features 4 lq .. 4 lq + 7, odd ones with
        // h = 1's 16 + 4 (lq - 1) .. + 7 — half the store instructions of 8-B stores, whose issue
        // rate, not HBM, sets this tail
#if IMGREC_VIT_EPI_EXP == 2
        {
            float cs = 0.f;
#pragma unroll
            for (int rb = 0; rb < kRB; ++rb) cs += acc[rb][0][0] + acc[rb][1][3];
            if (__float_as_uint(cs) == 0x7f812345u) y[lane] = 1;
        }
#else
#pragma unroll
        for (int rb = 0; rb < kRB; ++rb) {
            const int tok = row0 + 16 * rb + lc;
            uint32_t o[2][2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const f32x4 v = acc[rb][h] + bv[h];
                const f32x2 lo = (f32x2){activate<ACT>(v[0]), activate<ACT>(v[1])};
                const f32x2 hi = (f32x2){activate<ACT>(v[2]), activate<ACT>(v[3])};
                o[h][0] = __builtin_bit_cast(uint32_t, __builtin_convertvector(lo, bf16x2));
                o[h][1] = __builtin_bit_cast(uint32_t, __builtin_convertvector(hi, bf16x2));
            }
#pragma unroll
            for (int d = 0; d < 2; ++d) {
                const auto r = __builtin_amdgcn_permlane16_swap(o[0][d], o[1][d], false, false);
                o[0][d] = r[0];
                o[1][d] = r[1];
            }
#if IMGREC_VIT_EPI_EXP == 1
            if ((o[0][0] ^ o[1][1]) == 0x12345678u && 16 * rb + lc < valid)
#else
            if (16 * rb + lc < valid)
#endif
            {
                uint4* dst = reinterpret_cast<uint4*>(y + (size_t)tok * N + fcol + ((lq & 1) ? 12 : 0));
                if constexpr (NT)
                    __builtin_nontemporal_store((u32x4){o[0][0], o[0][1], o[1][0], o[1][1]},
                                                reinterpret_cast<u32x4*>(dst));
                else
                    *dst = make_uint4(o[0][0], o[0][1], o[1][0], o[1][1]);
            }
        }
#endif
        prev_full = valid == kBM;
        if (g < total) {
            read_a(smem + (g & 1) * kStage, 0, fa[0]);
            read_b(smem + (g & 1) * kStage, 0, fb[0]);
        }
    }
}

}  // namespace

// Token splits for N / 256 feature blocks on `cus` CUs (one 8-wave workgroup per CU): the fewest
// tiles per split the CUs allow, then as few splits as give that (less L2 contention, same time).
int vit_gemm_splits(int M, int N, int cus) {
    const int ntile = (M + kBM - 1) / kBM, nqb = N / kBN;
    const int most = cus / nqb > 0 ? cus / nqb : 1;
    const int per = (ntile + most - 1) / most;
    return (ntile + per - 1) / per;
}

}  // namespace imgrec

extern "C" int vit_linear_bf16(const uint16_t* x, const uint16_t* w, const float* bias, int64_t m,
                               int k, int n, int act, uint16_t* y, void* stream) {
    using namespace imgrec;
    if (!x || !w || !y || m < 0 || k <= 0 || n <= 0) return -1;
    if (k % 64 != 0 || n % kBN != 0 || m > INT32_MAX / 2) return -1;
    if (((uintptr_t)x | (uintptr_t)w | (uintptr_t)y | (uintptr_t)bias) & 15) return -1;
    // 32-bit DMA offsets: a tile's rows and a weight block stay below 4 GiB
    if ((int64_t)kBM * k * 2 >= ((int64_t)1 << 31)) return -1;
    if (m == 0) return 0;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
    const int nqb = n / kBN;
    const int nsplit = vit_gemm_splits((int)m, n, cus);
    const dim3 grid((unsigned)(nqb * nsplit)), block(kNW * 64);
    const uint32_t* xw = reinterpret_cast<const uint32_t*>(x);
    const uint32_t* ww = reinterpret_cast<const uint32_t*>(w);
    const hipStream_t st = (hipStream_t)stream;
    const bool nt = IMGREC_VIT_NT_STORE == 1 || (IMGREC_VIT_NT_STORE == 2 && m * n * 2 > kNtMinBytes);
#define IMGREC_VIT_LAUNCH(A)                                                                              \
    do {                                                                                                  \
        if (nt) hipLaunchKernelGGL((vit_gemm_kernel<A, true>), grid, block, 0, st, xw, ww, bias, y, (int)m, k / 2, n, nsplit, nqb); \
        else hipLaunchKernelGGL((vit_gemm_kernel<A, false>), grid, block, 0, st, xw, ww, bias, y, (int)m, k / 2, n, nsplit, nqb); \
    } while (0)
    switch (act) {
        case VIT_ACT_NONE: IMGREC_VIT_LAUNCH(VIT_ACT_NONE); break;
        case VIT_ACT_GELU_ERF: IMGREC_VIT_LAUNCH(VIT_ACT_GELU_ERF); break;
        case VIT_ACT_GELU_TANH: IMGREC_VIT_LAUNCH(VIT_ACT_GELU_TANH); break;
        case VIT_ACT_QUICK_GELU: IMGREC_VIT_LAUNCH(VIT_ACT_QUICK_GELU); break;
        default: return -1;
    }
#undef IMGREC_VIT_LAUNCH
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
