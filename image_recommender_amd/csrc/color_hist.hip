// color_hist.hip — per-image RGB histogram on gfx950 (row A15 of SURVEY.md §8a).
//
// Restates /root/reference/vector_scripts/create_color_vector.py:46-51 (cv2.calcHist with
// `bins` uniform bins over [0, 256) per channel, R|G|B concatenated, L2-normalised) for a batch of
// decoded images.  HBM-bound byte work: one workgroup per image streams the image's bytes with
// 16-B loads; every thread counts into its OWN column of an LDS histogram laid out
// [bin][thread] (u32, ds_add_u32), so no two lanes ever touch the same word and the 32 lanes of a
// half-wave always hit 32 different banks — no contention however skewed the image is.  The
// per-thread columns are then summed by wave reductions, normalised and written out.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include <algorithm>
#include <climits>
#include <cstdarg>
#include <cstdio>
#include <string>

#include "../../include/imgrec_color.h"

namespace {

constexpr int NT = 256;

__global__ void __launch_bounds__(NT)
color_hist_kernel(const uint8_t* __restrict__ pix, const int64_t* __restrict__ offsets,
                  const int64_t* __restrict__ npix, int bins, float* __restrict__ out,
                  uint32_t* __restrict__ counts) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];   // [3*bins][NT]
    const int tid = threadIdx.x;
    const int nb = 3 * bins;
    for (int i = tid; i < nb * NT; i += NT) hist[i] = 0u;
    __syncthreads();

    const int64_t img = blockIdx.x;
    const int64_t off = offsets[img];
    const int64_t nbytes = 3 * npix[img];
    const uint8_t* base = pix + off;

    auto count = [&](int c, uint32_t v) {
        const int b = (int)((v * (uint32_t)bins) >> 8);
        atomicAdd(&hist[(c * bins + b) * NT + tid], 1u);
    };

    // head: bytes before the first 16-B aligned address
    const int64_t head = std::min<int64_t>(nbytes, (int64_t)((16 - ((uintptr_t)base & 15)) & 15));
    if (tid < head) count((int)(tid % 3), base[tid]);
    // aligned body, 16 bytes per thread per iteration
    const int64_t body = (nbytes - head) & ~(int64_t)15;
    const uint4* vb = reinterpret_cast<const uint4*>(base + head);
    const int64_t nvec = body >> 4;
    // channel of the first byte of vector i is (head + 16 i) % 3; a stride of NT vectors moves it
    // by 16 * NT = 4096 = 1 (mod 3)
    int cv = (int)((head + (int64_t)tid * 16) % 3);
    for (int64_t i = tid; i < nvec; i += NT, cv = (cv == 2) ? 0 : cv + 1) {
        const uint4 w = vb[i];
        int c = cv;
        const uint32_t words[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                count(c, (words[q] >> (8 * j)) & 0xffu);
                c = (c == 2) ? 0 : c + 1;
            }
        }
    }
    // tail
    const int64_t t0 = head + body;
    if (t0 + tid < nbytes) count((int)((t0 + tid) % 3), base[t0 + tid]);
    __syncthreads();

    // column sums: wave w reduces bins w, w+4, ...; lane reads 4 consecutive-thread entries
    __shared__ float tot[3 * COLOR_HIST_MAX_BINS];
    const int lane = tid & 63, wave = tid >> 6;
    for (int b = wave; b < nb; b += NT / 64) {
        const uint32_t* row = hist + b * NT;
        uint32_t s = row[lane] + row[lane + 64] + row[lane + 128] + row[lane + 192];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        if (lane == 0) {
            tot[b] = (float)s;
            if (counts) counts[img * nb + b] = s;
        }
    }
    __syncthreads();
    if (wave == 0) {
        // L2 norm of the float32 count vector (np.linalg.norm on the calcHist output)
        float ss = 0.f;
        for (int b = lane; b < nb; b += 64) ss = fmaf(tot[b], tot[b], ss);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
        const float l2 = sqrtf(ss);
        for (int b = lane; b < nb; b += 64) out[img * nb + b] = (l2 != 0.f) ? tot[b] / l2 : tot[b];
    }
}


// Fast path for a compile-time bin count (cv2's 16 by default).  The generic kernel above spends
// ~9 VALU per byte (runtime bin scaling, runtime channel, channel rotation) and is VALU-bound at
// ~2.7 TB/s.  Here each lane takes 48-byte granules (three 16-B loads = 16 whole pixels): a
// granule starts at image offset head + 48 g, so its first byte's channel is head % 3 for every
// lane and granule — one uniform switch per workgroup picks a fully unrolled body in which every
// byte's channel is a constant.  Per byte: one bit-field extract, one shift-add into the thread's
// column address, one ds_add_u32 whose channel offset is the instruction's immediate.
template <int BINS, int P0>
__device__ __forceinline__ void count_granule(uint32_t* __restrict__ col, const uint4& a,
                                              const uint4& b, const uint4& c) {
    const uint32_t w[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
#pragma unroll
    for (int q = 0; q < 12; ++q) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int ch = (P0 + 4 * q + j) % 3;
            const uint32_t bin = (((w[q] >> (8 * j)) & 0xffu) * (uint32_t)BINS) >> 8;
            atomicAdd(col + (ch * BINS + (int)bin) * NT, 1u);
        }
    }
}

template <int BINS, int P0>
__device__ __forceinline__ void count_body_lds(uint32_t* __restrict__ col, const uint4* __restrict__ vb,
                                               int64_t ngran, int tid) {
    // software pipeline: the loads of granule g + NT are in flight while granule g is counted
    int64_t g = tid;
    if (g >= ngran) return;
    uint4 a = vb[3 * g], b = vb[3 * g + 1], c = vb[3 * g + 2];
    for (; g + NT < ngran; g += NT) {
        const int64_t h = g + NT;
        const uint4 an = vb[3 * h], bn = vb[3 * h + 1], cn = vb[3 * h + 2];
        count_granule<BINS, P0>(col, a, b, c);
        a = an; b = bn; c = cn;
    }
    count_granule<BINS, P0>(col, a, b, c);
}

// Register (SWAR) counting for 16 bins, bin = top nibble of the byte (color_hist16_kernel).
// Loads are fully coalesced: in iteration m thread tid reads the 16-B vectors
// c = NT (3m + j) + tid, j = 0..2.  As 16 = NT = 1 (mod 3), byte i of vector j has channel
// (lp + j + i) mod 3 with the lane's fixed phase lp = (phase of the first vector + tid) mod 3, so
// the counters are kept per SLOT k = (j + i) mod 3 (compile-time) and mapped to channel
// (lp + k) mod 3 only when flushed.  Per slot one u64 of sixteen 4-bit counters: a byte adds
// 1 << (4 * bin) (the shift amounts of a word's four bytes come from one shift-and-mask,
// (w >> 2) & 0x3c3c3c3c; a 64-bit shift uses the low 6 bits of its amount) — a 64-bit shift and
// a 64-bit add per byte, no LDS atomic.  After vectors 1 and 2 of an iteration (<= 11 counts per
// slot since the last widening) the nibbles are widened into two u64 of eight 8-bit counters per
// slot (even / odd bins), which are flushed into 48 u32 register totals every 11 iterations
// (<= 242 per 8-bit counter).  No per-thread LDS columns: 16 waves per CU and two iterations of
// loads in flight per thread keep enough bytes in flight for HBM (the LDS-column form held 12
// waves with one iteration in flight and ran at ~4.5 TB/s whether its counting was LDS atomics
// or registers).
struct Swar16 {
    uint64_t r4[3] = {0, 0, 0};
    uint64_t a8[3][2] = {{0, 0}, {0, 0}, {0, 0}};
    uint32_t tot[3][16] = {};                            // per SLOT
    __device__ __forceinline__ void widen() {
        constexpr uint64_t M = 0x0f0f0f0f0f0f0f0full;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            a8[k][0] += r4[k] & M;
            a8[k][1] += (r4[k] >> 4) & M;
            r4[k] = 0;
        }
    }
    __device__ __forceinline__ void flush() {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
#pragma unroll
            for (int f = 0; f < 8; ++f) {
                tot[k][2 * f] += (uint32_t)(a8[k][0] >> (8 * f)) & 0xffu;
                tot[k][2 * f + 1] += (uint32_t)(a8[k][1] >> (8 * f)) & 0xffu;
            }
            a8[k][0] = a8[k][1] = 0;
        }
    }
    // one 16-B vector whose byte i goes to slot (K0 + i) mod 3
    template <int K0>
    __device__ __forceinline__ void vec(const uint4& v) {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint32_t t = (w[q] >> 2) & 0x3c3c3c3cu;             // 4 * bin of each byte
            asm volatile("" : "+v"(t));   // keep the word-wide mask (else it is re-split per byte)
#pragma unroll
            for (int j = 0; j < 4; ++j) r4[(K0 + 4 * q + j) % 3] += (uint64_t)1 << ((t >> (8 * j)) & 63u);
        }
    }
};

// 16-bin counting of nvec 16-B vectors vb[0 .. nvec) (first byte at channel phase0) into S.tot
__device__ __forceinline__ void count_swar16(Swar16& S, const uint4* __restrict__ vb, int64_t nvec, int tid) {
    const int64_t nit = nvec / (3 * NT);                 // full iterations (3 vectors per thread)
    int since = 0;
    if (nit > 0) {
        // two iterations of loads in flight: three register sets in a fixed ring, the loop
        // unrolled by three so no set is copied (a rotating copy made the compiler wait for
        // every outstanding load at the top of each iteration); loads past the last iteration
        // re-read it
        auto ld = [&](int64_t m, uint4 (&v)[3]) __attribute__((always_inline)) {
            const int64_t b = (m < nit ? m : nit - 1) * 3 * NT + tid;
            v[0] = vb[b]; v[1] = vb[b + NT]; v[2] = vb[b + 2 * NT];
        };
        auto run = [&](const uint4 (&v)[3]) __attribute__((always_inline)) {
            S.vec<0>(v[0]);
            S.vec<1>(v[1]);
            S.widen();
            S.vec<2>(v[2]);
            S.widen();
            if (++since == 11) { S.flush(); since = 0; }
        };
        uint4 A[3], B[3], C[3];
        ld(0, A);
        ld(1, B);
        for (int64_t m = 0; m < nit; m += 3) {
            ld(m + 2, C);
            run(A);
            if (m + 1 >= nit) break;
            ld(m + 3, A);
            run(B);
            if (m + 2 >= nit) break;
            ld(m + 4, B);
            run(C);
        }
    }
    // remaining < 3 NT vectors: vector c = 3 NT nit + r NT + tid, phase (lp + r) mod 3
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const int64_t cidx = 3 * NT * nit + (int64_t)r * NT + tid;
        if (cidx < nvec) {
            const uint4 v = vb[cidx];
            if (r == 0) S.vec<0>(v); else if (r == 1) S.vec<1>(v); else S.vec<2>(v);
        }
        S.widen();
    }
    S.flush();
}

__global__ void __launch_bounds__(NT)
color_hist16_kernel(const uint8_t* __restrict__ pix, const int64_t* __restrict__ offsets,
                    const int64_t* __restrict__ npix, float* __restrict__ out,
                    uint32_t* __restrict__ counts) {
    constexpr int nb = 48;
    __shared__ uint32_t part[NT / 64][nb];               // per-wave totals
    __shared__ uint32_t edge[nb];                        // head / tail bytes
    __shared__ float tot[nb];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < nb) edge[tid] = 0u;
    __syncthreads();
    const int64_t img = blockIdx.x;
    const int64_t nbytes = 3 * npix[img];
    const uint8_t* base = pix + offsets[img];
    auto count1 = [&](int64_t o) {
        atomicAdd(&edge[(int)(o % 3) * 16 + (base[o] >> 4)], 1u);
    };
    const int64_t head = std::min<int64_t>(nbytes, (int64_t)((16 - ((uintptr_t)base & 15)) & 15));
    if (tid < head) count1(tid);
    const int64_t nvec = (nbytes - head) >> 4;
    Swar16 S;
    count_swar16(S, reinterpret_cast<const uint4*>(base + head), nvec, tid);
    for (int64_t o = head + 16 * nvec + tid; o < nbytes; o += NT) count1(o);   // < 16 bytes
    // slot k of this lane = channel (lp + k) mod 3: rotate to channel order, then sum the wave
    const int lp = (int)((head % 3 + tid) % 3);
    uint32_t byc[3][16];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch)
#pragma unroll
        for (int b = 0; b < 16; ++b) {
            const uint32_t k0 = S.tot[(3 + ch - 0) % 3][b], k1 = S.tot[(3 + ch - 1) % 3][b], k2 = S.tot[(3 + ch - 2) % 3][b];
            byc[ch][b] = lp == 0 ? k0 : (lp == 1 ? k1 : k2);     // slot (ch - lp) mod 3
        }
#pragma unroll
    for (int ch = 0; ch < 3; ++ch)
#pragma unroll
        for (int b = 0; b < 16; ++b) {
            uint32_t v = byc[ch][b];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            if (lane == 0) part[wave][ch * 16 + b] = v;
        }
    __syncthreads();
    if (tid < nb) {
        uint32_t v = edge[tid];
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) v += part[w][tid];
        tot[tid] = (float)v;
        if (counts) counts[img * nb + tid] = v;
    }
    __syncthreads();
    if (wave == 0) {
        float ss = 0.f;
        for (int b = lane; b < nb; b += 64) ss = fmaf(tot[b], tot[b], ss);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
        const float l2 = sqrtf(ss);
        for (int b = lane; b < nb; b += 64) out[img * nb + b] = (l2 != 0.f) ? tot[b] / l2 : tot[b];
    }
}

template <int BINS, int P0>
__device__ __forceinline__ void count_body(uint32_t* __restrict__ col, const uint4* __restrict__ vb,
                                           int64_t ngran, int tid) {
    count_body_lds<BINS, P0>(col, vb, ngran, tid);
}

template <int BINS>
__global__ void __launch_bounds__(NT)
color_hist_fixed_kernel(const uint8_t* __restrict__ pix, const int64_t* __restrict__ offsets,
                        const int64_t* __restrict__ npix, float* __restrict__ out,
                        uint32_t* __restrict__ counts) {
    constexpr int nb = 3 * BINS;
    // u32 counters: a thread would need 2^32 bytes of one bin to overflow.  (16-bit counters,
    // two bins per word with a fold every 1365 granules, doubled the workgroups per CU and ran
    // no faster — 4.40-4.48 vs 4.39-4.52 TB/s — so the per-CU LDS atomic rate, not occupancy,
    // bounds this kernel; profiles/r01_ab_color/.)  A chunk loop with a fold between chunks is
    // kept for such a counter format.
    constexpr int nw = nb;
    constexpr int64_t chunk = INT64_MAX / 64;
    __shared__ __attribute__((aligned(16))) uint32_t hist[nw * NT];   // [word][NT]
    __shared__ uint32_t tot32[nb];
    __shared__ float tot[nb];
    const int tid = threadIdx.x;
    for (int i = tid; i < nw * NT; i += NT) hist[i] = 0u;
    if (tid < nb) tot32[tid] = 0u;
    __syncthreads();

    const int64_t img = blockIdx.x;
    const int64_t nbytes = 3 * npix[img];
    const uint8_t* base = pix + offsets[img];
    uint32_t* col = hist + tid;
    const int lane = tid & 63, wave = tid >> 6;
    auto count1 = [&](int64_t o) {                      // one byte at image offset o
        const int ch = (int)(o % 3);
        const uint32_t bin = ((uint32_t)base[o] * (uint32_t)BINS) >> 8;
        atomicAdd(col + (ch * BINS + (int)bin) * NT, 1u);
    };
    // columns -> tot32 (and zeroed for the next chunk): wave w folds words w, w + 4, ...
    auto fold = [&]() {
        __syncthreads();
        for (int wd = wave; wd < nw; wd += NT / 64) {
            uint32_t* row = hist + wd * NT;
            const uint32_t v0 = row[lane], v1 = row[lane + 64], v2 = row[lane + 128], v3 = row[lane + 192];
            row[lane] = 0u; row[lane + 64] = 0u; row[lane + 128] = 0u; row[lane + 192] = 0u;
            uint32_t sm = v0 + v1 + v2 + v3;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) sm += __shfl_xor(sm, o, 64);
            if (lane == 0) tot32[wd] += sm;
        }
        __syncthreads();
    };

    const int64_t head = std::min<int64_t>(nbytes, (int64_t)((16 - ((uintptr_t)base & 15)) & 15));
    if (tid < head) count1(tid);
    const int64_t ngran = (nbytes - head) / 48;
    const uint4* vb = reinterpret_cast<const uint4*>(base + head);
    const int phase = (int)(head % 3);                  // uniform over the workgroup
    for (int64_t g0 = 0; g0 < ngran; g0 += chunk) {
        const int64_t ng = std::min<int64_t>(ngran - g0, chunk);
        const uint4* v = vb + 3 * g0;
        switch (phase) {
            case 0: count_body<BINS, 0>(col, v, ng, tid); break;
            case 1: count_body<BINS, 1>(col, v, ng, tid); break;
            default: count_body<BINS, 2>(col, v, ng, tid); break;
        }
        if (g0 + chunk < ngran) fold();
    }
    for (int64_t o = head + 48 * ngran + tid; o < nbytes; o += NT) count1(o);   // < 48 bytes
    fold();

    if (tid < nb) {
        tot[tid] = (float)tot32[tid];
        if (counts) counts[img * nb + tid] = tot32[tid];
    }
    __syncthreads();
    if (wave == 0) {
        float ss = 0.f;
        for (int b = lane; b < nb; b += 64) ss = fmaf(tot[b], tot[b], ss);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
        const float l2 = sqrtf(ss);
        for (int b = lane; b < nb; b += 64) out[img * nb + b] = (l2 != 0.f) ? tot[b] / l2 : tot[b];
    }
}

thread_local std::string g_err;

void set_err(const char* fmt, ...) {
    char buf[256];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
}

}  // namespace

extern "C" {

const char* color_hist_last_error(void) { return g_err.c_str(); }

int color_hist_device(const uint8_t* pixels, const int64_t* offsets, const int64_t* npix,
                      int64_t n_images, int bins, float* out, uint32_t* counts, void* stream) {
    if (n_images < 0 || bins < 1 || bins > COLOR_HIST_MAX_BINS) {
        set_err("bad arguments (n_images=%lld bins=%d, bins must be in [1,%d])",
                (long long)n_images, bins, COLOR_HIST_MAX_BINS);
        return -1;
    }
    if (n_images == 0) return 0;
    if (!pixels || !offsets || !npix || !out) {
        set_err("NULL pointer");
        return -1;
    }
    if (bins == 16) {
#ifdef IMGREC_COLOR_LDS_ATOMIC
        hipLaunchKernelGGL(color_hist_fixed_kernel<16>, dim3((unsigned)n_images), dim3(NT), 0,
                           (hipStream_t)stream, pixels, offsets, npix, out, counts);
#else
        hipLaunchKernelGGL(color_hist16_kernel, dim3((unsigned)n_images), dim3(NT), 0,
                           (hipStream_t)stream, pixels, offsets, npix, out, counts);
#endif
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
            set_err("color_hist_fixed_kernel launch failed: %s", hipGetErrorString(e));
            return -2;
        }
        return 0;
    }
    const size_t lds = (size_t)3 * bins * NT * sizeof(uint32_t);
    hipLaunchKernelGGL(color_hist_kernel, dim3((unsigned)n_images), dim3(NT), lds,
                       (hipStream_t)stream, pixels, offsets, npix, bins, out, counts);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_err("color_hist_kernel launch failed: %s", hipGetErrorString(e));
        return -2;
    }
    return 0;
}

int color_hist_host(const uint8_t* pixels, int64_t total_bytes, const int64_t* offsets,
                    const int64_t* npix, int64_t n_images, int bins, int device, float* out,
                    uint32_t* counts) {
    if (n_images == 0) return 0;
    if (total_bytes < 0 || !pixels || !offsets || !npix || !out || n_images < 0) {
        set_err("bad arguments");
        return -1;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        set_err("no HIP device visible");
        return -5;
    }
    for (int64_t i = 0; i < n_images; ++i) {
        if (offsets[i] < 0 || npix[i] < 0 || offsets[i] + 3 * npix[i] > total_bytes) {
            set_err("image %lld lies outside the pixel buffer", (long long)i);
            return -1;
        }
    }
    int old = -1;
    (void)hipGetDevice(&old);
    if (device >= 0) (void)hipSetDevice(device);
    uint8_t* dp = nullptr;
    int64_t* doff = nullptr;
    int64_t* dn = nullptr;
    float* dout = nullptr;
    uint32_t* dc = nullptr;
    const int nb = 3 * bins;
    int rc = 0;
    hipError_t e = hipMalloc((void**)&dp, (size_t)std::max<int64_t>(total_bytes, 16));
    if (e == hipSuccess) e = hipMalloc((void**)&doff, (size_t)n_images * 8);
    if (e == hipSuccess) e = hipMalloc((void**)&dn, (size_t)n_images * 8);
    if (e == hipSuccess) e = hipMalloc((void**)&dout, (size_t)n_images * nb * 4);
    if (e == hipSuccess && counts) e = hipMalloc((void**)&dc, (size_t)n_images * nb * 4);
    if (e == hipSuccess) e = hipMemcpy(dp, pixels, (size_t)total_bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(doff, offsets, (size_t)n_images * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dn, npix, (size_t)n_images * 8, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        set_err("staging failed: %s", hipGetErrorString(e));
        rc = -2;
    } else {
        rc = color_hist_device(dp, doff, dn, n_images, bins, dout, dc, nullptr);
        if (rc == 0) {
            e = hipMemcpy(out, dout, (size_t)n_images * nb * 4, hipMemcpyDeviceToHost);
            if (e == hipSuccess && counts)
                e = hipMemcpy(counts, dc, (size_t)n_images * nb * 4, hipMemcpyDeviceToHost);
            if (e != hipSuccess) {
                set_err("copy-back failed: %s", hipGetErrorString(e));
                rc = -2;
            }
        }
    }
    for (void* p : {(void*)dp, (void*)doff, (void*)dn, (void*)dout, (void*)dc})
        if (p) (void)hipFree(p);
    if (old >= 0) (void)hipSetDevice(old);
    return rc;
}

int color_host_register(void* ptr, int64_t bytes) {
    if (!ptr || bytes <= 0) {
        set_err("bad host range");
        return -1;
    }
    const hipError_t e = hipHostRegister(ptr, (size_t)bytes, hipHostRegisterDefault);
    if (e != hipSuccess) {
        set_err("hipHostRegister failed: %s", hipGetErrorString(e));
        return -2;
    }
    return 0;
}

int color_host_unregister(void* ptr) {
    if (!ptr) return 0;
    const hipError_t e = hipHostUnregister(ptr);
    if (e != hipSuccess) {
        set_err("hipHostUnregister failed: %s", hipGetErrorString(e));
        return -2;
    }
    return 0;
}

int color_hist_batch_async(const uint8_t* host_pixels, int64_t bytes, const int64_t* host_meta,
                           int64_t n, int bins, uint8_t* dev_pixels, int64_t* dev_meta,
                           float* dev_out, uint32_t* dev_counts, void* stream) {
    if (n < 0 || bytes < 0 || bins < 1 || bins > COLOR_HIST_MAX_BINS) {
        set_err("bad arguments (n=%lld bytes=%lld bins=%d)", (long long)n, (long long)bytes, bins);
        return -1;
    }
    if (n == 0) return 0;
    if (!host_pixels || !host_meta || !dev_pixels || !dev_meta || !dev_out) {
        set_err("NULL pointer");
        return -1;
    }
    for (int64_t i = 0; i < n; ++i) {
        const int64_t o = host_meta[i], np = host_meta[n + i];
        if (o < 0 || np < 0 || o + 3 * np > bytes) {
            set_err("image %lld lies outside the batch's pixel bytes", (long long)i);
            return -1;
        }
    }
    const hipStream_t st = (hipStream_t)stream;
    hipError_t e = hipMemcpyAsync(dev_pixels, host_pixels, (size_t)bytes, hipMemcpyHostToDevice, st);
    if (e == hipSuccess)
        e = hipMemcpyAsync(dev_meta, host_meta, (size_t)(2 * n) * sizeof(int64_t), hipMemcpyHostToDevice, st);
    if (e != hipSuccess) {
        set_err("batch upload failed: %s", hipGetErrorString(e));
        return -2;
    }
    return color_hist_device(dev_pixels, dev_meta, dev_meta + n, n, bins, dev_out, dev_counts, stream);
}

}  // extern "C"
