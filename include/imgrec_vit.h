/*
 * imgrec_vit.h — C ABI of the fused elementwise kernels of the DreamSim-architecture ViT forward
 * (image_recommender_amd/vector_scripts/create_dreamsim_vector.py).  The reference embeds images
 * with dreamsim's three ViT-B/16 towers (/root/reference/vector_scripts/create_dreamsim_vector.py:
 * 38-43, 51-93, `model.embed`); between the bf16 matrix products of every block the forward keeps
 * an fp32 residual stream and fp32 LayerNorms.  These kernels fuse what would otherwise be
 * separate passes over the activations.
 *
 * bf16 values are raw 16-bit patterns (uint16_t); device pointers; enqueued on `stream`
 * (hipStream_t, NULL = default stream), no synchronisation.  Return 0, or -1 on bad arguments.
 */
#ifndef IMGREC_VIT_H
#define IMGREC_VIT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Per row r of `rows` (row length dim <= 1024): x[r] += delta[r] (bf16, when delta != NULL;
 * x is updated in place), then y[r] = bf16(LayerNorm(x[r]) * gamma + beta) with the biased
 * variance and `eps` (torch.nn.LayerNorm semantics, fp32 arithmetic). */
int vit_add_layernorm_bf16(float* x, const uint16_t* delta, const float* gamma, const float* beta,
                           uint16_t* y, int64_t rows, int dim, float eps, void* stream);

/* In place on n bf16 values: h = bf16(h * sigmoid(1.702 h)) (CLIP's QuickGELU), fp32 inside. */
int vit_quick_gelu_bf16(uint16_t* h, int64_t n, void* stream);

/* In place on n bf16 values: h = bf16(0.5 h (1 + erf(h / sqrt 2))) (nn.GELU, the DINO and
 * OpenCLIP towers' MLP activation), fp32 inside. */
int vit_gelu_bf16(uint16_t* h, int64_t n, void* stream);

/* The tower input as GEMM rows: image (batch, 3, height, width) fp32 -> bf16(((x - mean[c]) /
 * std[c])) patches (batch, (height/patch)(width/patch), 3 patch patch), each laid out (c, kh, kw)
 * like the stride-`patch` patch conv's weight (patch a multiple of 8; 16-B aligned pointers). */
int vit_patchify_bf16(const float* img, int64_t batch, int height, int width, int patch,
                      const float* mean, const float* std_, uint16_t* out, void* stream);

/* Token rows: out (batch, npatch + 1, dim) fp32 = [cls + pos[0] ; fp32(patch_emb[b]) + pos[1:]]
 * (patch_emb bf16 (batch, npatch, dim); dim a multiple of 4; 16-B aligned fp32 pointers). */
int vit_tokens_f32(const uint16_t* patch_emb, const float* cls, const float* pos, int64_t batch,
                   int npatch, int dim, float* out, void* stream);

/* Multi-head self-attention softmax(q k^T * scale) v of every (image, head), without masks
 * (torch.nn.functional.scaled_dot_product_attention with scale = 1/sqrt(head_dim)): qkv is the
 * qkv Linear's output (batch, ntok, 3, heads, head_dim) bf16, out (batch, ntok, heads * head_dim)
 * bf16 (the output projection's input layout).  head_dim = 64, ntok <= 256; scores, softmax and
 * the output accumulate in fp32 (bf16 probabilities into the P.V products); 16-B aligned
 * pointers (csrc/vit_attn.hip). */
int vit_attention_bf16(const uint16_t* qkv, int64_t batch, int ntok, int heads, int head_dim,
                       float scale, uint16_t* out, void* stream);

/* Activation of vit_linear_bf16's epilogue, applied in fp32 before the bf16 rounding. */
enum vit_act {
    VIT_ACT_NONE = 0,
    VIT_ACT_GELU_ERF = 1,    /* nn.GELU: 0.5 x (1 + erf(x / sqrt 2)) (DINO, OpenCLIP MLPs) */
    VIT_ACT_GELU_TANH = 2,   /* nn.GELU(approximate="tanh") */
    VIT_ACT_QUICK_GELU = 3   /* CLIP's QuickGELU: x sigmoid(1.702 x) */
};

/* y (m x n) = bf16(act(x w^T + bias)): x (m x k) and w (n x k, nn.Linear's weight layout) bf16
 * row-major, bias fp32 (n) or NULL, fp32 accumulation (F.linear's product, csrc/vit_gemm.hip).
 * k a multiple of 64, n a multiple of 256, 16-B aligned pointers; any m. */
int vit_linear_bf16(const uint16_t* x, const uint16_t* w, const float* bias, int64_t m, int k,
                    int n, int act, uint16_t* y, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* IMGREC_VIT_H */
