"""The fused ViT elementwise kernels (include/imgrec_vit.h) against a plain PyTorch fp32 reference,
and the fused DreamSim-architecture forward against the unfused one (same weights)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,dim", [(1, 64), (197 * 3, 768), (50, 1000), (7, 300), (5, 1024), (9, 256)])
@pytest.mark.parametrize("with_delta", [True, False])
def test_add_layernorm_matches_torch(gpu, rows, dim, with_delta):
    from image_recommender_amd.vector_scripts.create_dreamsim_vector import _add_ln
    g = torch.Generator(device="cuda").manual_seed(rows * dim)
    x = torch.randn(rows, dim, device="cuda", generator=g) * 3 + 0.5
    delta = (torch.randn(rows, dim, device="cuda", generator=g)).bfloat16() if with_delta else None
    ln = torch.nn.LayerNorm(dim).cuda()
    with torch.no_grad():
        ln.weight.copy_(torch.randn(dim, device="cuda", generator=g))
        ln.bias.copy_(torch.randn(dim, device="cuda", generator=g))
    x_ref = x + delta.float() if with_delta else x.clone()
    y_ref = torch.nn.functional.layer_norm(x_ref, (dim,), ln.weight, ln.bias, ln.eps)
    y = _add_ln(x, delta, ln)
    torch.cuda.synchronize()
    assert torch.equal(x, x_ref)                           # the residual update is the same fp32 add
    # bf16 output: within one bf16 rounding of the fp32 reference (plus fp32 reduction-order slack)
    err = (y.float() - y_ref).abs()
    assert float((err - y_ref.abs() * 2.0 ** -8 - 1e-4).max()) <= 0.0


def test_quick_gelu_matches_torch(gpu):
    from image_recommender_amd.vector_scripts.create_dreamsim_vector import _quick_gelu_
    h = (torch.randn(3 * 197 * 3072 + 5, device="cuda") * 4).bfloat16()   # odd tail too
    ref = h.float() * torch.sigmoid(1.702 * h.float())
    out = _quick_gelu_(h.clone())
    torch.cuda.synchronize()
    err = (out.float() - ref).abs()
    assert float((err - ref.abs() * 2.0 ** -8 - 1e-6).max()) <= 0.0


def test_fused_forward_matches_unfused(gpu):
    from image_recommender_amd.vector_scripts.create_dreamsim_vector import build_ensemble
    x = torch.rand((6, 3, 224, 224), device="cuda", generator=torch.Generator(device="cuda").manual_seed(1))
    plain = build_ensemble(seed=0, depth=4).cuda().eval().prepare_inference(torch.bfloat16)
    fused = build_ensemble(seed=0, depth=4).cuda().eval().prepare_inference(torch.bfloat16, fused=True)
    with torch.no_grad():
        a = torch.nn.functional.normalize(plain.embed(x).float(), dim=-1)
        b = torch.nn.functional.normalize(fused.embed(x).float(), dim=-1)
    cos = (a * b).sum(-1)
    assert float(cos.min()) > 0.999, cos


def test_gelu_matches_torch(gpu):
    """vit_gelu_bf16 (erf form, in place) against torch's fp32 erf GELU: within one bf16 rounding."""
    from image_recommender_amd.vector_scripts.create_dreamsim_vector import _gelu_
    for n in (3 * 197 * 3072 + 11, 16, 5):                      # whole 16-element groups and tails
        h = (torch.randn(n, device="cuda") * 4).bfloat16()
        ref = torch.nn.functional.gelu(h.float())
        out = _gelu_(h.clone())
        torch.cuda.synchronize()
        err = (out.float() - ref).abs()
        assert float((err - ref.abs() * 2.0 ** -8 - 1e-6).max()) <= 0.0


def test_gelu_epilogue_within_bf16_of_erf_gelu(gpu):
    """The fc1 + GELU as one hipBLASLt launch (GELU_BIAS epilogue, tanh form; _lin_gelu) against
    the fp32 erf-form reference of the same bf16 GEMM: within 2 bf16 roundings (the tanh-erf gap
    is < 5e-4 absolute); and the forward built on it against the unfused forward, cos > 0.999."""
    from image_recommender_amd.vector_scripts.create_dreamsim_vector import _lin_gelu, build_ensemble
    g = torch.Generator(device="cuda").manual_seed(3)
    lin = torch.nn.Linear(768, 3072).cuda()
    lin.w_lp, lin.b_lp = lin.weight.detach().bfloat16(), lin.bias.detach().bfloat16()
    x = torch.randn(2, 197, 768, device="cuda", generator=g).bfloat16()
    ref = torch.nn.functional.gelu(torch.nn.functional.linear(x.float(), lin.w_lp.float(), lin.b_lp.float()))
    got = _lin_gelu(lin, x).float()
    err = (got - ref).abs()
    assert float((err - ref.abs() * 2.0 ** -7 - 2e-3).max()) <= 0.0
    xi = torch.rand((4, 3, 224, 224), device="cuda", generator=torch.Generator(device="cuda").manual_seed(2))
    plain = build_ensemble(seed=0, depth=4).cuda().eval().prepare_inference(torch.bfloat16)
    lt = build_ensemble(seed=0, depth=4).cuda().eval().prepare_inference(torch.bfloat16, fused=True,
                                                                          gelu_epilogue=True)
    with torch.no_grad():
        a = torch.nn.functional.normalize(plain.embed(xi).float(), dim=-1)
        b = torch.nn.functional.normalize(lt.embed(xi).float(), dim=-1)
    assert float((a * b).sum(-1).min()) > 0.999


def test_patchify_and_tokens_match_torch(gpu):
    """vit_patchify_bf16 = bf16((x - mean) / std) in the conv weight's (c, kh, kw) patch layout, and
    vit_tokens_f32 = cat(cls, pe.float()) + pos — both bit-exact against the torch ops they fuse."""
    from image_recommender_amd.vector_scripts.create_dreamsim_vector import _patchify, _tokens
    g = torch.Generator(device="cuda").manual_seed(4)
    x = torch.rand((3, 3, 224, 224), device="cuda", generator=g)
    mean = torch.tensor((0.48, 0.45, 0.40), device="cuda").view(1, 3, 1, 1)
    std = torch.tensor((0.26, 0.26, 0.27), device="cuda").view(1, 3, 1, 1)
    p = 16
    ref = ((x - mean) / std).bfloat16().reshape(3, 3, 14, p, 14, p).permute(0, 2, 4, 1, 3, 5)
    ref = ref.reshape(3, 196, 3 * p * p)
    got = _patchify(x, mean, std, p)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    pe = torch.randn((3, 196, 768), device="cuda", generator=g).bfloat16()
    cls = torch.randn((1, 1, 768), device="cuda", generator=g)
    pos = torch.randn((1, 197, 768), device="cuda", generator=g)
    tok = _tokens(pe, cls, pos)
    torch.cuda.synchronize()
    assert torch.equal(tok, torch.cat([cls.expand(3, -1, -1), pe.float()], 1) + pos)


@pytest.mark.parametrize("b,n,heads", [(3, 197, 12), (2, 16, 2), (1, 1, 1), (2, 50, 3), (1, 256, 4),
                                       (4, 33, 12), (2, 208, 1), (1, 17, 5)])
def test_attention_matches_torch(gpu, b, n, heads):
    """vit_attention_bf16 against torch's fp32 SDPA on the same bf16 q / k / v: within the bf16
    rounding of the probabilities (the P.V products take bf16 P) and of the output."""
    from image_recommender_amd.vector_scripts.create_dreamsim_vector import _attn
    g = torch.Generator(device="cuda").manual_seed(b * 1000 + n * 10 + heads)
    qkv = (torch.randn(b, n, 3 * heads * 64, device="cuda", generator=g) * 1.5).bfloat16()
    q, k, v = qkv.float().view(b, n, 3, heads, 64).permute(2, 0, 3, 1, 4).unbind(0)
    ref = torch.nn.functional.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(b, n, heads * 64)
    out = _attn(qkv, heads)
    torch.cuda.synchronize()
    err = (out.float() - ref).abs()
    # |P_bf16 - P| <= 2^-9 P per entry, so |sum (P_bf16 - P) v| <= 2^-9 max|v|; plus the output's
    # own bf16 rounding
    vmax = v.abs().amax(dim=(-2, -1))                    # (b, heads)
    bound = 2.0 ** -8 * ref.abs() + 2.0 ** -8 * vmax.repeat_interleave(64, dim=1)[:, None, :] + 1e-5
    assert float((err - bound).max()) <= 0.0, float(err.max())


def test_attention_rejects_bad_shapes(gpu):
    import ctypes as C
    from image_recommender_amd import _lib
    qkv = torch.zeros(1, 300, 3 * 64, dtype=torch.bfloat16, device="cuda")
    out = torch.zeros(1, 300, 64, dtype=torch.bfloat16, device="cuda")
    lib = _lib.load()
    assert lib.vit_attention_bf16(C.c_void_p(qkv.data_ptr()), 1, 300, 1, 64, C.c_float(0.125),
                                  C.c_void_p(out.data_ptr()), None) == -1          # ntok > 256
    assert lib.vit_attention_bf16(C.c_void_p(qkv.data_ptr()), 1, 100, 1, 32, C.c_float(0.125),
                                  C.c_void_p(out.data_ptr()), None) == -1          # head_dim != 64


def test_fused_forward_hip_attention_matches_sdpa(gpu):
    """The fused forward with the HIP attention against the same forward on torch SDPA."""
    from image_recommender_amd.vector_scripts.create_dreamsim_vector import build_ensemble
    x = torch.rand((4, 3, 224, 224), device="cuda", generator=torch.Generator(device="cuda").manual_seed(2))
    sdpa = build_ensemble(seed=0, depth=4).cuda().eval().prepare_inference(torch.bfloat16, fused=True,
                                                                           hip_attn=False)
    hip = build_ensemble(seed=0, depth=4).cuda().eval().prepare_inference(torch.bfloat16, fused=True)
    with torch.no_grad():
        a = sdpa.embed(x).float()
        c = hip.embed(x).float()
    cos = (torch.nn.functional.normalize(a, dim=-1) * torch.nn.functional.normalize(c, dim=-1)).sum(-1)
    assert float(cos.min()) > 0.999, cos
