"""DreamSim-ensemble embeddings on PyTorch-ROCm — drop-in for create_dreamsim_vector.py.

The reference (/root/reference/vector_scripts/create_dreamsim_vector.py:11-125) loads
``dreamsim(pretrained=True, dreamsim_type="ensemble", normalize_embeds=True)`` (dreamsim 0.2.1,
weights downloaded at run time), embeds batches of 128 images resized to 224x224 (LANCZOS) and
L2-normalises each embedding (:92).  The ensemble is three ViT-B/16 towers — DINO (768-d CLS),
OpenAI CLIP and OpenCLIP (512-d projected CLS) — concatenated to 1792 dimensions.

This module implements that architecture in plain PyTorch (bf16 matrix products with fp32
LayerNorm / residual stream, fused scaled-dot-product attention — it runs on PyTorch-ROCm, no hand
kernel is required for it).  Pretrained weights cannot be fetched here: ``DreamSimVectorIndexer``
needs ``weights_path`` and raises like the reference does when the model cannot be loaded;
``allow_random_init=True`` builds a randomly initialised model for throughput measurements only
(its embeddings are not DreamSim embeddings; embedding parity is unpinned).

Weights: ``weights_path`` holds either a state dict of ``DreamSimEnsemble`` (keys below) or the
three towers' own checkpoints, converted by ``ensemble_state_from_towers``:

=====================================  ==========================================================
ours (``towers.{t}.`` prefix)          source layout
=====================================  ==========================================================
``patch.weight`` / ``patch.bias``      DINO ``patch_embed.proj.*``; CLIP / OpenCLIP ``conv1.weight``
``cls`` (1, 1, 768)                    DINO ``cls_token``; CLIP ``class_embedding`` (768,)
``pos`` (1, 197, 768)                  DINO ``pos_embed``; CLIP ``positional_embedding`` (197, 768)
``ln_pre.*``                           CLIP ``ln_pre.*`` (DINO has none)
``blocks.{i}.ln1.*`` / ``ln2.*``       DINO ``blocks.{i}.norm1/norm2``; CLIP ``transformer.resblocks.{i}.ln_1/ln_2``
``blocks.{i}.qkv.*``                   DINO ``blocks.{i}.attn.qkv``; CLIP ``...attn.in_proj_weight/bias`` (q|k|v rows)
``blocks.{i}.proj.*``                  DINO ``blocks.{i}.attn.proj``; CLIP ``...attn.out_proj``
``blocks.{i}.fc1.*`` / ``fc2.*``       DINO ``blocks.{i}.mlp.fc1/fc2``; CLIP ``...mlp.c_fc/c_proj``
``ln_post.*``                          DINO ``norm``; CLIP ``ln_post``
``head.weight`` (512, 768)             CLIP ``proj`` (768, 512) transposed (DINO: none, CLS is the feature)
=====================================  ==========================================================

(t = 0 dino_vitb16 [timm / facebookresearch-dino names], 1 OpenAI clip_vitb16 visual, 2
open_clip_vitb16 visual; a ``visual.`` prefix is stripped.)  DreamSim's own fine-tuning ships
LoRA adapters for these towers; merged into the base weights (W + scale * B @ A) they are plain
weights of this layout.  tests/test_dreamsim_cpu.py checks the conversion against independent
forwards written in each source layout's own module structure.
"""
from __future__ import annotations

import math
from pathlib import Path

import numpy as np

from .create_vector_base import BaseVectorIndexer, load_image

_MEAN_STD = {
    "dino": ((0.485, 0.456, 0.406), (0.229, 0.224, 0.225)),                      # ImageNet
    "clip": ((0.48145466, 0.4578275, 0.40821073), (0.26862954, 0.26130258, 0.27577711)),
    "open_clip": ((0.48145466, 0.4578275, 0.40821073), (0.26862954, 0.26130258, 0.27577711)),
}


def _torch():
    import torch
    import torch.nn as nn
    import torch.nn.functional as F
    return torch, nn, F


def _lin(m, x):
    """A Linear / projection through its cached low-precision copy when prepared (see
    prepare_inference), else as is."""
    w = getattr(m, "w_lp", None)
    if w is None:
        return m(x)
    F = _torch()[2]
    return F.linear(x.to(w.dtype), w, m.b_lp)


def _add_ln(x, delta, ln):
    """x += delta (bf16, or None) in place, and the bf16 LayerNorm of the new x — one HIP pass
    (include/imgrec_vit.h vit_add_layernorm_bf16)."""
    import ctypes as C

    import torch
    from .. import _lib
    c = x.shape[-1]
    if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous()):
        raise TypeError("_add_ln: x must be a contiguous fp32 GPU tensor (updated in place)")
    if ln.weight.dtype != torch.float32 or ln.bias.dtype != torch.float32:
        raise TypeError("_add_ln: LayerNorm parameters must be fp32")
    if delta is not None:
        # kept alive in this frame until the kernel is enqueued (a temporary's storage could be
        # reused by the caching allocator before the launch)
        delta = delta.contiguous()
        if delta.dtype != torch.bfloat16 or delta.shape != x.shape:
            raise TypeError("_add_ln: delta must be bf16 with x's shape")
    y = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    d = 0 if delta is None else delta.data_ptr()
    rc = _lib.load().vit_add_layernorm_bf16(
        C.c_void_p(x.data_ptr()), C.c_void_p(d), C.c_void_p(ln.weight.data_ptr()),
        C.c_void_p(ln.bias.data_ptr()), C.c_void_p(y.data_ptr()), x.numel() // c, c, float(ln.eps),
        C.c_void_p(torch.cuda.current_stream(x.device).cuda_stream))
    if rc != 0:
        raise RuntimeError("vit_add_layernorm_bf16 failed")
    return y


def _lin_gelu(m, x):
    """GELU(x W^T + b) of a prepared Linear in ONE hipBLASLt launch (GELU_BIAS epilogue through
    torch._addmm_activation).  The epilogue's GELU is the tanh form; against the erf form of
    nn.GELU it differs by < 5e-4 absolute (< 2e-4 relative), below the bf16 rounding of the
    output it is applied to (2^-9 relative)."""
    import torch
    shp = x.shape
    y = torch._addmm_activation(m.b_lp, x.reshape(-1, shp[-1]), m.w_lp.t(), use_gelu=True)
    return y.view(*shp[:-1], y.shape[-1])


_ACT = {"none": 0, "gelu": 1, "gelu_tanh": 2, "quick_gelu": 3}     # include/imgrec_vit.h vit_act


def _hlin(m, x, act="none"):
    """act(x W^T + b) of a prepared Linear / patch projection in ONE HIP kernel
    (include/imgrec_vit.h vit_linear_bf16, csrc/vit_gemm.hip): bf16 operands, fp32 accumulation,
    the fp32 bias and the activation (nn.GELU's erf form, CLIP's QuickGELU) applied before the
    bf16 rounding of the output.  Shapes the kernel does not take (k % 64, n % 256) go through
    _lin (and the activation as a separate pass)."""
    import ctypes as C

    import torch
    from .. import _lib
    w = m.w_lp
    n, k = w.shape
    if k % 64 or n % 256 or x.dtype != torch.bfloat16:
        y = _lin(m, x)
        return {"none": lambda t: t, "gelu": _gelu_, "quick_gelu": _quick_gelu_,
                "gelu_tanh": _gelu_tanh}[act](y.contiguous())
    x = x.contiguous()
    y = torch.empty((*x.shape[:-1], n), dtype=torch.bfloat16, device=x.device)
    b = getattr(m, "b_f32", None)
    rc = _lib.load().vit_linear_bf16(C.c_void_p(x.data_ptr()), C.c_void_p(w.data_ptr()),
                                     C.c_void_p(b.data_ptr() if b is not None else None),
                                     x.numel() // k, k, n, _ACT[act], C.c_void_p(y.data_ptr()),
                                     C.c_void_p(torch.cuda.current_stream(x.device).cuda_stream))
    if rc != 0:
        raise RuntimeError("vit_linear_bf16 failed")
    return y


def _patchify(img, mean, std, p):
    """(B, 3, H, W) fp32 image -> bf16 GEMM rows (B, (H/p)(W/p), 3 p p) of ((img - mean) / std),
    patches laid out (c, kh, kw) — one HIP pass (vit_patchify_bf16) for the normalisation, the
    patch permute and the bf16 cast."""
    import ctypes as C

    import torch
    from .. import _lib
    img = img.contiguous().float()
    b, c, h, w = img.shape
    out = torch.empty((b, (h // p) * (w // p), c * p * p), dtype=torch.bfloat16, device=img.device)
    mean, std = mean.contiguous(), std.contiguous()
    rc = _lib.load().vit_patchify_bf16(C.c_void_p(img.data_ptr()), b, h, w, p,
                                       C.c_void_p(mean.data_ptr()), C.c_void_p(std.data_ptr()),
                                       C.c_void_p(out.data_ptr()),
                                       C.c_void_p(torch.cuda.current_stream(img.device).cuda_stream))
    if rc != 0:
        raise RuntimeError("vit_patchify_bf16 failed")
    return out


def _tokens(pe, cls, pos):
    """bf16 patch embeddings (B, np, C) -> fp32 tokens (B, np + 1, C) = cat(cls, pe) + pos in one
    HIP pass (vit_tokens_f32)."""
    import ctypes as C

    import torch
    from .. import _lib
    pe = pe.contiguous()
    b, n, c = pe.shape
    cls, pos = cls.detach().contiguous(), pos.detach().contiguous()
    out = torch.empty((b, n + 1, c), dtype=torch.float32, device=pe.device)
    rc = _lib.load().vit_tokens_f32(C.c_void_p(pe.data_ptr()), C.c_void_p(cls.data_ptr()),
                                    C.c_void_p(pos.data_ptr()), b, n, c, C.c_void_p(out.data_ptr()),
                                    C.c_void_p(torch.cuda.current_stream(pe.device).cuda_stream))
    if rc != 0:
        raise RuntimeError("vit_tokens_f32 failed")
    return out


def _attn(qkv, heads):
    """Self-attention of every (image, head) from the qkv Linear's output (B, N, 3 * C) bf16 ->
    (B, N, C) bf16 in one HIP kernel (vit_attention_bf16): no q / k / v permute copies, no output
    transpose, the 197-token rows unpadded."""
    import ctypes as C

    import torch
    from .. import _lib
    b, n, c3 = qkv.shape
    c = c3 // 3
    hd = c // heads
    qkv = qkv.contiguous()
    if qkv.dtype != torch.bfloat16 or not qkv.is_cuda:
        raise TypeError("_attn: qkv must be a bf16 GPU tensor")
    out = torch.empty((b, n, c), dtype=torch.bfloat16, device=qkv.device)
    rc = _lib.load().vit_attention_bf16(C.c_void_p(qkv.data_ptr()), b, n, heads, hd,
                                        C.c_float(1.0 / math.sqrt(hd)), C.c_void_p(out.data_ptr()),
                                        C.c_void_p(torch.cuda.current_stream(qkv.device).cuda_stream))
    if rc != 0:
        raise RuntimeError("vit_attention_bf16 failed")
    return out


def _gelu_(h):
    """nn.GELU (erf form) in place on a contiguous bf16 tensor (vit_gelu_bf16)."""
    import ctypes as C

    import torch
    from .. import _lib
    rc = _lib.load().vit_gelu_bf16(C.c_void_p(h.data_ptr()), h.numel(),
                                   C.c_void_p(torch.cuda.current_stream(h.device).cuda_stream))
    if rc != 0:
        raise RuntimeError("vit_gelu_bf16 failed")
    return h


def _gelu_tanh(h):
    """GELU's tanh form on a bf16 tensor, evaluated in fp32 (the fallback of _hlin's fused
    "gelu_tanh" epilogue for shapes vit_linear_bf16 does not take)."""
    import torch
    return torch.nn.functional.gelu(h.float(), approximate="tanh").to(torch.bfloat16)


def _quick_gelu_(h):
    """CLIP's QuickGELU in place on a contiguous bf16 tensor (vit_quick_gelu_bf16)."""
    import ctypes as C

    import torch
    from .. import _lib
    rc = _lib.load().vit_quick_gelu_bf16(C.c_void_p(h.data_ptr()), h.numel(),
                                         C.c_void_p(torch.cuda.current_stream(h.device).cuda_stream))
    if rc != 0:
        raise RuntimeError("vit_quick_gelu_bf16 failed")
    return h


def build_ensemble(seed: int | None = 0, depth: int = 12):
    torch, nn, F = _torch()

    class Block(nn.Module):
        def __init__(self, dim=768, heads=12, mlp=3072, quick_gelu=False):
            super().__init__()
            self.heads = heads
            self.ln1 = nn.LayerNorm(dim)
            self.qkv = nn.Linear(dim, 3 * dim)
            self.proj = nn.Linear(dim, dim)
            self.ln2 = nn.LayerNorm(dim)
            self.fc1 = nn.Linear(dim, mlp)
            self.fc2 = nn.Linear(mlp, dim)
            self.quick_gelu = quick_gelu

        def forward(self, x):
            b, n, c = x.shape
            qkv = _lin(self.qkv, self.ln1(x)).view(b, n, 3, self.heads, c // self.heads)
            q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)
            a = F.scaled_dot_product_attention(q, k, v)
            x = x + _lin(self.proj, a.transpose(1, 2).reshape(b, n, c))
            h = _lin(self.fc1, self.ln2(x))
            h = h * torch.sigmoid(1.702 * h) if self.quick_gelu else F.gelu(h)
            return x + _lin(self.fc2, h)

        def forward_fused(self, x, delta):
            """The same block on the fused kernels: x (fp32 residual, updated in place) first takes
            the previous block's bf16 output `delta`; returns this block's bf16 output."""
            b, n, c = x.shape
            if getattr(self, "hip_gemm", False):
                # every matrix product (and fc1's activation) on vit_linear_bf16
                qkv = _hlin(self.qkv, _add_ln(x, delta, self.ln1))
                a = _attn(qkv, self.heads) if getattr(self, "hip_attn", False) else \
                    F.scaled_dot_product_attention(
                        *qkv.view(b, n, 3, self.heads, c // self.heads).permute(2, 0, 3, 1, 4).unbind(0)
                    ).transpose(1, 2).reshape(b, n, c)
                y = _add_ln(x, _hlin(self.proj, a), self.ln2)
                # (gelu_epilogue: the tanh form, as hipBLASLt's GELU_BIAS epilogue computes it —
                # within the bf16 rounding of the erf form, test_gelu_epilogue_within_bf16_of_erf_gelu)
                h = _hlin(self.fc1, y, "quick_gelu" if self.quick_gelu else
                          ("gelu_tanh" if getattr(self, "gelu_epilogue", False) else "gelu"))
                return _hlin(self.fc2, h)
            qkv = _lin(self.qkv, _add_ln(x, delta, self.ln1))
            if getattr(self, "hip_attn", False):
                a = _attn(qkv, self.heads)
            else:
                q, k, v = qkv.view(b, n, 3, self.heads, c // self.heads).permute(2, 0, 3, 1, 4).unbind(0)
                a = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(b, n, c)
            y = _add_ln(x, _lin(self.proj, a), self.ln2)
            if self.quick_gelu:
                h = _quick_gelu_(_lin(self.fc1, y))
            elif getattr(self, "gelu_epilogue", False):
                h = _lin_gelu(self.fc1, y)
            else:
                h = _gelu_(_lin(self.fc1, y))
            return _lin(self.fc2, h)

    class ViT(nn.Module):
        """ViT-B/16 tower; `out_dim` adds a CLIP-style projection of the CLS token."""

        def __init__(self, kind, out_dim=None, blocks=12, dim=768, patch=16, img=224):
            super().__init__()
            self.kind = kind
            self.patch = nn.Conv2d(3, dim, patch, patch, bias=(kind == "dino"))
            self.cls = nn.Parameter(torch.zeros(1, 1, dim))
            self.pos = nn.Parameter(torch.zeros(1, (img // patch) ** 2 + 1, dim))
            self.ln_pre = nn.LayerNorm(dim) if kind != "dino" else nn.Identity()
            self.blocks = nn.ModuleList(Block(dim, quick_gelu=(kind == "clip")) for _ in range(blocks))
            self.ln_post = nn.LayerNorm(dim)
            self.head = nn.Linear(dim, out_dim, bias=False) if out_dim else nn.Identity()
            mean, std = _MEAN_STD[kind]
            self.register_buffer("mean", torch.tensor(mean).view(1, 3, 1, 1), persistent=False)
            self.register_buffer("std", torch.tensor(std).view(1, 3, 1, 1), persistent=False)
            nn.init.normal_(self.pos, std=0.02)
            nn.init.normal_(self.cls, std=0.02)

        def forward(self, x):                      # x: (B, 3, 224, 224) in [0, 1]
            w = getattr(self.patch, "w_lp", None)
            if getattr(self, "fused", False) and w is not None:
                # normalisation + patch extraction, the patch GEMM, then cls / pos in one pass
                p = self.patch.kernel_size[0]
                pt = _patchify(x, self.mean, self.std, p)
                t = _hlin(self.patch, pt) if getattr(self, "hip_gemm", False) else F.linear(pt, w, self.patch.b_lp)
                x = self.ln_pre(_tokens(t, self.cls, self.pos))
                delta = None
                for blk in self.blocks:
                    delta = blk.forward_fused(x, delta)
                x = self.ln_post(x[:, 0] + delta[:, 0].float())
                return x if isinstance(self.head, nn.Identity) else _lin(self.head, x)
            x = (x - self.mean) / self.std
            if w is None:
                x = self.patch(x).flatten(2).transpose(1, 2)
            else:
                # the stride-16 16x16 patch conv as ONE matrix product: (B*196, 3*16*16) x (768,
                # 768)^T, patches laid out (c, kh, kw) like the conv weight
                b, c, hh, ww = x.shape
                p = self.patch.kernel_size[0]
                x = x.to(w.dtype).reshape(b, c, hh // p, p, ww // p, p).permute(0, 2, 4, 1, 3, 5)
                x = F.linear(x.reshape(b, (hh // p) * (ww // p), c * p * p), w, self.patch.b_lp)
                x = x.float()
            x = torch.cat([self.cls.expand(x.shape[0], -1, -1), x], 1) + self.pos
            x = self.ln_pre(x)
            for blk in self.blocks:
                x = blk(x)
            x = self.ln_post(x[:, 0])
            return x if isinstance(self.head, nn.Identity) else _lin(self.head, x)

    class DreamSimEnsemble(nn.Module):
        """dino_vitb16 (768) | clip_vitb16 (512) | open_clip_vitb16 (512) -> 1792."""

        def __init__(self):
            super().__init__()
            self.towers = nn.ModuleList([ViT("dino", blocks=depth), ViT("clip", 512, blocks=depth),
                                         ViT("open_clip", 512, blocks=depth)])

        @property
        def dim(self):
            return 768 + 512 + 512

        def embed(self, x):
            parts = [F.normalize(t(x).float(), dim=-1) for t in self.towers]
            return torch.cat(parts, -1)

        def prepare_inference(self, dtype, fused=False, gelu_epilogue=False, hip_attn=None,
                              hip_gemm=None):
            """Cache low-precision copies of every matrix-product weight once (autocast would
            re-cast them on every forward); LayerNorms and the residual stream stay fp32.
            fused (bf16, on a GPU): residual add + LayerNorm + bf16 cast and QuickGELU run as
            single HIP passes (include/imgrec_vit.h).  gelu_epilogue (with fused, without
            hip_gemm): the GELU after fc1 as hipBLASLt's GELU_BIAS epilogue (_lin_gelu).
            hip_attn (with fused; default on): attention through the one-kernel
            vit_attention_bf16 (_attn) instead of torch SDPA.  hip_gemm (with fused; default
            on): every matrix product, with its bias and fc1's activation (QuickGELU; GELU in
            the erf form, or the tanh form with gelu_epilogue), on the HIP GEMM vit_linear_bf16
            (_hlin) instead of hipBLASLt."""
            for t in self.towers:
                t.fused = bool(fused) and dtype == torch.bfloat16
                t.hip_gemm = t.fused and (hip_gemm is None or bool(hip_gemm))
                for blk in t.blocks:
                    blk.gelu_epilogue = t.fused and bool(gelu_epilogue)
                    blk.hip_attn = t.fused and (hip_attn is None or bool(hip_attn))
                    blk.hip_gemm = t.hip_gemm
            for m in self.modules():
                if isinstance(m, (nn.Linear, nn.Conv2d)):
                    w = m.weight.detach()
                    m.w_lp = (w.reshape(w.shape[0], -1) if w.dim() > 2 else w).to(dtype).contiguous()
                    m.b_lp = m.bias.detach().to(dtype) if m.bias is not None else None
                    m.b_f32 = m.bias.detach().float().contiguous() if m.bias is not None else None
            return self

    if seed is not None:
        torch.manual_seed(seed)
    return DreamSimEnsemble()


def ensemble_state_from_towers(dino: dict, clip: dict, open_clip: dict) -> dict:
    """State dict of DreamSimEnsemble from the three towers' own checkpoints (layouts in the module
    docstring): DINO ViT-B/16 (timm / facebookresearch-dino names) and the ``visual`` parts of the
    OpenAI CLIP and OpenCLIP ViT-B/16 models (LoRA already merged)."""
    out = {}

    def strip(sd):
        return {(k[7:] if k.startswith("visual.") else k): v for k, v in sd.items()}

    d = strip(dino)
    pre = "towers.0."
    out[pre + "patch.weight"] = d["patch_embed.proj.weight"]
    out[pre + "patch.bias"] = d["patch_embed.proj.bias"]
    out[pre + "cls"] = d["cls_token"].reshape(1, 1, -1)
    out[pre + "pos"] = d["pos_embed"].reshape(1, -1, d["pos_embed"].shape[-1])
    nb = 1 + max(int(k.split(".")[1]) for k in d if k.startswith("blocks."))
    for i in range(nb):
        s_, o_ = f"blocks.{i}.", f"{pre}blocks.{i}."
        for a, b in (("norm1", "ln1"), ("norm2", "ln2"), ("attn.qkv", "qkv"), ("attn.proj", "proj"),
                     ("mlp.fc1", "fc1"), ("mlp.fc2", "fc2")):
            out[o_ + b + ".weight"] = d[s_ + a + ".weight"]
            out[o_ + b + ".bias"] = d[s_ + a + ".bias"]
    out[pre + "ln_post.weight"] = d["norm.weight"]
    out[pre + "ln_post.bias"] = d["norm.bias"]
    for t, sd in ((1, clip), (2, open_clip)):
        c = strip(sd)
        pre = f"towers.{t}."
        out[pre + "patch.weight"] = c["conv1.weight"]
        out[pre + "cls"] = c["class_embedding"].reshape(1, 1, -1)
        out[pre + "pos"] = c["positional_embedding"].reshape(1, *c["positional_embedding"].shape)
        out[pre + "ln_pre.weight"] = c["ln_pre.weight"]
        out[pre + "ln_pre.bias"] = c["ln_pre.bias"]
        nb = 1 + max(int(k.split(".")[2]) for k in c if k.startswith("transformer.resblocks."))
        for i in range(nb):
            s_, o_ = f"transformer.resblocks.{i}.", f"{pre}blocks.{i}."
            out[o_ + "ln1.weight"], out[o_ + "ln1.bias"] = c[s_ + "ln_1.weight"], c[s_ + "ln_1.bias"]
            out[o_ + "ln2.weight"], out[o_ + "ln2.bias"] = c[s_ + "ln_2.weight"], c[s_ + "ln_2.bias"]
            out[o_ + "qkv.weight"] = c[s_ + "attn.in_proj_weight"]
            out[o_ + "qkv.bias"] = c[s_ + "attn.in_proj_bias"]
            out[o_ + "proj.weight"] = c[s_ + "attn.out_proj.weight"]
            out[o_ + "proj.bias"] = c[s_ + "attn.out_proj.bias"]
            out[o_ + "fc1.weight"], out[o_ + "fc1.bias"] = c[s_ + "mlp.c_fc.weight"], c[s_ + "mlp.c_fc.bias"]
            out[o_ + "fc2.weight"], out[o_ + "fc2.bias"] = c[s_ + "mlp.c_proj.weight"], c[s_ + "mlp.c_proj.bias"]
        out[pre + "ln_post.weight"] = c["ln_post.weight"]
        out[pre + "ln_post.bias"] = c["ln_post.bias"]
        out[pre + "head.weight"] = c["proj"].t().contiguous()
    return out


class DreamSimVectorIndexer(BaseVectorIndexer):
    table_name = "dreamsim_vectors"
    vector_column = "dreamsim_vector_blob"
    id_column = "image_id"

    def __init__(self, db_path: str, base_dir: str, batch_size: int = 4096, model_batch: int = 128,
                 log_file: str = "dreamsim_indexer.log", log_dir: str = "logs",
                 weights_path: str | None = None, allow_random_init: bool = False,
                 device: str | None = None):
        super().__init__(db_path, base_dir, batch_size, log_file, log_dir)
        torch, _, _ = _torch()
        self.model_batch = model_batch
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self._log_and_print(f"Using device: {self.device}", level="info")
        self._setup_model(weights_path, allow_random_init)

    def _setup_model(self, weights_path, allow_random_init):
        torch, _, _ = _torch()
        model = build_ensemble(seed=0)
        if weights_path:
            state = torch.load(weights_path, map_location="cpu", weights_only=True)
            if {"dino", "clip", "open_clip"} <= set(state):       # the towers' own checkpoints
                state = ensemble_state_from_towers(state["dino"], state["clip"], state["open_clip"])
            model.load_state_dict(state)
        elif not allow_random_init:
            raise RuntimeError("DreamSim ensemble weights are not available (the reference "
                               "downloads them at run time; pass weights_path=...)")
        self.model = model.to(self.device).eval()
        if self.device.type == "cuda":       # bf16 products + the fused HIP elementwise passes
            self.model.prepare_inference(torch.bfloat16, fused=True, gelu_epilogue=True)
        self.dim = model.dim
        self._log_and_print("DreamSim model loaded and warmed up.", level="info")

    def embed_tensor(self, images):
        """(B, 3, 224, 224) float tensor in [0, 1] on the model device -> (B, 1792) normalised.
        On the GPU the matrix products run in bf16 from weights cast once (prepare_inference),
        LayerNorm and the residual stream in fp32 — what autocast does, without re-casting every
        weight on every forward — with the residual add + LayerNorm + bf16 cast and QuickGELU as
        single HIP passes (include/imgrec_vit.h)."""
        torch, _, F = _torch()
        with torch.no_grad():
            emb = self.model.embed(images)
        return F.normalize(emb.float(), dim=-1)

    def _batch_image_to_vector(self, image_paths):
        torch, _, _ = _torch()
        images, valid = [], []
        for rel in image_paths:
            arr = load_image(self.base_dir / rel, img_size=(224, 224), normalize=True, as_array=True)
            if arr is None:
                self._log_and_print(f"Error loading {self.base_dir / rel}", level="warning")
                continue
            images.append(torch.from_numpy(np.ascontiguousarray(arr.transpose(2, 0, 1))))
            valid.append(rel)
        if not images:
            return torch.empty(0, self.dim), []
        batch = torch.stack(images).to(self.device)
        return self.embed_tensor(batch).cpu(), valid

    def compute_vectors(self, paths):
        results = [None] * len(paths)
        for start in range(0, len(paths), self.model_batch):
            chunk = paths[start:start + self.model_batch]
            emb, valid = self._batch_image_to_vector(chunk)
            pos = {p: i for i, p in enumerate(valid)}
            for j, rel in enumerate(chunk):
                if rel in pos:
                    results[start + j] = emb[pos[rel]].numpy().astype("float32")
        return results
