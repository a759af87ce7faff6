"""DreamSim-ensemble embeddings on PyTorch-ROCm — drop-in for create_dreamsim_vector.py.

The reference (/root/reference/vector_scripts/create_dreamsim_vector.py:11-125) loads
``dreamsim(pretrained=True, dreamsim_type="ensemble", normalize_embeds=True)`` (dreamsim 0.2.1,
weights downloaded at run time), embeds batches of 128 images resized to 224x224 (LANCZOS) and
L2-normalises each embedding (:92).  The ensemble is three ViT-B/16 towers — DINO (768-d CLS),
OpenAI CLIP and OpenCLIP (512-d projected CLS) — concatenated to 1792 dimensions.

This module implements that architecture in plain PyTorch (bf16 autocast, fused
scaled-dot-product attention — it runs on PyTorch-ROCm, no hand kernel is required for it).
Pretrained weights cannot be fetched here: ``DreamSimVectorIndexer`` needs ``weights_path`` (a
state dict for ``DreamSimEnsemble``) and raises like the reference does when the model cannot be
loaded; ``allow_random_init=True`` builds a randomly initialised model for throughput
measurements only (its embeddings are not DreamSim embeddings).
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


def build_ensemble(seed: int | None = 0):
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
            qkv = self.qkv(self.ln1(x)).view(b, n, 3, self.heads, c // self.heads)
            q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)
            a = F.scaled_dot_product_attention(q, k, v)
            x = x + self.proj(a.transpose(1, 2).reshape(b, n, c))
            h = self.fc1(self.ln2(x))
            h = h * torch.sigmoid(1.702 * h) if self.quick_gelu else F.gelu(h)
            return x + self.fc2(h)

    class ViT(nn.Module):
        """ViT-B/16 tower; `out_dim` adds a CLIP-style projection of the CLS token."""

        def __init__(self, kind, out_dim=None, depth=12, dim=768, patch=16, img=224):
            super().__init__()
            self.kind = kind
            self.patch = nn.Conv2d(3, dim, patch, patch, bias=(kind == "dino"))
            self.cls = nn.Parameter(torch.zeros(1, 1, dim))
            self.pos = nn.Parameter(torch.zeros(1, (img // patch) ** 2 + 1, dim))
            self.ln_pre = nn.LayerNorm(dim) if kind != "dino" else nn.Identity()
            self.blocks = nn.ModuleList(Block(dim, quick_gelu=(kind == "clip")) for _ in range(depth))
            self.ln_post = nn.LayerNorm(dim)
            self.head = nn.Linear(dim, out_dim, bias=False) if out_dim else nn.Identity()
            mean, std = _MEAN_STD[kind]
            self.register_buffer("mean", torch.tensor(mean).view(1, 3, 1, 1), persistent=False)
            self.register_buffer("std", torch.tensor(std).view(1, 3, 1, 1), persistent=False)
            nn.init.normal_(self.pos, std=0.02)
            nn.init.normal_(self.cls, std=0.02)

        def forward(self, x):                      # x: (B, 3, 224, 224) in [0, 1]
            x = (x - self.mean) / self.std
            x = self.patch(x).flatten(2).transpose(1, 2)
            x = torch.cat([self.cls.expand(x.shape[0], -1, -1), x], 1) + self.pos
            x = self.ln_pre(x)
            for blk in self.blocks:
                x = blk(x)
            return self.head(self.ln_post(x[:, 0]))

    class DreamSimEnsemble(nn.Module):
        """dino_vitb16 (768) | clip_vitb16 (512) | open_clip_vitb16 (512) -> 1792."""

        def __init__(self):
            super().__init__()
            self.towers = nn.ModuleList([ViT("dino"), ViT("clip", 512), ViT("open_clip", 512)])

        @property
        def dim(self):
            return 768 + 512 + 512

        def embed(self, x):
            parts = [F.normalize(t(x).float(), dim=-1) for t in self.towers]
            return torch.cat(parts, -1)

    if seed is not None:
        torch.manual_seed(seed)
    return DreamSimEnsemble()


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
            model.load_state_dict(state)
        elif not allow_random_init:
            raise RuntimeError("DreamSim ensemble weights are not available (the reference "
                               "downloads them at run time; pass weights_path=...)")
        self.model = model.to(self.device).eval()
        self.dim = model.dim
        self._log_and_print("DreamSim model loaded and warmed up.", level="info")

    def embed_tensor(self, images):
        """(B, 3, 224, 224) float tensor in [0, 1] on the model device -> (B, 1792) normalised."""
        torch, _, F = _torch()
        with torch.no_grad(), torch.autocast(device_type=self.device.type, dtype=torch.bfloat16,
                                             enabled=self.device.type == "cuda"):
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
