#!/usr/bin/env python3
"""DreamSim-architecture forward (vector_scripts/create_dreamsim_vector.py) on PyTorch-ROCm:
images/s of variants on one GPU, random weights, bf16 autocast, 224 x 224 inputs.

  autocast   bf16 autocast over the fp32 module (round 1's form: every weight re-cast per call)
  base       the module as shipped (weights cast to bf16 once, patch embedding as one GEMM,
             fp32 LayerNorm / residual, SDPA default backend)
  bN         model batch N
  sdpa=X     SDPA restricted to one backend (flash / efficient / math)
  graph      the forward captured once in a HIP graph and replayed
  fused      residual add + LayerNorm + bf16 cast and QuickGELU as single HIP passes
             (include/imgrec_vit.h)
  fused_gelu_lt  fused + fc1's GELU as the hipBLASLt GELU_BIAS epilogue (torch._addmm_activation)
             + attention as one HIP kernel (vit_attention_bf16, the default since round 3)
  fused_gelu_lt_sdpa  the same with attention on torch SDPA (round 3's earlier form)
  hip_gemm   fused + every GEMM (bias, fc1's erf GELU / QuickGELU in the epilogue) on the HIP
             kernel vit_linear_bf16 instead of hipBLASLt (the default since round 4)
  hip_gemm_tanh  the same with fc1's GELU in the tanh form (gelu_epilogue: what
             DreamSimVectorIndexer ships, as hipBLASLt's GELU_BIAS epilogue computes it)
  X@B        variant X with SDPA restricted to backend B (flash / efficient / math)

FLOP per image: 3 ViT-B/16 towers at 224 (197 tokens): 2 x 17.58 GMAC each -> 105.5 GFLOP;
bf16 MFMA fraction = images/s x 105.5 GFLOP / 2516.8 TFLOP/s.  Prints one JSON line per variant.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GFLOP_PER_IMAGE = 3 * 2 * 17.58
PEAK = 2516.8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="128,256,512")
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--variants", default="autocast,base,sdpa=flash,sdpa=efficient,graph")
    a = ap.parse_args()
    import torch
    from torch.nn.attention import SDPBackend, sdpa_kernel
    from image_recommender_amd.vector_scripts.create_dreamsim_vector import build_ensemble
    dev = torch.device("cuda", 0)
    model = build_ensemble(seed=0).to(dev).eval()
    cached = build_ensemble(seed=0).to(dev).eval().prepare_inference(torch.bfloat16)
    fused = build_ensemble(seed=0).to(dev).eval().prepare_inference(torch.bfloat16, fused=True,
                                                                   hip_attn=False, hip_gemm=False)
    fused_lt = build_ensemble(seed=0).to(dev).eval().prepare_inference(torch.bfloat16, fused=True,
                                                                      gelu_epilogue=True, hip_gemm=False)
    fused_lt_sdpa = build_ensemble(seed=0).to(dev).eval().prepare_inference(
        torch.bfloat16, fused=True, gelu_epilogue=True, hip_attn=False, hip_gemm=False)
    hip_gemm = build_ensemble(seed=0).to(dev).eval().prepare_inference(torch.bfloat16, fused=True)
    hip_gemm_tanh = build_ensemble(seed=0).to(dev).eval().prepare_inference(torch.bfloat16, fused=True,
                                                                           gelu_epilogue=True)

    def embed(x):
        if var_now[0].startswith("autocast"):        # per-call weight casts (the r01 form)
            with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
                return torch.nn.functional.normalize(model.embed(x).float(), dim=-1)
        with torch.no_grad():                          # weights cast once (the shipped form)
            m = {"fused": fused, "fused_gelu_lt": fused_lt, "fused_gelu_lt_sdpa": fused_lt_sdpa,
                 "hip_gemm": hip_gemm, "hip_gemm_tanh": hip_gemm_tanh}.get(var_now[0].split("@")[0], cached)
            return torch.nn.functional.normalize(m.embed(x).float(), dim=-1)

    var_now = [""]
    backends = {"flash": SDPBackend.FLASH_ATTENTION, "efficient": SDPBackend.EFFICIENT_ATTENTION,
                "math": SDPBackend.MATH}
    for bs in [int(v) for v in a.batches.split(",")]:
        x = torch.rand((bs, 3, 224, 224), device=dev)
        for var in a.variants.split(","):
            var_now[0] = var
            try:
                if var.startswith("sdpa="):
                    ctx = sdpa_kernel([backends[var[5:]]])
                elif "@" in var:                          # model variant @ SDPA backend
                    ctx = sdpa_kernel([backends[var.split("@")[1]]])
                else:
                    import contextlib
                    ctx = contextlib.nullcontext()
                with ctx:
                    if var == "graph":
                        embed(x)
                        torch.cuda.synchronize()
                        g = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(g):
                            y = embed(x)
                        run = g.replay
                    else:
                        run = lambda: embed(x)
                    for _ in range(2):
                        run()
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(a.iters):
                        run()
                    torch.cuda.synchronize()
                    dt = (time.perf_counter() - t0) / a.iters
                ips = bs / dt
                print(json.dumps({"variant": var, "batch": bs, "images_per_s": ips,
                                  "tflops": ips * GFLOP_PER_IMAGE / 1e3,
                                  "bf16_mfma_frac": ips * GFLOP_PER_IMAGE / 1e3 / PEAK}), flush=True)
            except Exception as e:   # a backend unavailable for these shapes
                print(json.dumps({"variant": var, "batch": bs, "error": str(e)[:200]}), flush=True)


if __name__ == "__main__":
    main()
