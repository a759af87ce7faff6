#!/usr/bin/env python3
"""Micro-probes of the DreamSim-architecture block at batch 512 (ViT-B/16: 197 tokens, 768 wide,
12 heads, MLP 3072), bf16 — which per-op forms are cheaper on this GPU.  One JSON line per probe:

  fc1+gelu     F.linear(bias) then F.gelu (erf)  vs  torch._addmm_activation(use_gelu=True)
               (hipBLASLt GELU_BIAS epilogue, tanh form) — time and max |difference| in bf16 ulps
  sdpa         SDPA on q/k/v as permuted views of the qkv GEMM output  vs  contiguous q/k/v
               (copies included), per backend that accepts the shape
  out-proj     a.transpose(1, 2).reshape(b, n, c) copy + F.linear  vs  the copy alone
"""
from __future__ import annotations

import json
import sys

import torch
import torch.nn.functional as F


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    b = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    n, c, h, mlp = 197, 768, 12, 3072
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(b * n, c, generator=g, device=dev).to(torch.bfloat16)
    w1 = (torch.randn(mlp, c, generator=g, device=dev) * c ** -0.5).to(torch.bfloat16)
    b1 = (torch.randn(mlp, generator=g, device=dev) * 0.02).to(torch.bfloat16)
    t_ref = timeit(lambda: F.gelu(F.linear(x, w1, b1)))
    t_lin = timeit(lambda: F.linear(x, w1, b1))
    try:
        t_fused = timeit(lambda: torch._addmm_activation(b1, x, w1.t(), use_gelu=True))
        ref = F.gelu(F.linear(x, w1, b1).float())
        got = torch._addmm_activation(b1, x, w1.t(), use_gelu=True).float()
        ulp = (ref.abs() * 2.0 ** -8).clamp_min(2.0 ** -133)
        dmax = float(((got - ref).abs() / ulp).max())
    except Exception as e:   # noqa: BLE001
        t_fused, dmax = None, repr(e)
    print(json.dumps({"probe": "fc1+gelu", "batch": b, "linear_then_gelu_ms": t_ref,
                      "linear_alone_ms": t_lin, "addmm_activation_gelu_ms": t_fused,
                      "max_diff_bf16_ulps_vs_erf_fp32": dmax}), flush=True)

    wq = (torch.randn(3 * c, c, generator=g, device=dev) * c ** -0.5).to(torch.bfloat16)
    bq = torch.zeros(3 * c, device=dev, dtype=torch.bfloat16)
    qkv = F.linear(x, wq, bq).view(b, n, 3, h, c // h)
    q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)
    qc, kc, vc = q.contiguous(), k.contiguous(), v.contiguous()
    from torch.nn.attention import SDPBackend, sdpa_kernel
    res = {"probe": "sdpa", "batch": b}
    for name, be in (("default", None), ("flash", SDPBackend.FLASH_ATTENTION),
                     ("efficient", SDPBackend.EFFICIENT_ATTENTION), ("math", SDPBackend.MATH)):
        for form, args in (("views", (q, k, v)), ("contiguous", (qc, kc, vc))):
            try:
                if be is None:
                    t = timeit(lambda: F.scaled_dot_product_attention(*args), iters=10)
                else:
                    with sdpa_kernel(be):
                        t = timeit(lambda: F.scaled_dot_product_attention(*args), iters=10)
            except Exception as e:   # noqa: BLE001
                t = repr(e)[:80]
            res[f"{name}_{form}_ms"] = t
    res["contiguous_copy_ms"] = timeit(lambda: (q.contiguous(), k.contiguous(), v.contiguous()))
    print(json.dumps(res), flush=True)

    a = F.scaled_dot_product_attention(qc, kc, vc)
    wp = (torch.randn(c, c, generator=g, device=dev) * c ** -0.5).to(torch.bfloat16)
    print(json.dumps({"probe": "out-proj", "batch": b,
                      "copy_ms": timeit(lambda: a.transpose(1, 2).reshape(b, n, c)),
                      "copy_plus_linear_ms": timeit(lambda: F.linear(a.transpose(1, 2).reshape(b, n, c), wp))}),
          flush=True)


if __name__ == "__main__":
    main()
