"""Colour-histogram kernel rate (csrc/color_hist.hip) on device-resident 256 x 256 RGB images:
GB/s of pixel bytes per launch from HIP events.  Measurement tool; one JSON line per bin count."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from image_recommender_amd.vector_scripts.create_color_vector import color_histograms_device  # noqa: E402

torch.cuda.set_device(0)
n, h, w = int(os.environ.get("IMAGES", 16384)), 256, 256
g = torch.Generator(device="cuda").manual_seed(5)
pix = torch.randint(0, 256, (n * h * w * 3,), dtype=torch.uint8, device="cuda", generator=g)
npix = torch.full((n,), h * w, dtype=torch.int64, device="cuda")
offs = torch.arange(n, dtype=torch.int64, device="cuda") * (h * w * 3)
for bins in (16, 8):
    for _ in range(3):
        color_histograms_device(pix, offs, npix, bins)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    e0.record()
    for _ in range(reps):
        color_histograms_device(pix, offs, npix, bins)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(json.dumps({"bins": bins, "images": n, "ms": ms, "images_per_s": n / ms * 1e3,
                      "gbs": pix.numel() / ms / 1e6, "lib": os.environ.get("IMGREC_LIB_NAME", "libimgrec.so")}),
          flush=True)
