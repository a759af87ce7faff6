"""Slot packing of the colour decode pipeline (CPU: the worker function run in-process).

A slot's pixel region is rounded down to a multiple of 48 and the worker reports the end of its
last image as the bytes to upload, so an upload never exceeds the device buffer of pix_cap bytes
(with chunk = 32 the unrounded pix_cap % 48 == 32 and a nearly full slot reported up
to 47 bytes past it)."""
from multiprocessing import shared_memory

import numpy as np
import pytest

from image_recommender_amd.vector_scripts import decode_pipeline as dp
from oracle.color_hist import color_counts


@pytest.mark.parametrize("chunk", [32, 64, 7])
def test_slot_never_overflows_pix_cap(tmp_path, chunk):
    from PIL import Image
    slot_bytes = 1 << 16
    pix_cap = dp._pix_cap(slot_bytes, chunk)
    assert pix_cap % dp._ALIGN == 0 and pix_cap <= slot_bytes - 16 * chunk
    # images whose sizes are not multiples of 48 bytes, enough to overflow one slot
    rng = np.random.default_rng(chunk)
    paths, imgs = [], []
    side = int((1.6 * slot_bytes / chunk / 3) ** 0.5)     # ~1.6 slots of pixels per chunk
    for i in range(chunk):
        h, w = int(rng.integers(side * 2 // 3, side * 4 // 3)), int(rng.integers(side * 2 // 3, side * 4 // 3))
        a = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        p = tmp_path / f"im{i}.png"
        Image.fromarray(a, "RGB").save(p)
        paths.append(str(p))
        imgs.append(a)
    shm = shared_memory.SharedMemory(create=True, size=2 * slot_bytes)
    try:
        dp._attach(shm.name, slot_bytes, chunk)
        slot, status, used, n, spill = dp._decode_chunk((1, paths))
        assert slot == 1 and 0 < n <= chunk
        assert used <= pix_cap, (used, pix_cap)
        base = slot_bytes
        meta = np.ndarray((2 * chunk,), np.int64, buffer=shm.buf, offset=base + slot_bytes - 16 * chunk)
        offs, npix = meta[:n], meta[n:2 * n]
        assert used == offs[-1] + 3 * npix[-1]
        buf = np.ndarray((slot_bytes,), np.uint8, buffer=shm.buf, offset=base)
        for i, st in enumerate(status):
            if st >= 0:
                a = imgs[i]
                assert offs[st] % dp._ALIGN == 0 and offs[st] + a.nbytes <= pix_cap
                got = buf[offs[st]:offs[st] + a.nbytes]
                np.testing.assert_array_equal(got, a.reshape(-1))
                assert npix[st] == a.shape[0] * a.shape[1]
            else:
                assert st == -2
                np.testing.assert_array_equal(color_counts(spill[i]), color_counts(imgs[i]))
        assert (np.array(status) == -2).any(), "the case must fill the slot"
    finally:
        dp._W.clear()
        shm.close()
        shm.unlink()
