/*
 * imgrec_color.h — C ABI of the per-image RGB colour histogram (the reference's colour feature).
 *
 * Replaces ColorVectorIndexer.compute_color_vector_worker
 * (/root/reference/vector_scripts/create_color_vector.py:18-52): per channel
 * cv2.calcHist([c], [0], None, [bins], [0, 256]) (bin = floor(v * bins / 256)), channels
 * concatenated in R, G, B order (the image was converted BGR->RGB by load_image,
 * vector_scripts/create_vector_base.py:239-247), then divided by its L2 norm when that norm is
 * non-zero (create_color_vector.py:48-51).  Output per image: 3*bins float32.
 *
 * Input is a batch of decoded images, each stored as interleaved 8-bit RGB (HWC), concatenated in
 * one byte buffer: image i occupies bytes [offsets[i], offsets[i] + 3*npix[i]).
 */
#ifndef IMGREC_COLOR_H
#define IMGREC_COLOR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define COLOR_HIST_MAX_BINS 32

/* Device pointers; enqueued on `stream` (hipStream_t, NULL = default stream), no sync.
 * counts (nullable): n_images * 3*bins raw uint32 bin counts. */
int color_hist_device(const uint8_t* pixels, const int64_t* offsets, const int64_t* npix,
                      int64_t n_images, int bins, float* out, uint32_t* counts, void* stream);

/* Host convenience wrapper: copies in, computes on `device` (-1 = current), copies out, syncs. */
int color_hist_host(const uint8_t* pixels, int64_t total_bytes, const int64_t* offsets,
                    const int64_t* npix, int64_t n_images, int bins, int device, float* out,
                    uint32_t* counts);

/* Page-lock a host range (hipHostRegister) so hipMemcpyAsync from it is an asynchronous DMA — the
 * shared-memory slots the decode pipeline's worker processes write decoded images into
 * (vector_scripts/decode_pipeline.py).  color_host_unregister releases it. */
int color_host_register(void* ptr, int64_t bytes);
int color_host_unregister(void* ptr);

/* One decoded batch in a page-locked host slot: `bytes` of pixels and the batch's meta (n image
 * offsets into the pixels, then n pixel counts, int64) are copied to dev_pixels / dev_meta on
 * `stream`, then the n histograms are computed into dev_out (and dev_counts when not NULL).
 * Asynchronous: the slot may be rewritten once the stream has passed this call. */
int color_hist_batch_async(const uint8_t* host_pixels, int64_t bytes, const int64_t* host_meta,
                           int64_t n, int bins, uint8_t* dev_pixels, int64_t* dev_meta,
                           float* dev_out, uint32_t* dev_counts, void* stream);

/* Same error-string convention as knn_last_error(). */
const char* color_hist_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* IMGREC_COLOR_H */
