#ifndef LIBWEBP_AMD_H2D_SDMA_H_
#define LIBWEBP_AMD_H2D_SDMA_H_
#include <stddef.h>

/* Copy `bytes` from pinned host memory to device memory of HIP device
 * `device` on an SDMA engine and wait for it (h2d_sdma.c). Returns 1 when
 * done, 0 when the copy could not be issued (the caller then uses
 * hipMemcpy). */
int h2d_sdma_upload(int device, void* dst, const void* src, size_t bytes);

/* The other direction: device memory of `device` to pinned host memory.
 * The caller has drained the stream that produced `src`. */
int d2h_sdma_download(int device, void* dst, const void* src, size_t bytes);

#endif
