#ifndef LIBWEBP_AMD_H2D_SDMA_H_
#define LIBWEBP_AMD_H2D_SDMA_H_
#include <stddef.h>
#include <stdint.h>

/* Copy `bytes` from pinned host memory to device memory of HIP device
 * `device` on an SDMA engine and wait for it (h2d_sdma.c). Returns 1 when
 * done, 0 when the copy could not be issued (the caller then uses
 * hipMemcpy). */
int h2d_sdma_upload(int device, void* dst, const void* src, size_t bytes);

/* Start such a copy without waiting (the next batch's frames while this one
 * encodes): 1 and *handle set when issued, 0 when not (nothing to finish).
 * h2d_sdma_finish waits for it and releases the handle. */
int h2d_sdma_upload_start(int device, void* dst, const void* src, size_t bytes, uint64_t* handle);
void h2d_sdma_finish(uint64_t handle);

/* The other direction: device memory of `device` to pinned host memory.
 * The caller has drained the stream that produced `src`. */
int d2h_sdma_download(int device, void* dst, const void* src, size_t bytes);

/* WEBP_AMD_FAULT_REPORT=1: print GPU memory faults (address, reason) to stderr */
void vp8g_fault_report_init(void);

#endif
