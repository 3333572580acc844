/* libwebp_amd -- basic types for the libwebp-compatible encoder C ABI.
 * Mirrors the reference's src/webp/types.h:21-66 (same type names and the
 * WEBP_EXTERN / WebPMalloc / WebPFree contract) so that callers written
 * against libwebp compile and link unchanged. */
#ifndef WEBP_WEBP_TYPES_H_
#define WEBP_WEBP_TYPES_H_

#include <stddef.h>
#include <stdint.h>

/* like the reference (src/webp/types.h:19-37): the headers write
 * `static WEBP_INLINE`, and so do callers that define their own helpers
 * (cwebp's stopwatch.h, the decoder and mux headers) */
#ifndef WEBP_INLINE
#if defined(__cplusplus) || !defined(__STRICT_ANSI__) || \
    (defined(__STDC_VERSION__) && __STDC_VERSION__ >= 199901L)
#define WEBP_INLINE inline
#else
#define WEBP_INLINE
#endif
#endif

#ifndef WEBP_EXTERN
#if defined(_WIN32)
#define WEBP_EXTERN extern __declspec(dllexport)
#else
#define WEBP_EXTERN extern __attribute__((visibility("default")))
#endif
#endif

/* Major byte of an ABI version must match; minor may differ. */
#define WEBP_ABI_IS_INCOMPATIBLE(a, b) (((a) >> 8) != ((b) >> 8))

#ifdef __cplusplus
extern "C" {
#endif

/* Allocation helpers: buffers handed out by this library (e.g. the output of
 * WebPEncodeRGBA) must be released with WebPFree. */
WEBP_EXTERN void* WebPMalloc(size_t size);
WEBP_EXTERN void WebPFree(void* ptr);

#ifdef __cplusplus
}
#endif

#endif /* WEBP_WEBP_TYPES_H_ */
