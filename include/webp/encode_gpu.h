/* libwebp_amd -- batched MI355X extension of the libwebp encoder ABI.
 *
 * The reference has no batch entry point: its unit of work is one
 * WebPEncode(config, picture) call (src/webp/encode.h:544,
 * src/enc/webp_enc.c:330-410). This header adds the batched form that the
 * GPU needs for occupancy: many same-sized frames resident in HBM are
 * converted, analysed, rate-distortion searched and tokenised in one set of
 * kernel launches, then the boolean-coder tail runs on a host thread pool.
 * The bitstream of every frame is byte-identical to what WebPEncode() of the
 * reference produces for the same pixels and config.
 *
 * All pointers are plain device or host addresses; streams are hipStream_t
 * passed as void*. No framework types cross this boundary.
 */
#ifndef WEBP_WEBP_ENCODE_GPU_H_
#define WEBP_WEBP_ENCODE_GPU_H_

#include "./encode.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct WebPGpuBatch WebPGpuBatch;

/* Create an encoder for up to max_frames frames of width x height, on HIP
 * device `device`, with `config` (lossy, method 3..6). host_threads <= 0
 * picks a default (env WEBP_AMD_THREADS, else min(16, the rank's host-thread
 * budget, WebPGpuHostThreadBudget)).
 * Returns NULL on error (no GPU, bad config, out of memory). */
WEBP_EXTERN WebPGpuBatch* WebPGpuBatchNew(int device, int width, int height,
                                          int max_frames,
                                          const WebPConfig* config,
                                          int host_threads);
WEBP_EXTERN void WebPGpuBatchDelete(WebPGpuBatch* batch);

/* Encode num_frames RGBA frames already in device memory: frame f starts at
 * (const uint8_t*)rgba_dev + f * frame_stride, rows are row_stride bytes.
 * `stream` (hipStream_t or NULL) orders the device work after the caller's
 * producer kernels. Returns 1 on success; per-frame status via
 * WebPGpuBatchError(). Outputs stay valid until the next call. */
WEBP_EXTERN int WebPGpuBatchEncodeRGBA(WebPGpuBatch* batch,
                                       const void* rgba_dev,
                                       size_t frame_stride, int row_stride,
                                       int num_frames, void* stream);

/* Same, from host memory (includes the PCIe upload). */
WEBP_EXTERN int WebPGpuBatchEncodeRGBAHost(WebPGpuBatch* batch,
                                           const uint8_t* rgba_host,
                                           size_t frame_stride, int row_stride,
                                           int num_frames);

/* Same, and while this batch encodes, upload the next one: rgba_next
 * (page-locked host memory, same frame count and strides) goes to the
 * device on a copy engine, and the next call whose rgba_host is rgba_next
 * (same geometry) encodes from that copy instead of uploading. rgba_next
 * must not change until then; a call for other frames discards it.
 * rgba_next NULL (or pageable): WebPGpuBatchEncodeRGBAHost. */
WEBP_EXTERN int WebPGpuBatchEncodeRGBAHostPrefetch(WebPGpuBatch* batch,
                                                   const uint8_t* rgba_host,
                                                   const uint8_t* rgba_next,
                                                   size_t frame_stride,
                                                   int row_stride,
                                                   int num_frames);

/* Results of the last encode call. */
WEBP_EXTERN size_t WebPGpuBatchOutputSize(const WebPGpuBatch* batch, int frame);
WEBP_EXTERN const uint8_t* WebPGpuBatchOutput(const WebPGpuBatch* batch,
                                              int frame);
WEBP_EXTERN int WebPGpuBatchError(const WebPGpuBatch* batch, int frame);

/* Per-stage times of the last call in microseconds:
 * [0] import+analysis kernels (wall), [1] host segment setup, [2] RD/token
 * and boolean-coder kernels + result copies (wall), [3] partition copies,
 * [4] host tail (partition 0 + assembly), [5] total; from HIP events on the
 * batch's stream: [6] k_encode, [7] k_import + k_analyze, [8] k_emit. */
WEBP_EXTERN void WebPGpuBatchTimings(const WebPGpuBatch* batch,
                                     double timings_us[10]);

/* Number of 16-bit VP8 tokens the RD/token kernel produced for frame f of
 * the last call (token_enc.c:31-35 format); used to price the kernel's HBM
 * traffic in benchmarks. */
WEBP_EXTERN size_t WebPGpuBatchTokenCount(const WebPGpuBatch* batch, int frame);

/* Profiling: shader-clock cycles the RD/token kernel spent per stage of
 * frame f, summed over its macroblocks: [0] MB load + cost refresh +
 * predictors, [1] intra16, [2] intra4, [3] chroma (+ m5 final pass),
 * [4] mode info + SSE, [5] token count/write, [6] statistics fold/replay,
 * [7] context + boundary update. */
WEBP_EXTERN int WebPGpuBatchStageCycles(const WebPGpuBatch* batch, int frame,
                                        uint64_t cycles[8]);

/* Debug/parity hooks (used by tests): copy the device YUV420 planes of frame
 * f (Y | U | V, contiguous, strides width and (width+1)/2), and the per-MB
 * decisions (20 bytes per MB: type, uv_mode, segment, skip, modes[16]). */
WEBP_EXTERN int WebPGpuBatchGetYUV(const WebPGpuBatch* batch, int frame,
                                   uint8_t* dst);
/* Debug: frame f's VP8 token stream (token_enc.c:31-35 format) and the final
 * probabilities, available when the batch codes partition 1 on the host
 * (WEBP_AMD_HOST_EMIT=1); returns 0 otherwise. */
WEBP_EXTERN int WebPGpuBatchGetTokens(const WebPGpuBatch* batch, int frame, uint16_t* dst,
                                      size_t max_tokens);
WEBP_EXTERN int WebPGpuBatchGetMBInfo(const WebPGpuBatch* batch, int frame,
                                      uint8_t* dst);

/* Benchmark/test utility: write frames first_frame .. first_frame+n-1 of
 * the syn-v1 synthetic RGBA sequence into device memory. */
WEBP_EXTERN int WebPGpuSynthRGBA(void* rgba_dev, size_t frame_stride, int width,
                                 int height, int first_frame, int num_frames,
                                 int seed, void* stream);

/* Text of the first HIP/runtime error seen by this thread ("" if none). */
WEBP_EXTERN const char* WebPGpuLastError(void);

/* The host CPUs this process's engines on `device` run their threads on:
 * the device's NUMA node (sysfs), within the process affinity, split evenly
 * between the LOCAL_WORLD_SIZE ranks sharing the node (rank r on device r).
 * Writes up to max_cpus CPU ids into cpus and returns how many there are
 * (0 when the node is unknown: threads are then not pinned). */
WEBP_EXTERN int WebPGpuHostCpus(int device, int* cpus, int max_cpus);

/* Host-thread budget of this rank on `device`: the cgroup CPU quota (or
 * WEBP_AMD_CPU_QUOTA) over LOCAL_WORLD_SIZE, capped by the pinned CPUs above
 * and the online CPUs. All engines of the process draw the helper threads of
 * their host phases from one pool of this size; *busy (may be NULL) receives
 * the threads inside host phases right now. */
WEBP_EXTERN int WebPGpuHostThreadBudget(int device, int* busy);

/* Number of HIP devices visible (0 when no GPU / no driver). */
WEBP_EXTERN int WebPGpuDeviceCount(void);

#ifdef __cplusplus
}
#endif

#endif /* WEBP_WEBP_ENCODE_GPU_H_ */
