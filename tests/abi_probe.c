/* Prints sizeof/offsetof of the encoder ABI structs; compiled by
 * tests/test_abi.py against our include/webp/encode.h (and, in the dev
 * container, by tests/golden/make_golden.py against the reference header). */
#include <stddef.h>
#include <stdio.h>
#include "webp/encode.h"
#define F(T, m) printf("\"%s.%s\": %zu,\n", #T, #m, offsetof(T, m))
int main(void) {
  printf("{\n");
  printf("\"sizeof.WebPConfig\": %zu,\n", sizeof(WebPConfig));
  printf("\"sizeof.WebPPicture\": %zu,\n", sizeof(WebPPicture));
  printf("\"sizeof.WebPAuxStats\": %zu,\n", sizeof(WebPAuxStats));
  printf("\"sizeof.WebPMemoryWriter\": %zu,\n", sizeof(WebPMemoryWriter));
  F(WebPConfig, quality); F(WebPConfig, method); F(WebPConfig, segments);
  F(WebPConfig, pass); F(WebPConfig, partition_limit); F(WebPConfig, use_sharp_yuv);
  F(WebPConfig, qmax);
  F(WebPPicture, width); F(WebPPicture, y); F(WebPPicture, y_stride); F(WebPPicture, a);
  F(WebPPicture, argb); F(WebPPicture, writer); F(WebPPicture, custom_ptr);
  F(WebPPicture, stats); F(WebPPicture, error_code); F(WebPPicture, progress_hook);
  F(WebPPicture, user_data); F(WebPPicture, memory_); F(WebPPicture, memory_argb_);
  F(WebPAuxStats, PSNR); F(WebPAuxStats, block_count); F(WebPAuxStats, residual_bytes);
  F(WebPAuxStats, segment_level); F(WebPAuxStats, lossless_features); F(WebPAuxStats, pad);
  F(WebPMemoryWriter, size); F(WebPMemoryWriter, max_size);
  printf("\"abi\": %d\n}\n", WEBP_ENCODER_ABI_VERSION);
  return 0;
}
