/* Internal: WebPPicture buffer helpers shared by webp_api.c and
 * picture_tools.c (reference src/enc/picture_enc.c:25-183). */
#ifndef LIBWEBP_AMD_PICTURE_INTERNAL_H_
#define LIBWEBP_AMD_PICTURE_INTERNAL_H_

#include "webp/encode.h"

/* first error wins (webp_enc.c:306-315); returns 0 */
int vp8h_pic_error(const WebPPicture* pic, WebPEncodingError e);
/* size and colourspace checks of WebPEncode / picture allocation (sets the
 * picture's error code, returns 0 on failure) */
int vp8h_pic_validate(const WebPPicture* pic);
/* (re)allocate the ARGB / YUV(A) buffers of pic (previous ones freed) */
int vp8h_pic_alloc_argb(WebPPicture* p);
int vp8h_pic_alloc_yuva(WebPPicture* p);
/* forget (do not free) the buffers */
void vp8h_pic_reset_argb(WebPPicture* p);
void vp8h_pic_reset_yuva(WebPPicture* p);

#endif
