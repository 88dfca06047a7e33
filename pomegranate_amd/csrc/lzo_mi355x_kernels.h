/* lzo_mi355x_kernels.h -- internal launch interface between the host C code
 * (lzo_host.c) and the HIP kernels (lzo1x_kernels.hip). */
#ifndef POM_LZO_MI355X_KERNELS_H
#define POM_LZO_MI355X_KERNELS_H 1

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

int lzo_mi355x_launch_compress(const uint8_t *src, const uint64_t *src_off,
                               const uint32_t *src_len, uint8_t *dst,
                               const uint64_t *dst_off, const uint32_t *dst_cap,
                               uint32_t *out_len, int32_t *status, uint32_t nblocks,
                               hipStream_t stream);

/* Exact (grammar-serial) decoder, lzo1x_decompress_safe semantics.  fb NULL:
 * grid entry b decodes block b (ngrid = nblocks).  Otherwise the fb[0] blocks
 * listed at fb[1..] are decoded by a grid of ngrid workgroups. */
int lzo_mi355x_launch_decompress_exact(const uint8_t *src, const uint64_t *src_off,
                                       const uint32_t *src_len, uint8_t *dst,
                                       const uint64_t *dst_off, const uint32_t *dst_cap,
                                       uint32_t *out_len, int32_t *status,
                                       const uint32_t *fb, uint32_t ngrid,
                                       uint32_t nblocks, hipStream_t stream);

/* Throughput decoder (lzo1x_decode_fast.hip).  Blocks it does not finish
 * exactly are appended to fb (fb[0] = count, must be 0 on entry) and get
 * status 0x7FFF0001 until the exact decoder runs on them. */
int lzo_mi355x_launch_decompress_fast(const uint8_t *src, const uint64_t *src_off,
                                      const uint32_t *src_len, uint8_t *dst,
                                      const uint64_t *dst_off, const uint32_t *dst_cap,
                                      uint32_t *out_len, int32_t *status, uint32_t *fb,
                                      uint32_t nblocks, hipStream_t stream);

int lzo_mi355x_launch_decoded_length(const uint8_t *src, const uint64_t *src_off,
                                     const uint32_t *src_len, uint32_t *out_len,
                                     int32_t *status, uint32_t nblocks, hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif
