/* lzo_mi355x_kernels.h -- internal launch interface between the host C code
 * (lzo_host.c) and the HIP kernels (lzo1x_kernels.hip). */
#ifndef POM_LZO_MI355X_KERNELS_H
#define POM_LZO_MI355X_KERNELS_H 1

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status of a block lzo1x_encode_fast_kernel left to the general encoder */
#define LZO_MI355X_ENC_PENDING 0x7FFF0002

#define LZO_MI355X_FAST_MAX_N (1u << 24)   /* the throughput encoder's largest block (kMaxN) */

/* Throughput encoder (lzo1x_encode_fast.hip), blocks of up to 16 MiB; larger
 * blocks get status LZO_MI355X_ENC_PENDING.  With scratch (scratch_bytes of
 * device memory, lzo_mi355x_compress_scratch()) the dictionaries live there
 * and 16 blocks per CU are parsed at once; without, in LDS (4 per CU). */
int lzo_mi355x_launch_compress_fast(const uint8_t *src, const uint64_t *src_off,
                                    const uint32_t *src_len, uint8_t *dst,
                                    const uint64_t *dst_off, const uint32_t *dst_cap,
                                    uint32_t *out_len, int32_t *status, uint32_t nblocks,
                                    void *scratch, size_t scratch_bytes, hipStream_t stream);

/* General encoder (lzo1x_kernels.hip), any block size.
 * pending_only: only blocks whose status is LZO_MI355X_ENC_PENDING. */
int lzo_mi355x_launch_compress(const uint8_t *src, const uint64_t *src_off,
                               const uint32_t *src_len, uint8_t *dst,
                               const uint64_t *dst_off, const uint32_t *dst_cap,
                               uint32_t *out_len, int32_t *status, uint32_t nblocks,
                               int pending_only, hipStream_t stream);

/* Exact (grammar-serial) decoder, lzo1x_decompress_safe semantics, or with
 * `unchecked` those of the unchecked lzo1x_decompress.  fb NULL: grid entry b
 * decodes block b (ngrid = nblocks).  Otherwise the *fb blocks listed at
 * fb_ids[] are decoded by a grid of ngrid workgroups. */
int lzo_mi355x_launch_decompress_exact(const uint8_t *src, const uint64_t *src_off,
                                       const uint32_t *src_len, uint8_t *dst,
                                       const uint64_t *dst_off, const uint32_t *dst_cap,
                                       uint32_t *out_len, int32_t *status,
                                       const uint32_t *fb, const uint32_t *fb_ids,
                                       uint32_t ngrid, uint32_t nblocks, int unchecked,
                                       hipStream_t stream);

/* Exact decoder over blocks of consecutive streams (the hvfs_fwritev column
 * layout): each stream decodes with lzo1x_decompress_safe semantics right
 * after the previous one's output; out_len = the total. */
int lzo_mi355x_launch_decompress_concat(const uint8_t *src, const uint64_t *src_off,
                                        const uint32_t *src_len, uint8_t *dst,
                                        const uint64_t *dst_off, const uint32_t *dst_cap,
                                        uint32_t *out_len, int32_t *status, uint32_t nblocks,
                                        hipStream_t stream);

/* Throughput decoder (lzo1x_decode_fast.hip).  Blocks it does not finish
 * exactly are appended to fallback_ids[] (*fallback = count, must be 0 on
 * entry) and get status 0x7FFF0001 until the exact decoder runs on them.
 * ops: nsets op-slot sets of lzo_mi355x_fast_ops_bytes_per_block() bytes,
 * shared by the workgroups through a pool (pool: LZO_MI355X_FAST_POOL_BYTES
 * of counters, ring: nsets u64, all zero on entry); nsets = min(nblocks,
 * lzo_mi355x_fast_resident_blocks()) keeps every resident workgroup busy. */
#define LZO_MI355X_FAST_POOL_BYTES 8192
size_t lzo_mi355x_fast_ops_bytes_per_block(void);
uint32_t lzo_mi355x_fast_resident_blocks(void);
int lzo_mi355x_launch_decompress_fast(const uint8_t *src, const uint64_t *src_off,
                                      const uint32_t *src_len, uint8_t *dst,
                                      const uint64_t *dst_off, const uint32_t *dst_cap,
                                      uint32_t *out_len, int32_t *status, uint32_t *fallback,
                                      uint32_t *fallback_ids, uint32_t *pool, void *ring,
                                      void *ops, uint32_t nsets, uint32_t nblocks,
                                      uint32_t *order, hipStream_t stream);

/* Batches with more blocks than resident workgroups start them largest first
 * (order[i] = the i-th block to start; key: src_len to compress, dst_cap to
 * decompress, in 4 KiB classes): the last blocks to start are then the
 * smallest, and the batch does not wait on a large block started last (C4,
 * mixed 4-256 KiB: decompress 37.6 -> 35.2 ms, compress 119.6 -> 117.2 ms).
 * One workgroup, a counting sort, a few tens of microseconds. */
int lzo_mi355x_launch_order_by_size(const uint32_t *key, uint32_t n, uint32_t *order,
                                    hipStream_t stream);

/* Windowed throughput decoder (lzo1x_decode_win.hip): one workgroup of 512
 * threads per block, 64 KiB LDS output ring.  Blocks it does not finish
 * exactly go to fallback_ids[] as with the fast decoder (*fallback = 0 on
 * entry). */
int lzo_mi355x_launch_decompress_win(const uint8_t *src, const uint64_t *src_off,
                                     const uint32_t *src_len, uint8_t *dst,
                                     const uint64_t *dst_off, const uint32_t *dst_cap,
                                     uint32_t *out_len, int32_t *status, uint32_t *fallback,
                                     uint32_t *fallback_ids, uint32_t nblocks, hipStream_t stream);

/* Latency decoder (lzo1x_decode_lat.hip): ONE block of z compressed bytes
 * into out (capacity cap) by a pipeline of grid-wide kernels; out_len[b] /
 * status[b] and the fallback list as above.  scratch: at least
 * lzo_mi355x_decompress_lat_scratch(z, cap) bytes of device memory (0: the
 * block is outside the decoder's range -- z or cap 0, 2z + 3 or cap over
 * 16 Mi).  Returns -1 (nothing launched) outside that range or with too little
 * scratch. */
size_t lzo_mi355x_decompress_lat_scratch(uint32_t z, uint32_t cap);
int lzo_mi355x_launch_decompress_lat(const uint8_t *in, uint32_t z, uint8_t *out, uint32_t cap,
                                     uint32_t *out_len, int32_t *status, uint32_t *fallback,
                                     uint32_t *fallback_ids, uint32_t b, void *scratch,
                                     size_t scratch_bytes, hipStream_t stream);

/* Up to 8 blocks side by side in one latency-decoder pipeline (host arrays:
 * block b is z[b] bytes at src + src_off[b] into dst + dst_off[b], capacity
 * cap[b]; results at b0 + b; src_off[b] + z[b] < 2^31).  Scratch 0: outside
 * the range. */
size_t lzo_mi355x_decompress_lat_scratch_n(const uint64_t *src_off, const uint32_t *z, const uint32_t *cap,
                                           uint32_t nb);
int lzo_mi355x_launch_decompress_lat_n(const uint8_t *src, const uint64_t *src_off, const uint32_t *z,
                                       uint8_t *dst, const uint64_t *dst_off, const uint32_t *cap, uint32_t nb,
                                       uint32_t *out_len, int32_t *status, uint32_t *fallback,
                                       uint32_t *fallback_ids, uint32_t b0, void *scratch, size_t scratch_bytes,
                                       hipStream_t stream);

/* Unchecked-decoder pre-scan: decoded length and status per block; with
 * cap_out, also min(length, cap_limit) per block (a decode's capacity). */
int lzo_mi355x_launch_decoded_length(const uint8_t *src, const uint64_t *src_off,
                                     const uint32_t *src_len, uint32_t *out_len,
                                     int32_t *status, uint32_t nblocks, uint32_t *cap_out,
                                     uint32_t cap_limit, hipStream_t stream);

/* Host side (lzo_host.c), not part of the ABI: the debug switches of
 * POM_LZO_DEBUG ("key=value,..."; NULL / dflt when the key is absent). */
const char *pom_dbg_str(const char *key, char *buf, size_t n);
long pom_dbg_int(const char *key, long dflt);

/* Host side (lzo_host.c), not part of the ABI: lzo_mi355x_compress_batch
 * with on_chunk(ctx, ids, nb) called as each chunk's blocks are delivered
 * (ids: indices into the caller's arrays), from the thread running that
 * device's chunks -- concurrently when the batch is split over GPUs. */
typedef void (*pom_chunk_fn)(void *ctx, const size_t *ids, size_t nb);
int pom_compress_batch_chunked(const uint8_t *const *src, const size_t *src_len, uint8_t *const *dst,
                               size_t *dst_len, int *status, size_t nblocks, pom_chunk_fn on_chunk,
                               void *ctx);
/* lzo_mi355x_decompress_batch with pre_chunk(ctx, ids, nb) called before each
 * chunk's inputs are staged (the caller fills src[ids[i]] then). */
int pom_decompress_batch_chunked(const uint8_t *const *src, const size_t *src_len, uint8_t *const *dst,
                                 size_t *dst_len, int *status, size_t nblocks, pom_chunk_fn pre_chunk,
                                 void *ctx);

/* Host side (lzo_host.c), not part of the ABI: len[i] bytes from src[i] to
 * dst[i] for every i, split over up to 8 threads once the total is large. */
void pom_copy_parallel(uint8_t *const *dst, const uint8_t *const *src, const size_t *len, size_t n);

/* Block b's first min(len[b], cap[b]) bytes at from + from_off[b] go to
 * to + to_off[b] (offsets 16-byte aligned, regions padded to 16 bytes). */
int lzo_mi355x_launch_pack(const uint8_t *from, const uint64_t *from_off, const uint32_t *len,
                           const uint32_t *cap, const uint64_t *to_off, uint8_t *to,
                           uint32_t nblocks, hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif
