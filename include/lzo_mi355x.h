/*
 * lzo_mi355x.h -- batch C-ABI of the MI355X LZO1X codec (liblzo_mi355x.so).
 *
 * The reference has no batch interface: every caller invokes the single-block
 * functions of lib/minilzo.h synchronously.  These entry
 * points let the same callers hand over many ITB-sized blocks at once:
 *   - mds/txg.c:700-770   (txg_wb_itb: one lzo1x_1_compress per dirty ITB)
 *   - mds/itb.c:2949-2980, mdsl/gc.c:755-786 (itb_lzo_decompress per ITB)
 *   - api/api.c:6509-6541, :6427-6446 (client column data)
 * Output of every block is identical to the single-block functions in
 * minilzo.h (and so to lib/minilzo.c with a zero-filled wrkmem).
 *
 * Plain C types only: pointers, sizes, and the HIP stream as void*.
 */
#ifndef POM_LZO_MI355X_H
#define POM_LZO_MI355X_H 1

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Worst-case LZO1X-1 output for n input bytes: n + n/16 + 64 + 3. */
size_t lzo_mi355x_worst_compress(size_t n);

/* Number of usable GPUs (0 when none: every codec call then fails). */
int lzo_mi355x_device_count(void);

/* Re-read the POM_LZO_DEBUG environment variable (debug and experiment keys,
 * INTEGRATION.md section 6).  The library reads it once, at the first use;
 * a caller that changes it between calls (the tests) calls this after. */
void lzo_mi355x_debug_reload(void);

/* ---- device-resident batches ------------------------------------------------
 * All pointers are device (HBM) pointers; the call only enqueues work on
 * `stream` (a hipStream_t, NULL = default stream) and returns 0 or -1 on a
 * launch failure.  Block b reads src + src_off[b] .. + src_len[b] and writes
 * at most dst_cap[b] bytes at dst + dst_off[b]; out_len[b] and status[b]
 * (LZO_E_* code) are written when the stream reaches the work.
 */
/* `scratch`: device memory of lzo_mi355x_compress_scratch(nblocks) bytes for
 * the per-workgroup match dictionaries (32 KiB each; 16 blocks per CU are then
 * parsed at once) after a 256-byte head (the block ticket of batches larger
 * than the grid, reset by the call on `stream`), then, for batches of more
 * blocks than resident workgroups, 4 bytes a block for the start order
 * (largest blocks first, sorted by the call on `stream`); or NULL
 * (dictionaries in LDS: 4 blocks per CU).  No initial contents are required. */
int lzo_mi355x_compress_dev(const uint8_t *src, const uint64_t *src_off,
                            const uint32_t *src_len, uint8_t *dst,
                            const uint64_t *dst_off, const uint32_t *dst_cap,
                            uint32_t *out_len, int32_t *status, uint32_t nblocks,
                            void *scratch, void *stream);
size_t lzo_mi355x_compress_scratch(uint32_t nblocks);

/* Decompression with lzo1x_decompress_safe semantics per block (capacity
 * dst_cap[b]).  `scratch` is device memory of lzo_mi355x_decompress_scratch()
 * bytes for nblocks, or NULL (every block then takes the exact one-wave
 * decoder).  The scratch holds a 4-byte-a-block list plus op slots for the
 * workgroups resident at once (not per block): about 100 MB plus 4 bytes a
 * block (8 for batches of more blocks than resident workgroups: their start
 * order, largest first, sorted by the call on `stream`).  After the call, the u32 at scratch byte 0 counts the blocks the
 * throughput decoder handed to the exact (one wave per block, ~20x slower)
 * decoder: malformed streams, capacity or look-behind errors, destinations not
 * 16-byte aligned (the windowed decoder, which small batches take, needs only
 * 8), empty or >= 16 MiB inputs.  Every valid stream with a 16-byte aligned
 * destination stays on the throughput decoders. */
int lzo_mi355x_decompress_dev(const uint8_t *src, const uint64_t *src_off,
                              const uint32_t *src_len, uint8_t *dst,
                              const uint64_t *dst_off, const uint32_t *dst_cap,
                              uint32_t *out_len, int32_t *status, uint32_t nblocks,
                              void *scratch, void *stream);
size_t lzo_mi355x_decompress_scratch(uint32_t nblocks);
/* The number of blocks the last lzo_mi355x_decompress_dev() on `scratch` handed
 * to the exact decoder: waits for `stream`, then reads scratch byte 0 into
 * *count.  Returns 0, or -1 on a copy failure. */
int lzo_mi355x_decompress_fallbacks(const void *scratch, uint32_t *count, void *stream);

/* Decoded length of each block (the unchecked decoder's view), no output. */
int lzo_mi355x_decoded_length_dev(const uint8_t *src, const uint64_t *src_off,
                                  const uint32_t *src_len, uint32_t *out_len,
                                  int32_t *status, uint32_t nblocks, void *stream);

/* Decoded length of one host-resident LZO1X stream (GPU pre-scan): the size
 * the destination of lzo1x_decompress() must have.  Returns the status the
 * decoder would return with unlimited capacity; *dst_len = bytes it produces. */
int lzo_mi355x_decoded_length(const uint8_t *src, unsigned long src_len,
                              unsigned long *dst_len);

/* ---- host-resident batches --------------------------------------------------
 * Blocks start and end in host memory (the mdsl/aio.c write path and the
 * xnet wire).  The blocks are ordered largest first and dealt round robin
 * over the GPUs (POM_LZO_DEVICES, default all; a batch below 64 MiB a GPU
 * stays on the caller's current GPU).  Each GPU's share is cut into chunks of
 * at most 128 MiB of input plus output capacity (debug key chunk_mb of POM_LZO_DEBUG; the first
 * chunk a quarter of that), each packed into pinned staging, copied to the
 * GPU with hipMemcpyAsync, coded and copied back, up to four chunks in flight
 * on four streams, so staging stays bounded whatever the batch size.
 * Synchronous; thread-safe (each host thread owns its streams and staging on
 * each GPU).  Returns 0, or LZO_E_ERROR when a GPU is unusable (its blocks
 * then read LZO_E_ERROR); per-block results are in status[].
 */
int lzo_mi355x_compress_batch(const uint8_t *const *src, const size_t *src_len,
                              uint8_t *const *dst, size_t *dst_len, int *status,
                              size_t nblocks);
/* dst_len[b] is the capacity in and the produced length out.  A block's
 * input is staged before its output is written, so dst[b] may overlap src[b]
 * (in-place decoding); it must not overlap another block's input. */
int lzo_mi355x_decompress_batch(const uint8_t *const *src, const size_t *src_len,
                                uint8_t *const *dst, size_t *dst_len, int *status,
                                size_t nblocks);
/* As lzo_mi355x_decompress_batch, for blocks made of consecutive LZO1X
 * streams: the hvfs_fwritev column layout (api/api.c:6666-6680, one
 * lzo1x_1_compress stream per iovec, back to back).  Each stream decodes as
 * its own lzo1x_decompress_safe call would, right after the previous one's
 * output; dst_len[b] is the total and status[b] the last stream's code (0
 * when the last stream ends exactly at the end of the block). */
int lzo_mi355x_decompress_concat_batch(const uint8_t *const *src, const size_t *src_len,
                                       uint8_t *const *dst, size_t *dst_len, int *status,
                                       size_t nblocks);

#ifdef __cplusplus
}
#endif

#endif /* POM_LZO_MI355X_H */
