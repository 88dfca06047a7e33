/*
 * pom_column.h -- the client column-data codec of api/api.c on the MI355X
 * LZO1X batch path (liblzo_mi355x.so).
 *
 * Column data written with SCD_LZO is [size_t original length][LZO1X-1
 * stream] (LP64: an 8-byte length), sent raw when that is not smaller than
 * the data:
 *   pom_col_zip_batch   <- hvfs_fwrite SCD_LZO     api/api.c:6509-6541
 *   pom_col_zipv        <- hvfs_fwritev SCD_LZO    api/api.c:6652-6689
 *   pom_col_unzip_batch <- the read side           api/api.c:6427-6446
 *
 * Two reference defects are not reproduced:
 *   - the zip buffer is len + 8 bytes (api/api.c:6512), which LZO1X-1 output
 *     can overrun on incompressible data (up to len + len/16 + 67): here the
 *     output never exceeds the caller's capacity;
 *   - hvfs_fwritev compresses each iovec into its own stream and
 *     concatenates them, which the read side (one lzo1x_decompress call)
 *     cannot decode (INPUT_NOT_CONSUMED after the first stream).  Here
 *     pom_col_zipv writes the iovecs as one stream, which that same read side
 *     decodes, and pom_col_unzip_batch also reads the reference writer's
 *     layout (consecutive streams until the input is used up), so columns the
 *     reference already wrote stay readable.
 */
#ifndef POM_COLUMN_H
#define POM_COLUMN_H 1

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define POM_COL_HDR 8u              /* sizeof(size_t) on LP64 */

/* Capacity that always holds the zipped form of len bytes. */
size_t pom_col_zip_bound(size_t len);

/* n columns.  zip_len[b] = bytes written to zip[b]; compressed[b] = 1 for
 * [len][LZO1X], 0 when the column goes raw (nothing is written then, as the
 * reference falls back to the caller's buffer).  Returns 0, or an LZO_E_*
 * code when the GPU path is unusable. */
int pom_col_zip_batch(const uint8_t *const *data, const size_t *len, size_t n,
                      uint8_t *const *zip, const size_t *zip_cap, size_t *zip_len,
                      int *compressed);

/* The iovec form: the iovecs are one column of sum(iov_len) bytes. */
int pom_col_zipv(const uint8_t *const *iov_base, const size_t *iov_len, size_t iovcnt,
                 uint8_t *zip, size_t zip_cap, size_t *zip_len, int *compressed);

/* n zipped columns -> out[b] (capacity out_cap[b]).  err[b] = 0 when the
 * stream (or the reference fwritev layout's consecutive streams) decodes to
 * exactly its recorded length, else the decoder's LZO_E_* code, or
 * LZO_E_ERROR for a length mismatch or a column shorter than its header.
 * out_len[b] = bytes produced. */
int pom_col_unzip_batch(const uint8_t *const *zip, const size_t *zip_len, size_t n,
                        uint8_t *const *out, const size_t *out_cap, size_t *out_len, int *err);

#ifdef __cplusplus
}
#endif

#endif /* POM_COLUMN_H */
