/*
 * pom_itb.h -- ITB record codec and MDSL append-file loopback on the MI355X
 * LZO1X batch path (liblzo_mi355x.so).
 *
 * An ITB record is [struct itbh, 264 B][payload]: the payload starts at
 * &itb->lock and is h.len - 264 bytes (include/xtable.h:43-102; sizeof and
 * field offsets on LP64 with the reference's build flags, where
 * _USE_SPINLOCK is not defined, so ilock is a pthread mutex).  These entry
 * points batch what the reference does one ITB at a time:
 *
 *   pom_itb_lzo_compress_batch   <- itb_lzo_compress   mds/itb.c:2904-2945
 *                                   (called from txg_wb_itb, mds/txg.c:733-770)
 *   pom_itb_lzo_decompress_batch <- itb_lzo_decompress mds/itb.c:2949-2980
 *                                   and its twin       mdsl/gc.c:755-786
 *   pom_abuf_*                   <- append_buf_write / append_buf_flush_remap
 *                                   mdsl/storage.c:384-519 (ITB append file)
 *   pom_itb_read, pom_itb_read_batch
 *                                <- the header-then-payload ITB read of the
 *                                   MDSL read path (mdsl/storage.c:2507-2640)
 */
#ifndef POM_ITB_H
#define POM_ITB_H 1

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define POM_ITBH_SIZE 264u          /* sizeof(struct itbh) */
#define POM_ITBH_LEN_OFF 240u       /* atomic_t len: total record length */
#define POM_ITBH_ZLEN_OFF 244u      /* atomic_t zlen: uncompressed length when compressed */
#define POM_ITBH_ALGO_OFF 248u      /* u16 compress_algo */
#define POM_COMPR_NONE 0u
#define POM_COMPR_LZO 1u
/* Payload bounds of a real ITB: 3584 B locks + 128 B bitmap + 8192 B index +
 * 512 B per ITE, 1 ... 1024 ITEs (mds/itb.c:314, include/xtable.h:136-144). */
#define POM_ITB_PAYLOAD_MIN 12416u
#define POM_ITB_PAYLOAD_MAX 536192u

/* itb_lzo_compress for n ITBs.  For each b: the header of in[b] is copied to
 * tmp[b]; the payload (in[b] + 264, h.len - 264 bytes) is LZO1X-1 compressed
 * to tmp[b] + 264.  If the result is not smaller than the payload, oi[b] =
 * in[b] (kept uncompressed); otherwise tmp[b].zlen = tmp[b].len, tmp[b].len =
 * 264 + zlen, tmp[b].compress_algo = COMPR_LZO and oi[b] = tmp[b].  err[b] is
 * 0 or an LZO_E_* code (-EINVAL: h.len below the header size).
 * tmp_cap[b] is the size of tmp[b]; the output never exceeds it (the
 * reference writes past a full-size buffer on incompressible payloads).
 * Returns 0, or LZO_E_ERROR when the GPU path is unusable. */
int pom_itb_lzo_compress_batch(uint8_t *const *in, uint8_t *const *tmp, const size_t *tmp_cap,
                               uint8_t **oi, int *err, size_t n);

/* itb_lzo_decompress for n ITBs, in place: the payload of in[b] is decoded
 * into in[b] + 264 (cap[b] = size of the in[b] buffer bounds it, where the
 * reference's unchecked decoder has no bound).  err[b] = the decoder's LZO_E_*
 * code, as in the reference (an output length other than zlen - 264 is logged
 * there, not returned; it is reported here through len_ok[b] when non-NULL).
 * Always: compress_algo = COMPR_NONE, len = produced + 264. */
int pom_itb_lzo_decompress_batch(uint8_t *const *in, const size_t *cap, int *err,
                                 int *len_ok, size_t n);

/* MDSL append buffer: records are copied into an mmap'ed window of the file;
 * a full window is unmapped and the next one mapped (the file grows by
 * ftruncate in steps of 2 windows).  location = file offset of the record. */
struct pom_abuf {
    int fd;
    size_t win;             /* window length (page multiple) */
    uint8_t *addr;          /* current window */
    uint64_t file_offset;   /* file offset of the window */
    size_t offset;          /* bytes used in the window */
    uint64_t falloc_end;    /* file length reserved by ftruncate */
    uint64_t acclen;        /* bytes appended */
};
int pom_abuf_open(struct pom_abuf *ab, const char *path, size_t win);
int pom_abuf_append(struct pom_abuf *ab, const void *rec, size_t len, uint64_t *location);
/* n appends in one call: the same file bytes and locations as n calls of
 * pom_abuf_append in order (each window's share pre-faulted, copied by host
 * threads).  recs[b] may be NULL only when lens[b] == 0. */
int pom_abuf_append_batch(struct pom_abuf *ab, const void *const *recs, const size_t *lens,
                          size_t n, uint64_t *locations);
/* unmaps and trims the file to the appended length */
int pom_abuf_close(struct pom_abuf *ab);

/* The MDS write-back path on the loopback (mds/txg.c:733-770 compressing,
 * mdsl/storage.c:455-519 appending): pom_itb_lzo_compress_batch, and every
 * record oi[b] (h.len bytes) appended to ab as soon as the chunk of the
 * batch holding it is compressed, while the GPU compresses the next chunks.
 * locations[b] = the record's file offset (UINT64_MAX for a record with
 * err[b] == -EINVAL, which is not written).  Records are appended in the
 * order their chunks finish on the GPU, not in index order: two runs of the
 * same batch can lay the file out differently (readers go by locations[];
 * the debug key ooo=0 delivers chunks in launch order, largest blocks first).
 * Returns 0, LZO_E_ERROR when the GPU path is unusable, or the first append's
 * -errno; on any failure the append point is put back where it was on entry,
 * the bytes the batch's appends had written past it are zeroed, and every
 * locations[b] is UINT64_MAX, so the caller may retry the whole batch.  If the
 * append point's window cannot be mapped again, it returns POM_ABUF_E_BROKEN:
 * the abuf then refuses appends, and pom_abuf_close still cuts the file at
 * the append point of entry. */
#define POM_ABUF_E_BROKEN (-4096)
int pom_itb_lzo_compress_append_batch(uint8_t *const *in, uint8_t *const *tmp, const size_t *tmp_cap,
                                      uint8_t **oi, int *err, size_t n, struct pom_abuf *ab,
                                      uint64_t *locations);

/* Reads the ITB record at `location` of fd: the 264-byte header first, then
 * the rest of h.len.  *len = h.len.  -EINVAL: h.len < 264 or > cap. */
int pom_itb_read(int fd, uint64_t location, uint8_t *buf, size_t cap, size_t *len);

/* pom_itb_read of n records (an MDSL batch of ITB loads), split over up to 8
 * threads: record i from locations[i] into buf[i] (capacity cap[i]); len[i]
 * and err[i] (0 or the -errno pom_itb_read returns) per record.  Returns 0,
 * or -ENOMEM. */
int pom_itb_read_batch(int fd, const uint64_t *locations, size_t n, uint8_t *const *buf,
                       const size_t *cap, size_t *len, int *err);

/* The MDS load path on the loopback (mdsl/storage.c:2507-2640 reading,
 * mds/itb.c:2949-2980 decoding): pom_itb_read_batch, then, for every record
 * whose header says COMPR_LZO, pom_itb_lzo_decompress_batch in place -- with
 * each chunk's payloads read just before the decode batch stages that chunk,
 * while the GPU decodes the chunks before it.  err[i] = 0 or the read's
 * -errno (-EINVAL: h.len < 264 or > cap[i]); derr[i] = the decoder's LZO_E_*
 * code (0 for an uncompressed record); len_ok[i] (may be NULL) as in
 * pom_itb_lzo_decompress_batch (1 for an uncompressed record); len[i] = the
 * record's h.len after decoding (0 when err[i] != 0: the buffer past the
 * header is then undefined).  Returns 0, LZO_E_ERROR when the GPU path is
 * unusable, or LZO_E_OUT_OF_MEMORY. */
int pom_itb_read_lzo_decompress_batch(int fd, const uint64_t *locations, size_t n, uint8_t *const *buf,
                                      const size_t *cap, size_t *len, int *err, int *derr, int *len_ok);

#ifdef __cplusplus
}
#endif

#endif /* POM_ITB_H */
