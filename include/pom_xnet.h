/*
 * pom_xnet.h -- xnet wire framing of ITB messages on the MI355X LZO1X batch
 * path (liblzo_mi355x.so), SURVEY.md §8(f) row 4.
 *
 * ITBs travel between MDS and MDSL as xnet messages: a struct xnet_msg_tx
 * header (include/xnet.h:27-67, 72 bytes on LP64) followed by tx.len data
 * bytes, the ITB record itself (xnet-simple without XNET_EAGER_WRITEV:
 * xnet/xnet_simple.c:480-578).  These entry points batch what the reference
 * does one message at a time:
 *
 *   pom_xnet_itb_wb_batch    <- txg_wb_itb: itb_lzo_compress, then the
 *                               ITB write-back REQ (mds/txg.c:733-770, :548-584)
 *   pom_xnet_itb_reply_batch <- __mdsl_send_rpy_data(..., flag 1): the
 *                               XNET_RPY_DATA_ITB reply (mdsl/m2ml.c:87-120)
 *   pom_xnet_parse           <- the receive loop: header, then tx.len bytes;
 *                               magic check (xnet/xnet_simple.c:480-587)
 *   pom_xnet_itb_recv_batch  <- the MDS side of an ITB reply: the data lands
 *                               in a whole free ITB (test/xnet/mds.c:683-691),
 *                               tx.len must equal h.len, a COMPR_LZO record is
 *                               decompressed in place (mds/itb.c:140-168)
 *
 * Only ITB-only messages are framed: the write-back REQ that opens or closes
 * a TXG also carries BEGIN/END sections (mds/txg.c:560-583), which are not
 * part of the codec path.
 */
#ifndef POM_XNET_H
#define POM_XNET_H 1

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* struct xnet_msg_tx, byte for byte (LP64, little endian) */
struct pom_xnet_tx {
    uint8_t vm;             /* version:4 (low nibble), magic:4 (high nibble) */
    uint8_t type;
    uint16_t flag;
    int32_t err;
    uint64_t ssite_id;
    uint64_t dsite_id;
    uint64_t cmd;
    uint64_t arg0;
    uint64_t arg1;
    uint32_t reqno;
    uint32_t len;           /* data bytes after the header */
    uint64_t handle;
    uint64_t reserved;
};
#define POM_XNET_TX_SIZE 72u
#define POM_XNET_MAGIC(tx) ((uint8_t)((tx).vm >> 4))

/* include/xnet.h, include/hvfs.h */
#define POM_XNET_MSG_REQ 1u
#define POM_XNET_MSG_RPY 2u
#define POM_XNET_NEED_DATA_FREE 0x0004u
#define POM_XNET_RPY_DATA 0x03u
#define POM_XNET_RPY_DATA_ITB 0x04u
#define POM_HVFS_MDS2MDSL_WBTXG 0x0000000080030000ull
#define POM_HVFS_WBTXG_ITB 0x0002ull

/* One parsed frame: its header and data (pointing into the wire buffer). */
struct pom_xnet_frame {
    struct pom_xnet_tx tx;
    const uint8_t *data;
    int dropped;            /* magic mismatch: the reference frees the message */
};

/* Header + data into wire (cap bytes); hdr->len is replaced by len.
 * Returns the bytes written, 0 if they do not fit. */
size_t pom_xnet_frame(uint8_t *wire, size_t cap, const struct pom_xnet_tx *hdr,
                      const void *data, uint32_t len);

/* Frames of a byte stream, at most max.  A frame whose header or data is not
 * complete ends the parse: *consumed is where the next read resumes.
 * magic (4 bits; 0 accepts all): a frame with a nonzero magic other than it is
 * marked dropped.  Returns 0. */
int pom_xnet_parse(const uint8_t *wire, size_t len, uint8_t magic, struct pom_xnet_frame *f,
                   size_t max, size_t *nframes, size_t *consumed);

/* The requester of an ITB load (its REQ header fields the reply echoes). */
struct pom_xnet_req {
    uint64_t ssite_id;
    uint32_t reqno;
    uint64_t handle;
};

/* MDSL: n XNET_RPY_DATA_ITB replies, one per stored ITB record (sent as
 * stored, h.len bytes), appended to wire.  *wire_len = bytes written.
 * Returns 0, or -ENOSPC (nothing partial is counted: *wire_len covers the
 * whole replies written before the one that did not fit). */
int pom_xnet_itb_reply_batch(const uint8_t *const *itb, const struct pom_xnet_req *req, size_t n,
                             uint64_t site_id, uint8_t magic, uint8_t *wire, size_t cap,
                             size_t *wire_len);

/* The destination of one ITB write-back. */
struct pom_xnet_wb {
    uint64_t dsite_id;      /* the MDSL site of the ITB (ring point) */
    uint64_t vid;           /* tx.reserved */
};

/* MDS: itb_lzo_compress of n ITBs (pom_itb_lzo_compress_batch, GPU), then one
 * write-back REQ per ITB carrying the compressed record, or the original one
 * when compression did not pay, appended to wire.  err[b] as
 * pom_itb_lzo_compress_batch (the original record is sent on error, as
 * txg_wb_itb does).  Returns 0, -ENOSPC, or LZO_E_ERROR (GPU unusable). */
int pom_xnet_itb_wb_batch(uint8_t *const *itb, uint8_t *const *tmp, const size_t *tmp_cap,
                          const struct pom_xnet_wb *wb, size_t n, uint64_t site_id, uint64_t txg,
                          uint8_t magic, uint8_t *wire, size_t cap, size_t *wire_len, int *err);

/* MDS: n received ITB replies.  Frame b's ITB lands in itb[b] (a whole ITB
 * buffer of itb_cap bytes): an uncompressed record is copied; a COMPR_LZO
 * record's header is copied and its payload decoded straight from the wire
 * into itb[b] after the header (GPU), the header then left as
 * itb_lzo_decompress leaves it (algo NONE, len = header + decoded bytes;
 * mds/itb.c:2949-2980).  err[b]:
 *   0        the ITB in itb[b] is ready;
 *   -EBADMSG the frame was dropped (magic);
 *   -EIO     data longer than itb_cap, or tx.len != h.len;
 *   -EFAULT  the decoder failed.
 * Returns 0, or LZO_E_ERROR when the GPU path is unusable. */
int pom_xnet_itb_recv_batch(const struct pom_xnet_frame *f, size_t n, uint8_t *const *itb,
                            size_t itb_cap, int *err);

#ifdef __cplusplus
}
#endif

#endif /* POM_XNET_H */
