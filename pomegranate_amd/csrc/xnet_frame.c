/*
 * xnet_frame.c -- xnet wire framing of ITB messages over the ITB codec
 * (include/pom_xnet.h).
 *
 *   frame / parse  struct xnet_msg_tx + tx.len data bytes, the magic check
 *                  (include/xnet.h:27-67, xnet/xnet_simple.c:480-587, :1912)
 *   reply          __mdsl_send_rpy_data with flag 1 (mdsl/m2ml.c:87-120)
 *   write-back     txg_wb_itb: compress, then the REQ (mds/txg.c:548-584, :733-770)
 *   receive        the MDS load path (mds/itb.c:140-168, test/xnet/mds.c:683-691)
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "lzo_mi355x.h"
#include "lzo_mi355x_kernels.h"
#include "minilzo.h"
#include "pom_itb.h"
#include "pom_xnet.h"

_Static_assert(sizeof(struct pom_xnet_tx) == POM_XNET_TX_SIZE, "struct xnet_msg_tx is 72 bytes");

static uint32_t rd32(const uint8_t *p)
{
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}

static uint16_t rd16(const uint8_t *p)
{
    uint16_t v;
    memcpy(&v, p, 2);
    return v;
}

size_t pom_xnet_frame(uint8_t *wire, size_t cap, const struct pom_xnet_tx *hdr,
                      const void *data, uint32_t len)
{
    const size_t need = POM_XNET_TX_SIZE + (size_t)len;
    if (cap < need)
        return 0;
    struct pom_xnet_tx tx = *hdr;
    tx.len = len;
    memcpy(wire, &tx, POM_XNET_TX_SIZE);
    if (len)
        memcpy(wire + POM_XNET_TX_SIZE, data, len);
    return need;
}

int pom_xnet_parse(const uint8_t *wire, size_t len, uint8_t magic, struct pom_xnet_frame *f,
                   size_t max, size_t *nframes, size_t *consumed)
{
    size_t off = 0, nf = 0;
    magic &= 15u;                                   /* a 4-bit field on the wire */
    while (nf < max && len - off >= POM_XNET_TX_SIZE) {
        struct pom_xnet_tx tx;
        memcpy(&tx, wire + off, POM_XNET_TX_SIZE);
        if (len - off - POM_XNET_TX_SIZE < tx.len)
            break;                                  /* data not all here yet */
        f[nf].tx = tx;
        f[nf].data = wire + off + POM_XNET_TX_SIZE;
        /* our magic 0 accepts all, and so does a message without one */
        f[nf].dropped = magic && POM_XNET_MAGIC(tx) && POM_XNET_MAGIC(tx) != magic;
        off += POM_XNET_TX_SIZE + tx.len;
        nf++;
    }
    *nframes = nf;
    *consumed = off;
    return 0;
}

static struct pom_xnet_tx header(uint8_t type, uint16_t flag, uint64_t ssite, uint64_t dsite,
                                 uint8_t magic)
{
    struct pom_xnet_tx tx;
    memset(&tx, 0, sizeof(tx));                     /* xnet_alloc_msg zero-fills */
    tx.vm = (uint8_t)((magic & 15u) << 4);          /* version stays 0 */
    tx.type = type;                                 /* xnet_msg_fill_tx */
    tx.flag = flag;
    tx.ssite_id = ssite;
    tx.dsite_id = dsite;
    return tx;
}

/* Headers of n messages with data[b] (len[b] bytes) laid out back to back in
 * `wire`: headers written here, the data copied by pom_copy_parallel (threads
 * once the batch is large).  *wire_len = the bytes of the messages that fit;
 * -ENOSPC when not all of them did, LZO_E_OUT_OF_MEMORY without scratch. */
static int frame_batch(const struct pom_xnet_tx *tx, const uint8_t *const *data, const uint32_t *len,
                       size_t n, uint8_t *wire, size_t cap, size_t *wire_len)
{
    uint8_t **dp = malloc(n * sizeof(*dp));
    size_t *ln = malloc(n * sizeof(*ln));
    if (!dp || !ln) {
        free(dp);
        free(ln);
        return LZO_E_OUT_OF_MEMORY;
    }
    size_t off = 0, k = 0;
    int rc = 0;
    for (; k < n; k++) {
        const size_t need = POM_XNET_TX_SIZE + (size_t)len[k];
        if (cap - off < need) {
            rc = -ENOSPC;
            break;
        }
        struct pom_xnet_tx t = tx[k];
        t.len = len[k];
        memcpy(wire + off, &t, POM_XNET_TX_SIZE);
        dp[k] = wire + off + POM_XNET_TX_SIZE;
        ln[k] = len[k];
        off += need;
    }
    pom_copy_parallel(dp, data, ln, k);
    *wire_len = off;
    free(dp);
    free(ln);
    return rc;
}

int pom_xnet_itb_reply_batch(const uint8_t *const *itb, const struct pom_xnet_req *req, size_t n,
                             uint64_t site_id, uint8_t magic, uint8_t *wire, size_t cap,
                             size_t *wire_len)
{
    *wire_len = 0;
    if (n == 0)
        return 0;
    struct pom_xnet_tx *tx = malloc(n * sizeof(*tx));
    uint32_t *len = malloc(n * sizeof(*len));
    int rc = LZO_E_OUT_OF_MEMORY;
    if (tx && len) {
        for (size_t b = 0; b < n; b++) {
            tx[b] = header(POM_XNET_MSG_RPY, POM_XNET_NEED_DATA_FREE, site_id, req[b].ssite_id, magic);
            tx[b].reqno = req[b].reqno;             /* xnet_msg_fill_reqno */
            tx[b].cmd = POM_XNET_RPY_DATA_ITB;      /* xnet_msg_fill_cmd(rpy, ..., 0, 0) */
            tx[b].handle = req[b].handle;           /* match the request at its source */
            len[b] = rd32(itb[b] + POM_ITBH_LEN_OFF);
        }
        rc = frame_batch(tx, itb, len, n, wire, cap, wire_len);
    }
    free(tx);
    free(len);
    return rc;
}

int pom_xnet_itb_wb_batch(uint8_t *const *itb, uint8_t *const *tmp, const size_t *tmp_cap,
                          const struct pom_xnet_wb *wb, size_t n, uint64_t site_id, uint64_t txg,
                          uint8_t magic, uint8_t *wire, size_t cap, size_t *wire_len, int *err)
{
    *wire_len = 0;
    if (n == 0)
        return 0;
    uint8_t **oi = malloc(n * sizeof(*oi));
    struct pom_xnet_tx *tx = malloc(n * sizeof(*tx));
    uint32_t *len = malloc(n * sizeof(*len));
    const uint8_t **rec = malloc(n * sizeof(*rec));
    int rc = LZO_E_OUT_OF_MEMORY;
    if (oi && tx && len && rec) {
        rc = pom_itb_lzo_compress_batch(itb, tmp, tmp_cap, oi, err, n);
        if (rc == LZO_E_OK) {
            for (size_t b = 0; b < n; b++) {
                rec[b] = err[b] ? itb[b] : oi[b];
                tx[b] = header(POM_XNET_MSG_REQ, 0, site_id, wb[b].dsite_id, magic);
                tx[b].cmd = POM_HVFS_MDS2MDSL_WBTXG;    /* xnet_msg_fill_cmd(msg, WBTXG, ITB, txg) */
                tx[b].arg0 = POM_HVFS_WBTXG_ITB;
                tx[b].arg1 = txg;
                tx[b].reserved = wb[b].vid;
                len[b] = rd32(rec[b] + POM_ITBH_LEN_OFF);
            }
            rc = frame_batch(tx, rec, len, n, wire, cap, wire_len);
        }
    }
    free(oi);
    free(tx);
    free(len);
    free(rec);
    return rc;
}

/* The MDS load path for a batch of received messages: each message's ITB is
 * checked (the load path's length ASSERT), an uncompressed one copied into its
 * buffer, and a COMPR_LZO one decoded straight from the wire into its buffer
 * after the header -- the compressed payload is never copied on the host --
 * with the header then rewritten as itb_lzo_decompress leaves it
 * (mds/itb.c:2949-2980: algo NONE, len = header + decoded bytes). */
int pom_xnet_itb_recv_batch(const struct pom_xnet_frame *f, size_t n, uint8_t *const *itb,
                            size_t itb_cap, int *err)
{
    if (n == 0)
        return 0;
    const uint8_t **src = malloc(n * sizeof(*src));
    size_t *slen = malloc(n * sizeof(*slen));
    uint8_t **dst = malloc(n * sizeof(*dst));
    size_t *dlen = malloc(n * sizeof(*dlen));
    int *st = malloc(n * sizeof(*st));
    size_t *at = malloc(n * sizeof(*at));
    uint8_t **cdst = malloc(n * sizeof(*cdst));
    const uint8_t **csrc = malloc(n * sizeof(*csrc));
    size_t *clen = malloc(n * sizeof(*clen));
    int rc = LZO_E_OUT_OF_MEMORY;
    if (!src || !slen || !dst || !dlen || !st || !at || !cdst || !csrc || !clen)
        goto out;
    size_t nd = 0, nc = 0;
    for (size_t b = 0; b < n; b++) {
        const uint32_t len = f[b].tx.len;
        err[b] = f[b].dropped ? -EBADMSG : len < POM_ITBH_SIZE || len > itb_cap ? -EIO : 0;
        if (err[b])
            continue;
        const uint8_t *w = f[b].data;
        if (rd32(w + POM_ITBH_LEN_OFF) != len) {      /* the load path's ASSERT */
            err[b] = -EIO;
            continue;
        }
        if (rd16(w + POM_ITBH_ALGO_OFF) == POM_COMPR_LZO) {
            memcpy(itb[b], w, POM_ITBH_SIZE);
            src[nd] = w + POM_ITBH_SIZE;
            slen[nd] = len - POM_ITBH_SIZE;
            dst[nd] = itb[b] + POM_ITBH_SIZE;
            dlen[nd] = itb_cap - POM_ITBH_SIZE;
            at[nd] = b;
            nd++;
        } else {
            cdst[nc] = itb[b];
            csrc[nc] = w;
            clen[nc] = len;
            nc++;
        }
    }
    pom_copy_parallel(cdst, csrc, clen, nc);
    rc = nd ? lzo_mi355x_decompress_batch(src, slen, dst, dlen, st, nd) : LZO_E_OK;
    if (rc != LZO_E_OK)
        goto out;
    for (size_t i = 0; i < nd; i++) {
        uint8_t *h = itb[at[i]];
        const uint16_t none = POM_COMPR_NONE;
        const uint32_t nl = (uint32_t)(dlen[i] + POM_ITBH_SIZE);
        memcpy(h + POM_ITBH_ALGO_OFF, &none, 2);      /* clear the compress flag */
        memcpy(h + POM_ITBH_LEN_OFF, &nl, 4);
        if (st[i] != LZO_E_OK)
            err[at[i]] = -EFAULT;                     /* itb_lzo_decompress failed */
    }
out:
    free(src);
    free(slen);
    free(dst);
    free(dlen);
    free(st);
    free(at);
    free(cdst);
    free(csrc);
    free(clen);
    return rc;
}
