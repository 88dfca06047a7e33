/*
 * column_codec.c -- the client column-data codec (include/pom_column.h) over
 * the host-resident LZO1X batch API.  Format and fallback follow
 * api/api.c:6509-6541, :6652-6689 and :6427-6446.
 */
#include <stdlib.h>
#include <string.h>

#include "lzo_mi355x.h"
#include "minilzo.h"
#include "pom_column.h"

size_t pom_col_zip_bound(size_t len)
{
    return POM_COL_HDR + lzo_mi355x_worst_compress(len);
}

int pom_col_zip_batch(const uint8_t *const *data, const size_t *len, size_t n,
                      uint8_t *const *zip, const size_t *zip_cap, size_t *zip_len,
                      int *compressed)
{
    if (n == 0)
        return LZO_E_OK;
    uint8_t **dst = malloc(n * sizeof(*dst));
    uint8_t **aside = calloc(n, sizeof(*aside));
    size_t *zl = malloc(n * sizeof(*zl));
    int *st = malloc(n * sizeof(*st));
    int rc = LZO_E_OUT_OF_MEMORY;
    if (!dst || !aside || !zl || !st)
        goto out;
    for (size_t b = 0; b < n; b++) {
        zip_len[b] = 0;
        compressed[b] = 0;
        if (zip_cap[b] >= pom_col_zip_bound(len[b])) {
            dst[b] = zip[b] + POM_COL_HDR;
        } else {                                   /* never overrun the caller's buffer */
            aside[b] = malloc(lzo_mi355x_worst_compress(len[b]));
            if (!aside[b])
                goto out;
            dst[b] = aside[b];
        }
    }
    rc = lzo_mi355x_compress_batch(data, len, dst, zl, st, n);
    if (rc != LZO_E_OK)
        goto out;
    for (size_t b = 0; b < n; b++) {
        /* raw when compression failed or did not pay (api/api.c:6525-6538) */
        if (st[b] != LZO_E_OK || zl[b] + POM_COL_HDR >= len[b] ||
            zl[b] + POM_COL_HDR > zip_cap[b])
            continue;
        const uint64_t l64 = len[b];
        memcpy(zip[b], &l64, POM_COL_HDR);
        if (aside[b])
            memcpy(zip[b] + POM_COL_HDR, aside[b], zl[b]);
        zip_len[b] = zl[b] + POM_COL_HDR;
        compressed[b] = 1;
    }
out:
    if (aside)
        for (size_t b = 0; b < n; b++)
            free(aside[b]);
    free(aside);
    free(dst);
    free(zl);
    free(st);
    return rc;
}

int pom_col_zipv(const uint8_t *const *iov_base, const size_t *iov_len, size_t iovcnt,
                 uint8_t *zip, size_t zip_cap, size_t *zip_len, int *compressed)
{
    size_t total = 0;
    for (size_t i = 0; i < iovcnt; i++)
        total += iov_len[i];
    *zip_len = 0;
    *compressed = 0;
    if (total == 0)
        return LZO_E_OK;
    uint8_t *flat = malloc(total);
    if (!flat)
        return LZO_E_OUT_OF_MEMORY;
    size_t o = 0;
    for (size_t i = 0; i < iovcnt; i++) {
        memcpy(flat + o, iov_base[i], iov_len[i]);
        o += iov_len[i];
    }
    const uint8_t *d[1] = { flat };
    uint8_t *z[1] = { zip };
    const int rc = pom_col_zip_batch(d, &total, 1, z, &zip_cap, zip_len, compressed);
    free(flat);
    return rc;
}

/* Columns are first decoded as one stream each (what pom_col_zip_batch and
 * pom_col_zipv write, and what the reference reader expects,
 * api/api.c:6438-6446).  A column whose first stream ends short of the input
 * (INPUT_NOT_CONSUMED) is the reference writer's
 * hvfs_fwritev layout (api/api.c:6666-6680, one stream per iovec): it is
 * decoded again as consecutive streams until the input is used up. */
int pom_col_unzip_batch(const uint8_t *const *zip, const size_t *zip_len, size_t n,
                        uint8_t *const *out, const size_t *out_cap, size_t *out_len, int *err)
{
    if (n == 0)
        return LZO_E_OK;
    const uint8_t **src = malloc(n * sizeof(*src));
    size_t *slen = malloc(n * sizeof(*slen));
    size_t *dlen = malloc(n * sizeof(*dlen));
    uint64_t *want = malloc(n * sizeof(*want));
    int *st = malloc(n * sizeof(*st));
    size_t *multi = malloc(n * sizeof(*multi));
    const uint8_t **msrc = malloc(n * sizeof(*msrc));
    size_t *mslen = malloc(n * sizeof(*mslen));
    uint8_t **mdst = malloc(n * sizeof(*mdst));
    size_t *mdlen = malloc(n * sizeof(*mdlen));
    int *mst = malloc(n * sizeof(*mst));
    int rc = LZO_E_OUT_OF_MEMORY;
    if (!src || !slen || !dlen || !want || !st || !multi || !msrc || !mslen || !mdst || !mdlen ||
        !mst)
        goto out;
    for (size_t b = 0; b < n; b++) {
        want[b] = 0;
        if (zip_len[b] >= POM_COL_HDR)
            memcpy(&want[b], zip[b], POM_COL_HDR);
        src[b] = zip[b] + (zip_len[b] >= POM_COL_HDR ? POM_COL_HDR : 0);
        slen[b] = zip_len[b] >= POM_COL_HDR ? zip_len[b] - POM_COL_HDR : 0;
        dlen[b] = out_cap[b];
    }
    rc = lzo_mi355x_decompress_batch(src, slen, out, dlen, st, n);
    if (rc != LZO_E_OK)
        goto out;
    size_t nm = 0;
    for (size_t b = 0; b < n; b++)
        if (zip_len[b] >= POM_COL_HDR && st[b] == LZO_E_INPUT_NOT_CONSUMED) {
            multi[nm] = b;
            msrc[nm] = src[b];
            mslen[nm] = slen[b];
            mdst[nm] = out[b];
            mdlen[nm] = out_cap[b];
            nm++;
        }
    if (nm) {
        rc = lzo_mi355x_decompress_concat_batch(msrc, mslen, mdst, mdlen, mst, nm);
        if (rc != LZO_E_OK)
            goto out;
        for (size_t k = 0; k < nm; k++) {
            dlen[multi[k]] = mdlen[k];
            st[multi[k]] = mst[k];
        }
    }
    for (size_t b = 0; b < n; b++) {
        out_len[b] = dlen[b] < out_cap[b] ? dlen[b] : out_cap[b];
        if (zip_len[b] < POM_COL_HDR)
            err[b] = LZO_E_ERROR;
        else if (st[b] != LZO_E_OK)
            err[b] = st[b];
        else
            err[b] = dlen[b] == want[b] ? LZO_E_OK : LZO_E_ERROR;   /* olen == olen_cmp */
    }
out:
    free(src);
    free(slen);
    free(dlen);
    free(want);
    free(st);
    free(multi);
    free(msrc);
    free(mslen);
    free(mdst);
    free(mdlen);
    free(mst);
    return rc;
}
