/*
 * itb_callsite.c -- compiles the reference's call patterns, unchanged in shape,
 * against include/minilzo.h and links them to liblzo_mi355x.so.
 *
 *   lzo_init()                                  mds/mds.c:1197-1202
 *   itb_lzo_compress: header copy, compress the payload after the 264-B
 *     header, keep it raw when it does not shrink   mds/itb.c:2904-2945
 *   itb_lzo_decompress: copy payload aside, unchecked decode in place,
 *     success iff LZO_E_OK and outlen == zlen - 264  mds/itb.c:2949-2980
 *   client column data [size_t len][LZO1X]          api/api.c:6509-6541, 6427-6446
 *
 * The record layout below is this test's own stand-in for struct itb (only
 * the fields the wrappers touch).  Exit codes: 0 = round trips OK,
 * 2 = lzo_init() refused (no usable GPU), 1 = mismatch.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "minilzo.h"

#define HDR 264
#define COMPR_NONE 0
#define COMPR_LZO 1

struct rec_hdr {            /* stand-in for struct itbh's len/zlen/compress_algo */
    uint32_t len;           /* whole record length (header + payload) */
    uint32_t zlen;          /* length before compression */
    uint8_t compress_algo;
    uint8_t pad[HDR - 9];
};

struct rec {
    struct rec_hdr h;
    uint8_t payload[];
};

static int rec_compress(struct rec *in, struct rec *tmp, struct rec **oi, void *workmem)
{
    lzo_uint zlen = 0, inlen;
    int err;
    memcpy(&tmp->h, &in->h, HDR);
    inlen = in->h.len - HDR;
    err = lzo1x_1_compress((void *)in->payload, inlen, (void *)tmp->payload, &zlen, workmem);
    if (err != LZO_E_OK)
        return -1;
    if (zlen >= inlen) {
        *oi = in;                   /* keep the uncompressed record */
        return 0;
    }
    tmp->h.zlen = in->h.len;
    tmp->h.len = HDR + (uint32_t)zlen;
    tmp->h.compress_algo = COMPR_LZO;
    *oi = tmp;
    return 0;
}

static int rec_decompress(struct rec *in)
{
    lzo_uint outlen, inlen;         /* outlen deliberately uninitialised */
    void *p;
    int err;
    inlen = in->h.len - HDR;
    p = malloc(inlen ? inlen : 1);
    if (!p)
        return -1;
    memcpy(p, in->payload, inlen);
    err = lzo1x_decompress(p, inlen, (void *)in->payload, &outlen, NULL);
    free(p);
    if (err != LZO_E_OK || outlen != in->h.zlen - HDR)
        return -1;
    in->h.compress_algo = COMPR_NONE;
    in->h.len = (uint32_t)outlen + HDR;
    return 0;
}

int main(void)
{
    if (lzo_init() != LZO_E_OK) {
        fprintf(stderr, "lzo_init failed (no usable GPU)\n");
        return 2;
    }
    if (lzo_version() != 0x2040 || strcmp(lzo_version_string(), "2.04") != 0)
        return 1;
    const size_t maxp = 536192;     /* largest ITB payload */
    void *workmem = malloc(LZO1X_1_MEM_COMPRESS + (sizeof(lzo_align_t) - 1));
    struct rec *a = calloc(1, sizeof(struct rec) + maxp);
    struct rec *b = calloc(1, sizeof(struct rec) + maxp + maxp / 16 + 64 + 3);
    uint8_t *orig = malloc(maxp);
    if (!workmem || !a || !b || !orig)
        return 1;
    uint64_t s = 88172645463325252ull;
    size_t sizes[] = { 12416, 65536, 11904 + 512 * 40, maxp };
    for (int k = 0; k < 4; k++) {
        size_t n = sizes[k];
        memset(a->payload, 0, n);
        for (size_t i = 3712; i + 16 < n; i += 512) {   /* sparse records */
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            memcpy(a->payload + i, &s, 8);
            memcpy(a->payload + i + 104, "file-name.jpg", 13);
        }
        memcpy(orig, a->payload, n);
        a->h.len = (uint32_t)(HDR + n);
        struct rec *o = NULL;
        if (rec_compress(a, b, &o, workmem) != 0 || o != b) {
            fprintf(stderr, "compress failed at %zu\n", n);
            return 1;
        }
        memset(a->payload, 0xEE, n);
        memcpy(a, b, b->h.len);     /* the record as stored, then loaded */
        if (rec_decompress(a) != 0 || a->h.len != HDR + n || memcmp(a->payload, orig, n)) {
            fprintf(stderr, "decompress mismatch at %zu\n", n);
            return 1;
        }
        printf("record %zu B -> %u B ok\n", n, b->h.len - HDR);
    }
    /* client column data: [size_t orig_len][LZO1X] with raw fallback */
    const char *msg = "column column column column column data data data data";
    size_t len = strlen(msg);
    uint8_t *zip = malloc(len + len / 16 + 64 + 3 + sizeof(size_t));
    lzo_uint zlen = 0;
    *(size_t *)zip = len;
    if (lzo1x_1_compress((void *)msg, len, zip + sizeof(size_t), &zlen, workmem) != LZO_E_OK)
        return 1;
    uint8_t back[256];
    lzo_uint olen = sizeof(back);
    if (lzo1x_decompress_safe(zip + sizeof(size_t), zlen, back, &olen, NULL) != LZO_E_OK ||
        olen != *(size_t *)zip || memcmp(back, msg, len))
        return 1;
    printf("column data ok\n");
    return 0;
}
