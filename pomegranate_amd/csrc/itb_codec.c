/*
 * itb_codec.c -- ITB record codec and MDSL append-file loopback over the
 * host-resident LZO1X batch API (include/pom_itb.h).
 *
 * The per-record semantics follow the reference one for one:
 *   compress   mds/itb.c:2904-2945  (header copy, incompressible fallback,
 *                                    len/zlen swap, COMPR_LZO)
 *   decompress mds/itb.c:2949-2980, mdsl/gc.c:755-786 (decoded in place,
 *                                    COMPR_NONE, len back)
 *   append     mdsl/storage.c:455-519 (append_buf_write), :384-451
 *              (append_buf_flush_remap)
 * The LZO work of a whole batch is one GPU round trip (lzo_host.c).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <fcntl.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/uio.h>
#include <unistd.h>

#include "io_util.h"
#include "lzo_mi355x.h"
#include "minilzo.h"
#include "pom_itb.h"
#include "lzo_mi355x_kernels.h"

static uint32_t rd32(const uint8_t *p)
{
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}

static void wr32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }
static void wr16(uint8_t *p, uint16_t v) { memcpy(p, &v, 2); }

int pom_itb_lzo_compress_batch(uint8_t *const *in, uint8_t *const *tmp, const size_t *tmp_cap,
                               uint8_t **oi, int *err, size_t n)
{
    if (n == 0)
        return LZO_E_OK;
    const uint8_t **src = malloc(n * sizeof(*src));
    uint8_t **dst = malloc(n * sizeof(*dst));
    uint8_t **aside = calloc(n, sizeof(*aside));   /* when tmp cannot take the worst case */
    size_t *slen = malloc(n * sizeof(*slen));
    size_t *dlen = malloc(n * sizeof(*dlen));
    int *st = malloc(n * sizeof(*st));
    int rc = LZO_E_OUT_OF_MEMORY;
    if (!src || !dst || !aside || !slen || !dlen || !st)
        goto out;
    for (size_t b = 0; b < n; b++) {
        oi[b] = in[b];
        const uint32_t len = rd32(in[b] + POM_ITBH_LEN_OFF);
        slen[b] = len >= POM_ITBH_SIZE ? len - POM_ITBH_SIZE : 0;
        src[b] = in[b] + POM_ITBH_SIZE;
        dst[b] = tmp[b] + POM_ITBH_SIZE;
        const size_t worst = lzo_mi355x_worst_compress(slen[b]);
        if (tmp_cap[b] < POM_ITBH_SIZE + worst) {
            aside[b] = malloc(worst);
            if (!aside[b])
                goto out;
            dst[b] = aside[b];
        }
        err[b] = len >= POM_ITBH_SIZE ? 0 : -EINVAL;
    }
    rc = lzo_mi355x_compress_batch(src, slen, dst, dlen, st, n);
    if (rc != LZO_E_OK)
        goto out;
    for (size_t b = 0; b < n; b++) {
        if (err[b])
            continue;
        memcpy(tmp[b], in[b], POM_ITBH_SIZE);                  /* the itb header */
        if (st[b] != LZO_E_OK) {
            err[b] = st[b];
            continue;
        }
        if (dlen[b] >= slen[b])                                /* impossible to compress */
            continue;
        if (aside[b])
            memcpy(tmp[b] + POM_ITBH_SIZE, aside[b], dlen[b]);
        wr32(tmp[b] + POM_ITBH_ZLEN_OFF, rd32(tmp[b] + POM_ITBH_LEN_OFF));
        wr32(tmp[b] + POM_ITBH_LEN_OFF, (uint32_t)(POM_ITBH_SIZE + dlen[b]));
        wr16(tmp[b] + POM_ITBH_ALGO_OFF, POM_COMPR_LZO);
        oi[b] = tmp[b];
    }
out:
    if (aside)
        for (size_t b = 0; b < n; b++)
            free(aside[b]);
    free(aside);
    free(src);
    free(dst);
    free(slen);
    free(dlen);
    free(st);
    return rc;
}

int pom_itb_lzo_decompress_batch(uint8_t *const *in, const size_t *cap, int *err,
                                 int *len_ok, size_t n)
{
    if (n == 0)
        return LZO_E_OK;
    const uint8_t **src = malloc(n * sizeof(*src));
    uint8_t **dst = malloc(n * sizeof(*dst));
    size_t *slen = malloc(n * sizeof(*slen));
    size_t *dlen = malloc(n * sizeof(*dlen));
    int *st = malloc(n * sizeof(*st));
    int rc = LZO_E_OUT_OF_MEMORY;
    if (!src || !dst || !slen || !dlen || !st)
        goto out;
    for (size_t b = 0; b < n; b++) {
        const uint32_t len = rd32(in[b] + POM_ITBH_LEN_OFF);
        slen[b] = len >= POM_ITBH_SIZE ? len - POM_ITBH_SIZE : 0;
    }
    /* in place: the batch call stages a block's payload before it writes that
     * block's output (include/lzo_mi355x.h), so no copy aside is needed */
    for (size_t b = 0; b < n; b++) {
        src[b] = in[b] + POM_ITBH_SIZE;
        dst[b] = in[b] + POM_ITBH_SIZE;
        dlen[b] = cap[b] > POM_ITBH_SIZE ? cap[b] - POM_ITBH_SIZE : 0;
    }
    rc = lzo_mi355x_decompress_batch(src, slen, dst, dlen, st, n);
    if (rc != LZO_E_OK)
        goto out;
    for (size_t b = 0; b < n; b++) {
        const uint32_t zlen = rd32(in[b] + POM_ITBH_ZLEN_OFF);
        err[b] = st[b];
        if (len_ok)
            len_ok[b] = st[b] == LZO_E_OK && dlen[b] + POM_ITBH_SIZE == zlen;
        wr16(in[b] + POM_ITBH_ALGO_OFF, POM_COMPR_NONE);       /* clear the compress flag */
        wr32(in[b] + POM_ITBH_LEN_OFF, (uint32_t)(dlen[b] + POM_ITBH_SIZE));
    }
out:
    free(src);
    free(dst);
    free(slen);
    free(dlen);
    free(st);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* MDSL append buffer                                                       */
/* ------------------------------------------------------------------------ */
static int abuf_map(struct pom_abuf *ab)
{
    if (ab->file_offset + ab->win > ab->falloc_end) {
        /* reserve two windows ahead (mdsl/storage.c:419-430) */
        const uint64_t end = ab->file_offset + 2 * (uint64_t)ab->win;
        if (ftruncate(ab->fd, (off_t)end) != 0)
            return -errno;
        ab->falloc_end = end;
    }
    void *a = mmap(NULL, ab->win, PROT_READ | PROT_WRITE, MAP_SHARED, ab->fd,
                   (off_t)ab->file_offset);
    if (a == MAP_FAILED)
        return -errno;
    ab->addr = a;
    ab->offset = 0;
    return 0;
}

int pom_abuf_open(struct pom_abuf *ab, const char *path, size_t win)
{
    const size_t page = (size_t)sysconf(_SC_PAGESIZE);
    memset(ab, 0, sizeof(*ab));
    ab->fd = -1;
    if (win == 0)
        win = 64u << 20;
    ab->win = (win + page - 1) / page * page;
    ab->fd = open(path, O_RDWR | O_CREAT | O_TRUNC, 0644);
    if (ab->fd < 0)
        return -errno;
    const int rc = abuf_map(ab);
    if (rc) {
        close(ab->fd);
        ab->fd = -1;
    }
    return rc;
}

int pom_abuf_append(struct pom_abuf *ab, const void *rec, size_t len, uint64_t *location)
{
    if (!ab->addr || !rec)
        return -EINVAL;
    const uint8_t *p = rec;
    size_t done = 0;
    if (location)
        *location = ab->file_offset + ab->offset;
    while (done < len) {
        size_t w = ab->win - ab->offset;
        if (w > len - done)
            w = len - done;
        memcpy(ab->addr + ab->offset, p + done, w);
        done += w;
        ab->offset += w;
        if (ab->offset >= ab->win) {
            /* flush + remap the next window (mdsl/storage.c:384-451) */
            if (munmap(ab->addr, ab->win) != 0)
                return -errno;
            ab->addr = NULL;
            ab->file_offset += ab->win;
            const int rc = abuf_map(ab);
            if (rc)
                return rc;
        }
    }
    ab->acclen += len;
    return 0;
}

/* A batch of appends with the locations of n single appends in order.  Each
 * window's share goes to the file in one gathered write (pwritev); a full
 * window is unmapped and the next mapped as in pom_abuf_append, so single and
 * batched appends interleave freely.  (Pre-faulting the window with
 * MADV_POPULATE_WRITE and copying on 8 threads took twice as long.) */
enum { kIovMax = 1024 };
int pom_abuf_append_batch(struct pom_abuf *ab, const void *const *recs, const size_t *lens,
                          size_t n, uint64_t *locations)
{
    if (!ab->addr)
        return -EINVAL;
    uint8_t **dst = malloc((n + 1) * sizeof(*dst));
    const uint8_t **src = malloc((n + 1) * sizeof(*src));
    size_t *len = malloc((n + 1) * sizeof(*len));
    if (!dst || !src || !len) {
        free(dst);
        free(src);
        free(len);
        return -ENOMEM;
    }
    int rc = 0;
    size_t b = 0, done = 0;         /* record b, bytes of it already placed */
    while (b < n && !rc) {
        /* jobs of the current window: from ab->offset up to its end */
        size_t nj = 0, start = ab->offset, off = ab->offset;
        while (b < n && off < ab->win) {
            if (!recs[b] && lens[b]) {
                rc = -EINVAL;
                break;
            }
            if (done == 0 && locations)
                locations[b] = ab->file_offset + off;
            size_t w = ab->win - off;
            if (w > lens[b] - done)
                w = lens[b] - done;
            if (w) {
                dst[nj] = ab->addr + off;
                src[nj] = (const uint8_t *)recs[b] + done;
                len[nj] = w;
                nj++;
            }
            off += w;
            done += w;
            if (done == lens[b]) {
                ab->acclen += lens[b];
                b++;
                done = 0;
            }
        }
        if (rc)
            break;
        if (off > start) {
            /* one gathered write of the window's share into the page cache the
             * window maps (coherent on Linux): about twice as fast as faulting
             * the window's pages in and copying (C5 write), same file */
            struct iovec iov[kIovMax];
            uint64_t fo = ab->file_offset + start;
            for (size_t j0 = 0; j0 < nj && !rc; j0 += kIovMax) {
                const size_t m = nj - j0 < kIovMax ? nj - j0 : kIovMax;
                size_t want = 0;
                for (size_t j = 0; j < m; j++) {
                    iov[j].iov_base = (void *)src[j0 + j];
                    iov[j].iov_len = len[j0 + j];
                    want += len[j0 + j];
                }
                rc = pom_pwritev_all(ab->fd, iov, (int)m, (off_t)fo, NULL);
                fo += want;
            }
            if (rc)
                break;
        }
        ab->offset = off;
        if (ab->offset >= ab->win) {
            if (munmap(ab->addr, ab->win) != 0) {
                rc = -errno;
                break;
            }
            ab->addr = NULL;
            ab->file_offset += ab->win;
            rc = abuf_map(ab);
        }
    }
    free(dst);
    free(src);
    free(len);
    return rc;
}

int pom_abuf_close(struct pom_abuf *ab)
{
    int rc = 0;
    if (ab->addr && munmap(ab->addr, ab->win) != 0)
        rc = -errno;
    ab->addr = NULL;
    if (ab->fd >= 0) {
        if (ftruncate(ab->fd, (off_t)(ab->file_offset + ab->offset)) != 0 && !rc)
            rc = -errno;
        if (close(ab->fd) != 0 && !rc)
            rc = -errno;
    }
    ab->fd = -1;
    return rc;
}

static int pread_full(int fd, uint8_t *buf, size_t len, uint64_t off)
{
    size_t done = 0;
    while (done < len) {
        const ssize_t r = pread(fd, buf + done, len - done, (off_t)(off + done));
        if (r < 0) {
            if (errno == EINTR)
                continue;
            return -errno;
        }
        if (r == 0)
            return -EIO;
        done += (size_t)r;
    }
    return 0;
}

int pom_itb_read(int fd, uint64_t location, uint8_t *buf, size_t cap, size_t *len)
{
    if (cap < POM_ITBH_SIZE)
        return -EINVAL;
    int rc = pread_full(fd, buf, POM_ITBH_SIZE, location);            /* the header first */
    if (rc)
        return rc;
    const uint32_t l = rd32(buf + POM_ITBH_LEN_OFF);
    if (l < POM_ITBH_SIZE || l > cap)
        return -EINVAL;
    rc = pread_full(fd, buf + POM_ITBH_SIZE, l - POM_ITBH_SIZE, location + POM_ITBH_SIZE);
    if (rc)
        return rc;
    *len = l;
    return 0;
}

struct read_range {
    int fd;
    const uint64_t *loc;
    uint8_t *const *buf;
    const size_t *cap;
    size_t *len;
    int *err;
    size_t lo, hi;
};

static void *read_worker(void *arg)
{
    const struct read_range *r = arg;
    for (size_t i = r->lo; i < r->hi; i++) {
        r->len[i] = 0;
        r->err[i] = pom_itb_read(r->fd, r->loc[i], r->buf[i], r->cap[i], &r->len[i]);
    }
    return NULL;
}

int pom_itb_read_batch(int fd, const uint64_t *locations, size_t n, uint8_t *const *buf,
                       const size_t *cap, size_t *len, int *err)
{
    enum { kReadThreads = 8 };
    const size_t nt = n >= 64 ? kReadThreads : 1;
    struct read_range r[kReadThreads];
    pthread_t th[kReadThreads];
    int started[kReadThreads] = {0};
    for (size_t k = 0; k < nt; k++) {
        r[k] = (struct read_range){fd, locations, buf, cap, len, err, n * k / nt, n * (k + 1) / nt};
        if (k > 0)
            started[k] = pthread_create(&th[k], NULL, read_worker, &r[k]) == 0;
    }
    read_worker(&r[0]);
    for (size_t k = 1; k < nt; k++) {
        if (started[k])
            pthread_join(th[k], NULL);
        else
            read_worker(&r[k]);
    }
    return 0;
}
