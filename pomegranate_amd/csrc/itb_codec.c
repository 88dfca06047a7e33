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

/* One itb_lzo_compress batch: the arrays of pom_itb_lzo_compress_batch, the
 * LZO batch's own, and (compress + append) the append file. */
struct itb_wb {
    uint8_t *const *in;
    uint8_t *const *tmp;
    uint8_t **oi;
    int *err;
    const uint8_t **src;
    uint8_t **dst;
    uint8_t **aside;        /* when tmp cannot take the worst case */
    size_t *slen, *dlen;
    int *st;
    struct pom_abuf *ab;    /* NULL: compress only */
    uint64_t *locations;
    int arc;                /* first append error */
    pthread_mutex_t mu;     /* (chunks of a multi-GPU batch finish on several threads) */
    /* append worker (compress + append): delivered chunks queue here and one
     * thread finishes and appends them in delivery order, so the batch's
     * pipeline thread goes on staging and delivering the next chunks */
    struct wb_job *head, *tail;
    pthread_mutex_t qmu;
    pthread_cond_t qcv;
    int closing, worker;
    pthread_t th;
};

struct wb_job {
    struct wb_job *next;
    size_t nb;
    size_t ids[];
};

static void itb_wb_free(struct itb_wb *w, size_t n)
{
    if (w->aside)
        for (size_t b = 0; b < n; b++)
            free(w->aside[b]);
    free(w->aside);
    free(w->src);
    free(w->dst);
    free(w->slen);
    free(w->dlen);
    free(w->st);
}

/* mds/itb.c:2904-2921: the payload after the header, into tmp after its header */
static int itb_wb_init(struct itb_wb *w, uint8_t *const *in, uint8_t *const *tmp, const size_t *tmp_cap,
                       uint8_t **oi, int *err, size_t n)
{
    memset(w, 0, sizeof(*w));
    w->in = in;
    w->tmp = tmp;
    w->oi = oi;
    w->err = err;
    w->src = malloc(n * sizeof(*w->src));
    w->dst = malloc(n * sizeof(*w->dst));
    w->aside = calloc(n, sizeof(*w->aside));
    w->slen = malloc(n * sizeof(*w->slen));
    w->dlen = malloc(n * sizeof(*w->dlen));
    w->st = malloc(n * sizeof(*w->st));
    if (!w->src || !w->dst || !w->aside || !w->slen || !w->dlen || !w->st)
        return LZO_E_OUT_OF_MEMORY;
    for (size_t b = 0; b < n; b++) {
        oi[b] = in[b];
        const uint32_t len = rd32(in[b] + POM_ITBH_LEN_OFF);
        w->slen[b] = len >= POM_ITBH_SIZE ? len - POM_ITBH_SIZE : 0;
        w->src[b] = in[b] + POM_ITBH_SIZE;
        w->dst[b] = tmp[b] + POM_ITBH_SIZE;
        const size_t worst = lzo_mi355x_worst_compress(w->slen[b]);
        if (tmp_cap[b] < POM_ITBH_SIZE + worst) {
            w->aside[b] = malloc(worst);
            if (!w->aside[b])
                return LZO_E_OUT_OF_MEMORY;
            w->dst[b] = w->aside[b];
        }
        err[b] = len >= POM_ITBH_SIZE ? 0 : -EINVAL;
    }
    return LZO_E_OK;
}

/* mds/itb.c:2923-2944 for block b once its compressed bytes are in */
static void itb_wb_finish(struct itb_wb *w, size_t b)
{
    if (w->err[b])
        return;
    uint8_t *t = w->tmp[b];
    memcpy(t, w->in[b], POM_ITBH_SIZE);                        /* the itb header */
    if (w->st[b] != LZO_E_OK) {
        w->err[b] = w->st[b];
        return;
    }
    if (w->dlen[b] >= w->slen[b])                              /* impossible to compress */
        return;
    if (w->aside[b])
        memcpy(t + POM_ITBH_SIZE, w->aside[b], w->dlen[b]);
    wr32(t + POM_ITBH_ZLEN_OFF, rd32(t + POM_ITBH_LEN_OFF));
    wr32(t + POM_ITBH_LEN_OFF, (uint32_t)(POM_ITBH_SIZE + w->dlen[b]));
    wr16(t + POM_ITBH_ALGO_OFF, POM_COMPR_LZO);
    w->oi[b] = t;
}

/* A chunk of the batch is compressed: finish its records and append them to
 * the file while the GPU works on the next chunks. */
static void itb_wb_chunk_run(struct itb_wb *w, const size_t *ids, size_t nb)
{
    const void **recs = malloc(nb * sizeof(*recs));
    size_t *lens = malloc(nb * sizeof(*lens));
    uint64_t *locs = malloc(nb * sizeof(*locs));
    size_t m = 0;
    for (size_t i = 0; i < nb; i++) {
        const size_t b = ids[i];
        itb_wb_finish(w, b);
        if (w->ab)
            w->locations[b] = UINT64_MAX;
        if (!w->ab || w->err[b] == -EINVAL || !recs || !lens || !locs)
            continue;
        recs[m] = w->oi[b];
        lens[m] = rd32(w->oi[b] + POM_ITBH_LEN_OFF);
        locs[m] = b;                                           /* (the record's index, for now) */
        m++;
    }
    if (w->ab) {
        pthread_mutex_lock(&w->mu);
        int rc = !recs || !lens || !locs ? -ENOMEM : 0;
        uint64_t *at = rc ? NULL : malloc((m + 1) * sizeof(*at));
        if (!rc && !at)
            rc = -ENOMEM;
        if (!rc && !w->arc)
            rc = pom_abuf_append_batch(w->ab, recs, lens, m, at);
        if (!rc)
            for (size_t i = 0; i < m; i++)
                w->locations[locs[i]] = at[i];
        if (rc && !w->arc)
            w->arc = rc;
        pthread_mutex_unlock(&w->mu);
        free(at);
    }
    free(recs);
    free(lens);
    free(locs);
}

static void *itb_wb_worker(void *arg)
{
    struct itb_wb *w = arg;
    pthread_mutex_lock(&w->qmu);
    for (;;) {
        while (!w->head && !w->closing)
            pthread_cond_wait(&w->qcv, &w->qmu);
        struct wb_job *j = w->head;
        if (!j)
            break;                                   /* closing, queue drained */
        w->head = j->next;
        if (!w->head)
            w->tail = NULL;
        pthread_mutex_unlock(&w->qmu);
        itb_wb_chunk_run(w, j->ids, j->nb);
        free(j);
        pthread_mutex_lock(&w->qmu);
    }
    pthread_mutex_unlock(&w->qmu);
    return NULL;
}

/* on_chunk of the compress + append batch: the chunk goes to the append
 * worker (or is run here when there is none or no memory for the job) */
static void itb_wb_chunk(void *ctx, const size_t *ids, size_t nb)
{
    struct itb_wb *w = ctx;
    struct wb_job *j = w->worker ? malloc(sizeof(*j) + nb * sizeof(size_t)) : NULL;
    if (!j) {
        itb_wb_chunk_run(w, ids, nb);
        return;
    }
    j->next = NULL;
    j->nb = nb;
    memcpy(j->ids, ids, nb * sizeof(size_t));
    pthread_mutex_lock(&w->qmu);
    if (w->tail)
        w->tail->next = j;
    else
        w->head = j;
    w->tail = j;
    pthread_cond_signal(&w->qcv);
    pthread_mutex_unlock(&w->qmu);
}

int pom_itb_lzo_compress_batch(uint8_t *const *in, uint8_t *const *tmp, const size_t *tmp_cap,
                               uint8_t **oi, int *err, size_t n)
{
    if (n == 0)
        return LZO_E_OK;
    struct itb_wb w;
    int rc = itb_wb_init(&w, in, tmp, tmp_cap, oi, err, n);
    if (rc == LZO_E_OK)
        rc = lzo_mi355x_compress_batch(w.src, w.slen, w.dst, w.dlen, w.st, n);
    if (rc == LZO_E_OK)
        for (size_t b = 0; b < n; b++)
            itb_wb_finish(&w, b);
    itb_wb_free(&w, n);
    return rc;
}

static int abuf_map(struct pom_abuf *ab);

/* Puts the append point back to (file_offset, offset) and zeroes what the
 * rolled-back appends wrote past it, so neither a reader nor a crash before
 * close finds a record of the failed batch.  The bookkeeping is restored
 * first: even when the window cannot be mapped again, pom_abuf_close
 * truncates at the restored point.  A failed munmap or remap leaves addr
 * NULL (the abuf refuses appends) and returns -errno. */
static int abuf_rollback(struct pom_abuf *ab, uint64_t file_offset, size_t offset, uint64_t acclen)
{
    const uint64_t reached = ab->file_offset + ab->offset, at = file_offset + offset;
    int rc = 0;
    const int remap = ab->file_offset != file_offset || !ab->addr;
    if (remap) {
        if (ab->addr && munmap(ab->addr, ab->win) != 0)
            rc = -errno;
        ab->addr = NULL;
    }
    ab->file_offset = file_offset;
    ab->offset = offset;
    ab->acclen = acclen;
    if (reached > at &&
        fallocate(ab->fd, FALLOC_FL_PUNCH_HOLE | FALLOC_FL_KEEP_SIZE, (off_t)at, (off_t)(reached - at)) != 0) {
        static const uint8_t zeros[1 << 16];
        for (uint64_t o = at; o < reached && !rc;) {
            const size_t w = reached - o < sizeof zeros ? (size_t)(reached - o) : sizeof zeros;
            const ssize_t k = pwrite(ab->fd, zeros, w, (off_t)o);
            if (k <= 0)
                rc = k < 0 ? -errno : -EIO;
            else
                o += (uint64_t)k;
        }
    }
    if (remap && !rc) {
        rc = pom_dbg_int("fail_remap", 0) ? -ENOMEM : abuf_map(ab);   /* (debug key: tests) */
        ab->offset = offset;                       /* abuf_map starts a window at 0 */
        if (rc && ab->addr) {
            munmap(ab->addr, ab->win);
            ab->addr = NULL;
        }
    }
    return rc;
}

/* Page-cache pages for a batch's appends, allocated ahead by a helper thread
 * (fallocate, the file size unchanged) while the GPU compresses, so that the
 * appends copy into pages that exist instead of allocating each one: a sixth
 * of the payload plus the headers (ITB records compress to a seventh, C5), at
 * most 128 MiB; what the appends do not use is cut off at close.  Debug key
 * abuf_prealloc=0 turns it off, append_worker=0 runs the appends on the
 * batch's pipeline thread (C5 write, 8 alternating runs of each: 14.4 against
 * 14.0 GiB/s median with both on / off, 6 of 8 pairs faster;
 * profiles/r05h_c5/). */
struct prealloc {
    int fd, stop;
    uint64_t from, to;
};

static void *prealloc_run(void *arg)
{
    struct prealloc *p = arg;
    const uint64_t step = (uint64_t)2 << 20;
    for (uint64_t at = p->from; at < p->to && !__atomic_load_n(&p->stop, __ATOMIC_RELAXED); at += step) {
        const uint64_t len = p->to - at < step ? p->to - at : step;
        if (fallocate(p->fd, FALLOC_FL_KEEP_SIZE, (off_t)at, (off_t)len) != 0)
            break;
    }
    return NULL;
}

int pom_itb_lzo_compress_append_batch(uint8_t *const *in, uint8_t *const *tmp, const size_t *tmp_cap,
                                      uint8_t **oi, int *err, size_t n, struct pom_abuf *ab,
                                      uint64_t *locations)
{
    if (n == 0)
        return LZO_E_OK;
    if (!ab || !ab->addr || !locations)
        return -EINVAL;
    for (size_t b = 0; b < n; b++)
        locations[b] = UINT64_MAX;
    const uint64_t fo0 = ab->file_offset, acc0 = ab->acclen;
    const size_t off0 = ab->offset;
    struct itb_wb w;
    int rc = itb_wb_init(&w, in, tmp, tmp_cap, oi, err, n);
    w.ab = ab;
    w.locations = locations;
    pthread_mutex_init(&w.mu, NULL);
    pthread_mutex_init(&w.qmu, NULL);
    pthread_cond_init(&w.qcv, NULL);
    w.worker = rc == LZO_E_OK && pom_dbg_int("append_worker", 1) != 0 &&
               pthread_create(&w.th, NULL, itb_wb_worker, &w) == 0;
    struct prealloc pa = {ab->fd, 0, (ab->file_offset + ab->offset) & ~(uint64_t)4095, 0};
    uint64_t want = 0;
    for (size_t b = 0; rc == LZO_E_OK && b < n; b++)
        want += w.slen[b] / 6 + POM_ITBH_SIZE;
    pa.to = pa.from + (want < ((uint64_t)128 << 20) ? want : ((uint64_t)128 << 20));
    pthread_t pth;
    const int pre = rc == LZO_E_OK && pom_dbg_int("abuf_prealloc", 1) != 0 &&
                    pthread_create(&pth, NULL, prealloc_run, &pa) == 0;
    if (rc == LZO_E_OK)
        rc = pom_compress_batch_chunked(w.src, w.slen, w.dst, w.dlen, w.st, n, itb_wb_chunk, &w);
    if (pre) {
        __atomic_store_n(&pa.stop, 1, __ATOMIC_RELAXED);
        pthread_join(pth, NULL);
    }
    if (w.worker) {                                  /* the queued chunks' appends finish */
        pthread_mutex_lock(&w.qmu);
        w.closing = 1;
        pthread_cond_signal(&w.qcv);
        pthread_mutex_unlock(&w.qmu);
        pthread_join(w.th, NULL);
    }
    pthread_cond_destroy(&w.qcv);
    pthread_mutex_destroy(&w.qmu);
    if (rc == LZO_E_OK && w.arc)
        rc = w.arc;
    if (rc != LZO_E_OK) {
        /* all or nothing: the chunks delivered before the failure were
         * appended already; the append point goes back to where it was, so a
         * retry of the batch writes every record once */
        const int rb = abuf_rollback(ab, fo0, off0, acc0);
        for (size_t b = 0; b < n; b++)
            locations[b] = UINT64_MAX;
        if (rb)
            rc = POM_ABUF_E_BROKEN;                /* the caller must know the abuf is unusable */
    }
    pthread_mutex_destroy(&w.mu);
    itb_wb_free(&w, n);
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


/* ---- the MDS load path on the loopback: read, then decode as chunks fill ---- */
struct rd_payload {
    int fd;
    const uint64_t *loc;
    uint8_t *const *buf;
    const size_t *plen;     /* payload bytes to read per record */
    int *err;
    const size_t *ids;      /* records of this job */
    size_t lo, hi;
};

static void *payload_worker(void *arg)
{
    const struct rd_payload *r = arg;
    for (size_t i = r->lo; i < r->hi; i++) {
        const size_t b = r->ids ? r->ids[i] : i;
        if (r->err[b] || r->plen[b] == 0)
            continue;
        r->err[b] = pread_full(r->fd, r->buf[b] + POM_ITBH_SIZE, r->plen[b], r->loc[b] + POM_ITBH_SIZE);
    }
    return NULL;
}

struct rd_header {
    int fd;
    const uint64_t *loc;
    uint8_t *const *buf;
    int *err;
    size_t lo, hi;
};

static void *header_worker(void *arg)
{
    const struct rd_header *r = arg;
    for (size_t b = r->lo; b < r->hi; b++)
        if (!r->err[b])
            r->err[b] = pread_full(r->fd, r->buf[b], POM_ITBH_SIZE, r->loc[b]);
    return NULL;
}

static void read_headers(int fd, const uint64_t *loc, uint8_t *const *buf, int *err, size_t n)
{
    enum { kReadThreads = 8 };
    const size_t nt = n >= 256 ? kReadThreads : 1;
    struct rd_header r[kReadThreads];
    pthread_t th[kReadThreads];
    int started[kReadThreads] = {0};
    for (size_t k = 0; k < nt; k++) {
        r[k] = (struct rd_header){fd, loc, buf, err, n * k / nt, n * (k + 1) / nt};
        if (k > 0)
            started[k] = pthread_create(&th[k], NULL, header_worker, &r[k]) == 0;
    }
    header_worker(&r[0]);
    for (size_t k = 1; k < nt; k++) {
        if (started[k])
            pthread_join(th[k], NULL);
        else
            header_worker(&r[k]);
    }
}

/* payloads of records ids[0..n) (ids NULL: 0..n), on up to 8 threads */
static void read_payloads(int fd, const uint64_t *loc, uint8_t *const *buf, const size_t *plen, int *err,
                          const size_t *ids, size_t n)
{
    enum { kReadThreads = 8 };
    size_t bytes = 0;
    for (size_t i = 0; i < n; i++)
        bytes += plen[ids ? ids[i] : i];
    const size_t nt = n >= 8 && bytes >= ((size_t)1 << 20) ? kReadThreads : 1;
    struct rd_payload r[kReadThreads];
    pthread_t th[kReadThreads];
    int started[kReadThreads] = {0};
    for (size_t k = 0; k < nt; k++) {
        r[k] = (struct rd_payload){fd, loc, buf, plen, err, ids, n * k / nt, n * (k + 1) / nt};
        if (k > 0)
            started[k] = pthread_create(&th[k], NULL, payload_worker, &r[k]) == 0;
    }
    payload_worker(&r[0]);
    for (size_t k = 1; k < nt; k++) {
        if (started[k])
            pthread_join(th[k], NULL);
        else
            payload_worker(&r[k]);
    }
}

struct rd_dec {
    int fd;
    const uint64_t *loc;    /* per record */
    uint8_t *const *buf;    /* per record */
    const size_t *plen;     /* per record */
    int *err;               /* per record */
    const size_t *comp;     /* batch block -> record */
    pthread_mutex_t mu;     /* (chunks of a multi-GPU batch on several threads) */
};

/* a chunk of the decode batch is about to be staged: read its payloads */
static void rd_dec_chunk(void *ctx, const size_t *ids, size_t nb)
{
    struct rd_dec *d = ctx;
    size_t *rec = malloc(nb * sizeof(*rec));
    if (!rec) {
        pthread_mutex_lock(&d->mu);
        for (size_t i = 0; i < nb; i++)
            d->err[d->comp[ids[i]]] = -ENOMEM;
        pthread_mutex_unlock(&d->mu);
        return;
    }
    for (size_t i = 0; i < nb; i++)
        rec[i] = d->comp[ids[i]];
    read_payloads(d->fd, d->loc, d->buf, d->plen, d->err, rec, nb);
    free(rec);
}

int pom_itb_read_lzo_decompress_batch(int fd, const uint64_t *locations, size_t n, uint8_t *const *buf,
                                      const size_t *cap, size_t *len, int *err, int *derr, int *len_ok)
{
    if (n == 0)
        return LZO_E_OK;
    size_t *plen = calloc(n, sizeof(*plen));
    size_t *comp = malloc(n * sizeof(*comp));
    size_t *unc = malloc(n * sizeof(*unc));
    const uint8_t **src = malloc(n * sizeof(*src));
    uint8_t **dst = malloc(n * sizeof(*dst));
    size_t *slen = malloc(n * sizeof(*slen));
    size_t *dlen = malloc(n * sizeof(*dlen));
    int *st = malloc(n * sizeof(*st));
    int rc = LZO_E_OUT_OF_MEMORY;
    if (!plen || !comp || !unc || !src || !dst || !slen || !dlen || !st)
        goto out;
    /* 1. the headers (mdsl/storage.c:2507-2640 reads the itbh first), on up
     * to 8 threads */
    for (size_t b = 0; b < n; b++)
        err[b] = cap[b] < POM_ITBH_SIZE ? -EINVAL : 0;
    read_headers(fd, locations, buf, err, n);
    size_t nc = 0;
    for (size_t b = 0; b < n; b++) {
        derr[b] = 0;
        if (len_ok)
            len_ok[b] = 0;
        len[b] = 0;
        if (err[b])
            continue;
        const uint32_t hl = rd32(buf[b] + POM_ITBH_LEN_OFF);
        if (hl < POM_ITBH_SIZE || hl > cap[b]) {
            err[b] = -EINVAL;
            continue;
        }
        len[b] = hl;
        plen[b] = hl - POM_ITBH_SIZE;
        uint16_t algo;
        memcpy(&algo, buf[b] + POM_ITBH_ALGO_OFF, 2);
        if (algo == POM_COMPR_LZO) {
            comp[nc] = b;
            src[nc] = buf[b] + POM_ITBH_SIZE;
            dst[nc] = buf[b] + POM_ITBH_SIZE;       /* in place: staged before written */
            slen[nc] = plen[b];
            dlen[nc] = cap[b] - POM_ITBH_SIZE;
            nc++;
        } else if (len_ok) {
            len_ok[b] = 1;
        }
    }
    /* 2. the uncompressed records' payloads; the compressed ones are read chunk
     * by chunk just before the decode batch stages them */
    {
        size_t nu = 0;
        for (size_t b = 0; b < n; b++) {
            uint16_t algo;
            memcpy(&algo, buf[b] + POM_ITBH_ALGO_OFF, 2);
            if (!err[b] && algo != POM_COMPR_LZO)
                unc[nu++] = b;
        }
        read_payloads(fd, locations, buf, plen, err, unc, nu);
    }
    rc = LZO_E_OK;
    if (nc) {
        struct rd_dec d = {fd, locations, buf, plen, err, comp, PTHREAD_MUTEX_INITIALIZER};
        rc = pom_decompress_batch_chunked(src, slen, dst, dlen, st, nc, rd_dec_chunk, &d);
        pthread_mutex_destroy(&d.mu);
    }
    if (rc != LZO_E_OK)
        goto out;
    /* 3. itb_lzo_decompress's header updates (mds/itb.c:2949-2980) */
    for (size_t i = 0; i < nc; i++) {
        const size_t b = comp[i];
        if (err[b]) {                               /* the payload read failed: the */
            len[b] = 0;                             /* buffer past the header is undefined */
            continue;
        }
        const uint32_t zlen = rd32(buf[b] + POM_ITBH_ZLEN_OFF);
        derr[b] = st[i];
        if (len_ok)
            len_ok[b] = st[i] == LZO_E_OK && dlen[i] + POM_ITBH_SIZE == zlen;
        wr16(buf[b] + POM_ITBH_ALGO_OFF, POM_COMPR_NONE);
        wr32(buf[b] + POM_ITBH_LEN_OFF, (uint32_t)(dlen[i] + POM_ITBH_SIZE));
        len[b] = dlen[i] + POM_ITBH_SIZE;
    }
out:
    free(plen);
    free(comp);
    free(unc);
    free(src);
    free(dst);
    free(slen);
    free(dlen);
    free(st);
    return rc;
}
