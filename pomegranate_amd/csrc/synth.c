/*
 * synth.c -- deterministic synthetic block generators for the LZO1X harness
 * (libpom_synth.so).  Used by tests/, bench.py and tests/golden/make_golden.py
 * to build the same blocks here and on the GPU box; not part of the drop-in
 * codec library.
 *
 * Models:
 *   0 RANDOM   uniform bytes from xorshift64            (config C1)
 *   1 ITB      ITB payload image: zeroed lock array, ITE bitmap, index table,
 *              512-B ITEs (include/xtable.h:136-144, include/ite.h:78-114,
 *              include/hvfs_common.h:61-115)             (configs C2-C5)
 *   2 ZEROS    all zero
 *   3 ALPHA4   uniform over a 4-symbol alphabet
 *   4 LZLIKE   copies of earlier spans with sparse noise
 *   5 TEXT     words from a small vocabulary
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { uint64_t s; } xs64;

static inline uint64_t xs_next(xs64 *r)
{
    uint64_t s = r->s;
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    r->s = s;
    return s;
}

static inline void put64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }
static inline void put32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }
static inline void put16(uint8_t *p, uint16_t v) { memcpy(p, &v, 2); }

static void fill_random(xs64 *r, uint8_t *buf, size_t n)
{
    size_t i = 0;
    for (; i + 8 <= n; i += 8)
        put64(buf + i, xs_next(r));
    if (i < n) {
        uint64_t v = xs_next(r);
        memcpy(buf + i, &v, n - i);
    }
}

/* ITB payload layout, offsets relative to &itb->lock (mds/itb.c:2921). */
enum {
    ITB_LOCKS = 3584,      /* 64 x struct itb_lock (56 B), zeroed (mds/txg.c:754) */
    ITB_BITMAP = 3584,     /* 128 B */
    ITB_INDEX = 3712,      /* 2048 x u32 {entry:15, conflict:15, flag:2} */
    ITB_ITES = 11904,      /* struct ite[], 512 B each */
    ITE_SIZE = 512
};

static void fill_itb(xs64 *r, uint8_t *buf, size_t n)
{
    /* Build into a scratch image long enough for whole ITEs, then truncate. */
    size_t k = n > ITB_ITES ? (n - ITB_ITES + ITE_SIZE - 1) / ITE_SIZE : 0;
    size_t full = ITB_ITES + k * ITE_SIZE;
    uint8_t *img = full > n ? calloc(1, full) : buf;
    if (img == buf)
        memset(buf, 0, n);
    if (!img)
        return;
    for (size_t i = 0; i < k && i < 1024; i++) {
        img[ITB_BITMAP + i / 8] |= (uint8_t)(1u << (i % 8));
        put32(img + ITB_INDEX + 4 * i, (uint32_t)i | (1u << 30));
    }
    for (size_t i = 0; i < k; i++) {
        uint8_t *e = img + ITB_ITES + i * ITE_SIZE;
        uint64_t hash = xs_next(r);
        uint64_t uuid = xs_next(r) & 0x7FFFFFFFFFFFFFFFull;
        uint64_t size = xs_next(r) % 1000000u;
        uint64_t t0 = 1300000000ull + xs_next(r) % 1000000u;
        uint64_t c0 = xs_next(r);
        char name[32];
        int nl = snprintf(name, sizeof(name), "file-%08x.jpg", (unsigned)(hash >> 32));
        put64(e + 0, hash);
        put64(e + 8, uuid);
        put32(e + 16, 0x80000000u);              /* ITE_FLAG_NORMAL */
        put32(e + 20, (uint32_t)nl);             /* namelen */
        uint8_t *m = e + 24;                     /* struct mdu, 80 B */
        put32(m + 0, 0x02000400u);               /* SMALL | LZO */
        put32(m + 4, 1000);                      /* uid */
        put32(m + 8, 1000);                      /* gid */
        put16(m + 12, 0100644);                  /* mode */
        put16(m + 14, 1);                        /* nlink */
        put64(m + 16, size);
        put64(m + 32, t0);                       /* atime */
        put64(m + 40, t0 + (c0 & 0xFF));         /* ctime */
        put64(m + 48, t0 + (c0 & 0xFF));         /* mtime */
        memcpy(e + 104, name, (size_t)nl);       /* name[256] */
        uint8_t *col = e + 368;                  /* column[0] */
        put64(col + 0, c0 % 4096u);
        put64(col + 8, size);
        put64(col + 16, (uint32_t)(c0 >> 32));
    }
    if (img != buf) {
        memcpy(buf, img, n);
        free(img);
    }
}

static void fill_alpha4(xs64 *r, uint8_t *buf, size_t n)
{
    static const uint8_t sym[4] = { 'A', 'C', 'G', 'T' };
    uint64_t v = 0;
    for (size_t i = 0; i < n; i++) {
        if ((i & 31) == 0)
            v = xs_next(r);
        buf[i] = sym[v & 3];
        v >>= 2;
    }
}

static void fill_lzlike(xs64 *r, uint8_t *buf, size_t n)
{
    size_t i = 0;
    while (i < n) {
        uint64_t v = xs_next(r);
        size_t run = 3 + (v & 63);
        if (i < 64 || (v >> 8) % 4 == 0) {       /* fresh literals */
            for (size_t j = 0; j < run && i < n; j++, i++)
                buf[i] = (uint8_t)(xs_next(r) >> 24);
        } else {                                 /* copy from up to 64 KiB back */
            size_t back = 1 + (size_t)((v >> 16) % (i < 65536 ? i : 65536));
            for (size_t j = 0; j < run && i < n; j++, i++)
                buf[i] = buf[i - back];
            if (i < n && (v >> 40) % 8 == 0)
                buf[i - 1] ^= (uint8_t)(v >> 48);
        }
    }
}

static void fill_text(xs64 *r, uint8_t *buf, size_t n)
{
    static const char *words[] = {
        "the", "metadata", "server", "commits", "an", "index", "table",
        "block", "to", "storage", "layer", "with", "compressed", "entries",
        "of", "directory", "files", "and", "a", "ring", "manager", "\n" };
    const size_t nw = sizeof(words) / sizeof(words[0]);
    size_t i = 0;
    while (i < n) {
        const char *w = words[xs_next(r) % nw];
        size_t l = strlen(w);
        for (size_t j = 0; j < l && i < n; j++)
            buf[i++] = (uint8_t)w[j];
        if (i < n)
            buf[i++] = ' ';
    }
}

/* Fill one block.  The seed is mixed as in SURVEY.md Appendix B
 * (0x9E3779B97F4A7C15 ^ seed); a zero state is avoided. */
void pom_synth_fill(int model, uint64_t seed, uint8_t *buf, size_t n)
{
    xs64 r = { 0x9E3779B97F4A7C15ull ^ seed };
    if (r.s == 0)
        r.s = 1;
    switch (model) {
    case 0: fill_random(&r, buf, n); break;
    case 1: fill_itb(&r, buf, n); break;
    case 2: memset(buf, 0, n); break;
    case 3: fill_alpha4(&r, buf, n); break;
    case 4: fill_lzlike(&r, buf, n); break;
    default: fill_text(&r, buf, n); break;
    }
}

struct batch_job {
    int model;
    uint64_t seed0;
    const uint64_t *seeds;
    size_t nblocks;
    const uint64_t *offsets;
    const uint64_t *sizes;
    uint8_t *buf;
    size_t first, step;
};

static void *batch_worker(void *p)
{
    struct batch_job *j = p;
    for (size_t b = j->first; b < j->nblocks; b += j->step)
        pom_synth_fill(j->model, j->seeds ? j->seeds[b] : j->seed0 + b,
                       j->buf + j->offsets[b], j->sizes[b]);
    return NULL;
}

/* Fill nblocks blocks at buf + offsets[b]; block b uses seeds[b], or
 * seed0 + b when seeds is NULL. */
void pom_synth_batch_seeds(int model, uint64_t seed0, const uint64_t *seeds, size_t nblocks,
                           const uint64_t *offsets, const uint64_t *sizes,
                           uint8_t *buf, int nthreads)
{
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 64)
        nthreads = 64;
    pthread_t th[64];
    int started[64];
    struct batch_job jobs[64];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (struct batch_job){ model, seed0, seeds, nblocks, offsets, sizes, buf,
                                      (size_t)t, (size_t)nthreads };
        started[t] = pthread_create(&th[t], NULL, batch_worker, &jobs[t]) == 0;
        if (!started[t])
            batch_worker(&jobs[t]);   /* no thread: do this share inline */
    }
    for (int t = 0; t < nthreads; t++)
        if (started[t])
            pthread_join(th[t], NULL);
}

void pom_synth_batch(int model, uint64_t seed0, size_t nblocks, const uint64_t *offsets,
                     const uint64_t *sizes, uint8_t *buf, int nthreads)
{
    pom_synth_batch_seeds(model, seed0, NULL, nblocks, offsets, sizes, buf, nthreads);
}
