/*
 * split_mock.c -- test harness (not part of the product library): drives
 * pomegranate_amd/csrc/batch_split.c, the host-batch planner of
 * liblzo_mi355x.so, on the CPU with a stand-in for each GPU's work, so the
 * device split, chunking and reassembly are checked without a GPU
 * (tests/test_split.py).  The stand-in writes block b's input reversed into
 * dst[b] and records which device, chunk and position handled it.
 */
#include <stdint.h>
#include <stdlib.h>

#include "batch_split.h"

struct mock {
    const uint8_t *const *src;
    const size_t *len;
    uint8_t *const *dst;
    const size_t *cost;
    size_t budget, max_blocks;
    struct pom_plan plan;
    int *dev_of;
    long *chunk_of, *seq_of;
};

static int mock_device(void *arg, int d)
{
    struct mock *m = arg;
    const size_t *ids = m->plan.by_dev + m->plan.dev_off[d];
    const size_t n = m->plan.dev_off[d + 1] - m->plan.dev_off[d];
    long chunk = 0;
    for (size_t from = 0; from < n; chunk++) {
        const size_t end = pom_chunk_end(ids, from, n, m->cost, m->budget, m->max_blocks);
        for (size_t i = from; i < end; i++) {
            const size_t b = ids[i];
            for (size_t k = 0; k < m->len[b]; k++)
                m->dst[b][k] = m->src[b][m->len[b] - 1 - k];
            m->dev_of[b] = d;
            m->chunk_of[b] = chunk;
            m->seq_of[b] = (long)i;
        }
        from = end;
    }
    return 0;
}

int mock_batch(size_t n, const uint8_t *const *src, const size_t *len, uint8_t *const *dst,
               int ndev_max, size_t min_dev_cost, size_t budget, size_t max_blocks, int *dev_of,
               long *chunk_of, long *seq_of, int *ndev_used)
{
    size_t *cost = malloc((n ? n : 1) * sizeof(size_t));
    if (!cost)
        return -1;
    for (size_t b = 0; b < n; b++)
        cost[b] = 2 * len[b];                  /* input plus an output of the same size */
    struct mock m = {src, len, dst, cost, budget, max_blocks, {0, 1, NULL, NULL}, dev_of,
                     chunk_of, seq_of};
    int rc = pom_plan_make(&m.plan, n, cost, ndev_max, min_dev_cost);
    if (rc == 0) {
        *ndev_used = m.plan.ndev;
        rc = pom_run_devices(m.plan.ndev, mock_device, &m);
        pom_plan_free(&m.plan);
    }
    free(cost);
    return rc;
}

/* POM_LZO_DEVICES parsing (batch_split.c), exposed for tests/test_split.py */
int mock_parse_devices(const char *list, int count, int max_dev, int *devs)
{
    return pom_parse_devices(list, count, max_dev, devs);
}

/* pom_pwritev_all (io_util.c) under a writer that writes at most `g_step`
 * bytes per call, cut inside iovecs, and fails every third call with EINTR. */
#include <errno.h>
#include <string.h>
#include <sys/uio.h>
#include "io_util.h"

static size_t g_step;
static unsigned g_calls;
static uint8_t *g_file;

static ssize_t short_pwritev(int fd, const struct iovec *iov, int n, off_t off)
{
    (void)fd;
    if (++g_calls % 3 == 0) {
        errno = EINTR;
        return -1;
    }
    size_t left = g_step, w = 0;
    for (int i = 0; i < n && left; i++) {
        size_t k = iov[i].iov_len < left ? iov[i].iov_len : left;
        memcpy(g_file + off + w, iov[i].iov_base, k);
        w += k;
        left -= k;
    }
    return (ssize_t)w;
}

int mock_pwritev_all(uint8_t *file, const uint8_t *const *bufs, const size_t *lens, int n,
                     size_t step, long off)
{
    struct iovec iov[64];
    if (n > 64)
        return -1;
    for (int i = 0; i < n; i++) {
        iov[i].iov_base = (void *)bufs[i];
        iov[i].iov_len = lens[i];
    }
    g_step = step;
    g_calls = 0;
    g_file = file;
    return pom_pwritev_all(-1, iov, n, (off_t)off, short_pwritev);
}
