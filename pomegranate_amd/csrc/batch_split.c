/*
 * batch_split.c -- order, device split and chunking of host batches
 * (batch_split.h).  No HIP here: lzo_host.c supplies the per-device work.
 */
#include <pthread.h>
#include <stdlib.h>

#include "batch_split.h"

struct cost_id {
    size_t cost, id;
};

static int by_cost_desc(const void *a, const void *b)
{
    const struct cost_id *x = a, *y = b;
    if (x->cost != y->cost)
        return x->cost < y->cost ? 1 : -1;
    return x->id < y->id ? -1 : x->id > y->id;
}

int pom_plan_make(struct pom_plan *P, size_t n, const size_t *cost, int ndev_max,
                  size_t min_dev_cost)
{
    P->n = n;
    P->ndev = 1;
    P->by_dev = NULL;
    P->dev_off = NULL;
    size_t total = 0;
    for (size_t b = 0; b < n; b++)
        total += cost[b];
    size_t nd = ndev_max > 1 ? (size_t)ndev_max : 1;
    if (nd > n)
        nd = n ? n : 1;
    const size_t by_cost = min_dev_cost ? total / min_dev_cost : nd;
    if (nd > by_cost)
        nd = by_cost ? by_cost : 1;
    P->ndev = (int)nd;
    struct cost_id *o = malloc((n ? n : 1) * sizeof(*o));
    P->by_dev = malloc((n ? n : 1) * sizeof(size_t));
    P->dev_off = malloc((nd + 1) * sizeof(size_t));
    if (!o || !P->by_dev || !P->dev_off) {
        free(o);
        pom_plan_free(P);
        return -1;
    }
    for (size_t b = 0; b < n; b++) {
        o[b].cost = cost[b];
        o[b].id = b;
    }
    qsort(o, n, sizeof(*o), by_cost_desc);
    /* rank r -> device r mod nd; within a device the ranks stay in order */
    size_t at = 0;
    for (size_t d = 0; d < nd; d++) {
        P->dev_off[d] = at;
        for (size_t r = d; r < n; r += nd)
            P->by_dev[at++] = o[r].id;
    }
    P->dev_off[nd] = at;
    free(o);
    return 0;
}

void pom_plan_free(struct pom_plan *P)
{
    free(P->by_dev);
    free(P->dev_off);
    P->by_dev = NULL;
    P->dev_off = NULL;
}

size_t pom_chunk_end(const size_t *ids, size_t from, size_t n, const size_t *cost, size_t budget,
                     size_t max_blocks)
{
    if (from >= n)
        return n;
    size_t end = from + 1, used = cost[ids[from]];
    while (end < n && end - from < max_blocks && used + cost[ids[end]] <= budget)
        used += cost[ids[end++]];
    return end;
}

struct dev_job {
    pom_dev_fn fn;
    void *arg;
    int d;
    int rc;
};

static void *dev_thread(void *p)
{
    struct dev_job *j = p;
    j->rc = j->fn(j->arg, j->d);
    return NULL;
}

int pom_run_devices(int ndev, pom_dev_fn fn, void *arg)
{
    if (ndev <= 1)
        return fn(arg, 0);
    struct dev_job *jobs = calloc((size_t)ndev, sizeof(*jobs));
    pthread_t *th = calloc((size_t)ndev, sizeof(*th));
    char *started = calloc((size_t)ndev, 1);
    if (!jobs || !th || !started) {
        free(jobs);
        free(th);
        free(started);
        return -1;
    }
    for (int d = 0; d < ndev; d++) {
        jobs[d].fn = fn;
        jobs[d].arg = arg;
        jobs[d].d = d;
        started[d] = pthread_create(&th[d], NULL, dev_thread, &jobs[d]) == 0;
        if (!started[d])
            jobs[d].rc = -1;
    }
    int rc = 0;
    for (int d = 0; d < ndev; d++) {
        if (started[d])
            pthread_join(th[d], NULL);
        if (rc == 0 && jobs[d].rc != 0)
            rc = jobs[d].rc;
    }
    free(jobs);
    free(th);
    free(started);
    return rc;
}

/* A device listed twice is used once: two helper threads on one device would
 * share (and reallocate under each other) the calling thread's slots. */
int pom_parse_devices(const char *list, int count, int max_dev, int *devs)
{
    int n = 0;
    unsigned long long seen = 0;
    const char *p = list;
    if (max_dev > 64)
        max_dev = 64;
    while (*p && n < max_dev) {
        char *q;
        const long v = strtol(p, &q, 10);
        if (q == p)
            break;
        if (v >= 0 && v < count && v < max_dev && !(seen & (1ull << v))) {
            seen |= 1ull << v;
            devs[n++] = (int)v;
        }
        p = *q == ',' ? q + 1 : q;
    }
    return n;
}
