/* batch_split.h -- how a host batch is spread over GPUs and cut into chunks
 * (internal to liblzo_mi355x.so; plain C, no HIP, so the CPU tests drive it
 * through tests/native/split_mock.c).
 *
 * The reference codes one block per call on whichever thread holds it
 * (mds/txg.c:700-770 compresses each dirty ITB of a commit in turn).  Here a
 * batch of blocks is ordered largest first, dealt round robin over the GPUs
 * (rank r of that order goes to GPU r mod G, so every GPU gets a similar mix
 * of sizes), and each GPU's share is cut into chunks of bounded staging size
 * that are pipelined through two streams.
 */
#ifndef POM_BATCH_SPLIT_H
#define POM_BATCH_SPLIT_H 1

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

struct pom_plan {
    size_t n;           /* blocks */
    int ndev;           /* devices used, 1 <= ndev */
    size_t *by_dev;     /* n block ids grouped by device, each group largest cost first */
    size_t *dev_off;    /* ndev + 1: device d has by_dev[dev_off[d] .. dev_off[d + 1]) */
};

/* ndev = min(ndev_max, n, max(1, total cost / min_dev_cost)).  Returns 0, or
 * -1 when out of memory.  cost[b]: bytes block b moves (input + output). */
int pom_plan_make(struct pom_plan *P, size_t n, const size_t *cost, int ndev_max,
                  size_t min_dev_cost);
void pom_plan_free(struct pom_plan *P);

/* End of the chunk that starts at ids[from]: the longest run whose cost stays
 * within budget (at least one block) and holds at most max_blocks blocks. */
size_t pom_chunk_end(const size_t *ids, size_t from, size_t n, const size_t *cost, size_t budget,
                     size_t max_blocks);

/* fn(arg, d) for every d in [0, ndev): on ndev threads when ndev > 1 (the
 * caller's thread waits), inline when ndev == 1.  Returns 0 when every call
 * returned 0, else the first non-zero result in device order. */
typedef int (*pom_dev_fn)(void *arg, int d);
int pom_run_devices(int ndev, pom_dev_fn fn, void *arg);

/* POM_LZO_DEVICES parsing: device ids in [0, min(count, max_dev)) from a
 * comma list, in order, each at most once.  Returns how many were stored. */
int pom_parse_devices(const char *list, int count, int max_dev, int *devs);

#ifdef __cplusplus
}
#endif

#endif
