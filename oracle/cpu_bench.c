/* oracle/cpu_bench.c -- native CPU baseline harness (TEST/BENCH INFRASTRUCTURE
 * ONLY: bench.py's cpu_baseline leg runs it; no product path uses it).
 *
 * Times the reference's own lib/minilzo.c (oracle/_ref/libminilzo_ref.so,
 * compiled in place from the reference sources by oracle/Makefile) -- or, where
 * the reference was not built, the oracle port (oracle/liboracle.so) -- on a
 * fixed number of host threads with no Python in the loop:
 *
 *   cpu_bench LIB SAMPLE THREADS SECONDS [PIN] [WRK]
 *
 * SAMPLE holds the blocks: u32 count, then per block u32 n, u32 z, n plain
 * bytes, z compressed bytes (bench.py writes it from the GPU's own batch).
 * Each thread is pinned to one CPU of the process's affinity set (PIN "1",
 * the default: thread t to its t-th CPU, wrapping; "spread": CPU t * (set /
 * THREADS); "0": not pinned), owns its wrkmem and buffers, and takes the blocks
 * t, t + THREADS, ... round robin.  Phase 1 decompresses (lzo1x_decompress,
 * the unchecked decoder Pomegranate's callers use: mds/itb.c:2964,
 * mdsl/gc.c:770) for 0.6 * SECONDS, phase 2 compresses (lzo1x_1_compress,
 * mds/itb.c:2923) for 0.4 * SECONDS, both threads started together behind a
 * barrier.  WRK "reuse" (the default): as in mds/itb.c:2913, a thread reuses
 * its wrkmem across calls without clearing it, so the dictionary holds the
 * previous blocks' positions; "zero": the wrkmem is zeroed before every call
 * (inside the timed loop, as a caller that wants the defined output would).
 * Environment POM_CPU_AVOID=c: CPU c (the launching process's) takes no
 * thread while the threads are fewer than the affinity set.
 * Before timing, every block is checked: decompress
 * gives the plain bytes, and compress with a zero-filled wrkmem gives exactly
 * the compressed bytes of the sample (the GPU's -- C3 byte identity).
 *
 * Prints one JSON object: bytes/s per phase over the phase's wall time, the
 * per-thread rates, and the CPUs used.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef int (*ref_fn)(const uint8_t *, unsigned long, uint8_t *, unsigned long *, void *);
typedef int (*port_comp_fn)(const uint8_t *, size_t, uint8_t *, size_t *);
typedef int (*port_dec_fn)(const uint8_t *, size_t, uint8_t *, size_t *);

static ref_fn ref_compress, ref_decompress;
static port_comp_fn port_compress;
static port_dec_fn port_decompress;
static int is_ref;

struct block { uint32_t n, z; const uint8_t *plain, *comp; };
static struct block *blocks;
static uint32_t nblocks, max_n;

#define WRKMEM (1u << 17)          /* LZO1X_1_MEM_COMPRESS with 8-byte dict entries */

static int do_compress(const uint8_t *in, uint32_t n, uint8_t *out, size_t *olen, void *wrk)
{
    if (is_ref) {
        unsigned long ol = 0;
        int rc = ref_compress(in, n, out, &ol, wrk);
        *olen = ol;
        return rc;
    }
    return port_compress(in, n, out, olen);
}

static int do_decompress(const uint8_t *in, uint32_t z, uint8_t *out, size_t cap, size_t *olen)
{
    if (is_ref) {
        unsigned long ol = cap;
        int rc = ref_decompress(in, z, out, &ol, NULL);
        *olen = ol;
        return rc;
    }
    *olen = cap;
    return port_decompress(in, z, out, olen);
}

static double now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

struct thr {
    pthread_t tid;
    int index, cpu;
    double dec_s, comp_s;           /* phase lengths */
    pthread_barrier_t *bar;
    double dec_bytes, dec_time, comp_bytes, comp_time;
    int errors;
};
static int nthreads, zero_wrk;

static void *worker(void *arg)
{
    struct thr *t = arg;
    if (t->cpu >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(t->cpu, &set);
        pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
    }
    uint8_t *out = malloc((size_t)max_n + max_n / 16 + 128);
    void *wrk = calloc(1, WRKMEM);
    uint32_t b = (uint32_t)t->index % nblocks;
    pthread_barrier_wait(t->bar);
    double t0 = now(), end = t0 + t->dec_s, bytes = 0, t1 = t0;
    while (t1 < end) {
        size_t ol;
        int rc = do_decompress(blocks[b].comp, blocks[b].z, out, (size_t)max_n + 64, &ol);
        t->errors += rc != 0 || ol != blocks[b].n;
        bytes += blocks[b].n;
        b = (b + (uint32_t)nthreads) % nblocks;
        t1 = now();
    }
    t->dec_bytes = bytes;
    t->dec_time = t1 - t0;
    pthread_barrier_wait(t->bar);
    t0 = now();
    end = t0 + t->comp_s;
    bytes = 0;
    t1 = t0;
    b = (uint32_t)t->index % nblocks;
    while (t1 < end) {
        size_t ol;
        if (zero_wrk)
            memset(wrk, 0, WRKMEM);
        int rc = do_compress(blocks[b].plain, blocks[b].n, out, &ol, wrk);
        t->errors += rc != 0;
        bytes += blocks[b].n;
        b = (b + (uint32_t)nthreads) % nblocks;
        t1 = now();
    }
    t->comp_bytes = bytes;
    t->comp_time = t1 - t0;
    free(out);
    free(wrk);
    return NULL;
}

static uint8_t *slurp(const char *path, size_t *len)
{
    FILE *f = fopen(path, "rb");
    if (!f)
        return NULL;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *p = malloc(n > 0 ? (size_t)n : 1);
    if (p && fread(p, 1, (size_t)n, f) != (size_t)n) {
        free(p);
        p = NULL;
    }
    fclose(f);
    *len = (size_t)n;
    return p;
}

int main(int argc, char **argv)
{
    if (argc < 5) {
        fprintf(stderr, "usage: %s LIB SAMPLE THREADS SECONDS [PIN: 1|0|spread] [WRK: reuse|zero]\n",
                argv[0]);
        return 2;
    }
    void *lib = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    if (!lib) {
        fprintf(stderr, "dlopen %s: %s\n", argv[1], dlerror());
        return 2;
    }
    ref_compress = (ref_fn)dlsym(lib, "lzo1x_1_compress");
    ref_decompress = (ref_fn)dlsym(lib, "lzo1x_decompress");
    is_ref = ref_compress && ref_decompress;
    if (is_ref) {
        typedef int (*init_fn)(unsigned, int, int, int, int, int, int, int, int, int);
        init_fn init = (init_fn)dlsym(lib, "__lzo_init_v2");
        if (!init || init(0x2040, 2, 4, 8, 4, 8, 8, 8, 8, 48) != 0) {
            fprintf(stderr, "lzo_init failed\n");
            return 2;
        }
    } else {
        port_compress = (port_comp_fn)dlsym(lib, "oracle_lzo1x_1_compress");
        port_decompress = (port_dec_fn)dlsym(lib, "oracle_lzo1x_decompress_unchecked");
        if (!port_compress || !port_decompress) {
            fprintf(stderr, "%s: neither lib/minilzo.c nor the oracle port\n", argv[1]);
            return 2;
        }
    }
    size_t len;
    uint8_t *s = slurp(argv[2], &len);
    if (!s || len < 4) {
        fprintf(stderr, "cannot read %s\n", argv[2]);
        return 2;
    }
    memcpy(&nblocks, s, 4);
    blocks = calloc(nblocks ? nblocks : 1, sizeof(*blocks));
    size_t at = 4;
    for (uint32_t i = 0; i < nblocks; i++) {
        if (at + 8 > len)
            return 2;
        memcpy(&blocks[i].n, s + at, 4);
        memcpy(&blocks[i].z, s + at + 4, 4);
        at += 8;
        if (at + blocks[i].n + blocks[i].z > len)
            return 2;
        blocks[i].plain = s + at;
        blocks[i].comp = s + at + blocks[i].n;
        at += (size_t)blocks[i].n + blocks[i].z;
        max_n = blocks[i].n > max_n ? blocks[i].n : max_n;
    }
    if (!nblocks)
        return 2;
    nthreads = atoi(argv[3]);
    double secs = atof(argv[4]);
    if (nthreads < 1)
        nthreads = 1;

    /* the sample is checked first: decode, and byte identity of the
     * compressed bytes with a zero-filled wrkmem (SURVEY.md finding 3) */
    uint8_t *out = malloc((size_t)max_n + max_n / 16 + 128);
    void *wrk = malloc(WRKMEM);
    uint32_t identical = 0, decoded = 0;
    for (uint32_t i = 0; i < nblocks; i++) {
        size_t ol;
        memset(wrk, 0, WRKMEM);
        if (do_compress(blocks[i].plain, blocks[i].n, out, &ol, wrk) == 0 && ol == blocks[i].z &&
            memcmp(out, blocks[i].comp, ol) == 0)
            identical++;
        if (do_decompress(blocks[i].comp, blocks[i].z, out, (size_t)max_n + 64, &ol) == 0 &&
            ol == blocks[i].n && memcmp(out, blocks[i].plain, ol) == 0)
            decoded++;
    }
    free(out);
    free(wrk);

    /* PIN: "1" (default) thread t on the t-th CPU of the affinity set, "0" no
     * pinning (the scheduler places the threads), "spread" thread t on CPU
     * t * (affinity set / threads) of the set */
    const char *pin = argc > 5 ? argv[5] : "1";
    zero_wrk = argc > 6 && strcmp(argv[6], "zero") == 0;
    const int nthr_arg = atoi(argv[3]) > 0 ? atoi(argv[3]) : 1;
    const char *avoid_s = getenv("POM_CPU_AVOID");
    const int avoid = avoid_s && *avoid_s ? atoi(avoid_s) : -1;
    cpu_set_t aff;
    int cpus[CPU_SETSIZE], naff = 0, nset = 0;
    if (sched_getaffinity(0, sizeof(aff), &aff) == 0)
        for (int c = 0; c < CPU_SETSIZE; c++)
            nset += CPU_ISSET(c, &aff) ? 1 : 0;
    for (int c = 0; c < CPU_SETSIZE; c++)
        if (CPU_ISSET(c, &aff) && !(c == avoid && nthr_arg < nset))
            cpus[naff++] = c;
    const int stride = strcmp(pin, "spread") == 0 && naff > nthr_arg ? naff / nthr_arg : 1;
    if (strcmp(pin, "0") == 0)
        naff = 0;
    struct thr *T = calloc((size_t)nthreads, sizeof(*T));
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)nthreads);
    for (int i = 0; i < nthreads; i++) {
        T[i].index = i;
        T[i].cpu = naff ? cpus[(i * stride) % naff] : -1;
        T[i].dec_s = 0.6 * secs;
        T[i].comp_s = 0.4 * secs;
        T[i].bar = &bar;
        pthread_create(&T[i].tid, NULL, worker, &T[i]);
    }
    double db = 0, dt = 0, cb = 0, ct = 0;
    int errors = 0;
    for (int i = 0; i < nthreads; i++) {
        pthread_join(T[i].tid, NULL);
        db += T[i].dec_bytes;
        cb += T[i].comp_bytes;
        dt = T[i].dec_time > dt ? T[i].dec_time : dt;
        ct = T[i].comp_time > ct ? T[i].comp_time : ct;
        errors += T[i].errors;
    }
    double sample_bytes = 0;
    for (uint32_t i = 0; i < nblocks; i++)
        sample_bytes += (double)blocks[i].n + blocks[i].z;
    const uint32_t per_thr = (nblocks + (uint32_t)nthreads - 1) / (uint32_t)nthreads;
    printf("{\"wrkmem\": \"%s\", \"avoided_cpu\": %d, \"sample_bytes\": %.0f, "
           "\"per_thread_working_set_bytes\": %.0f, ",
           zero_wrk ? "zero" : "reuse", avoid, sample_bytes, sample_bytes / nblocks * per_thr);
    printf("\"kind\": \"%s\", \"threads\": %d, \"affinity_cpus\": %d, \"pin\": \"%s\", \"blocks\": %u, "
           "\"decompress_Bps\": %.1f, \"compress_Bps\": %.1f, \"decompress_s\": %.3f, "
           "\"compress_s\": %.3f, \"byte_identical\": %u, \"decoded\": %u, \"errors\": %d, "
           "\"per_thread_decompress_Bps\": [",
           is_ref ? "reference" : "port", nthreads, naff, pin, nblocks, dt > 0 ? db / dt : 0.0,
           ct > 0 ? cb / ct : 0.0, dt, ct, identical, decoded, errors);
    for (int i = 0; i < nthreads; i++)
        printf("%s%.1f", i ? ", " : "", T[i].dec_time > 0 ? T[i].dec_bytes / T[i].dec_time : 0.0);
    printf("], \"per_thread_compress_Bps\": [");
    for (int i = 0; i < nthreads; i++)
        printf("%s%.1f", i ? ", " : "", T[i].comp_time > 0 ? T[i].comp_bytes / T[i].comp_time : 0.0);
    printf("], \"cpus\": [");
    for (int i = 0; i < nthreads; i++)
        printf("%s%d", i ? ", " : "", T[i].cpu);
    printf("]}\n");
    return errors ? 1 : 0;
}
