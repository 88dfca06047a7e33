/*
 * lzo_host.c -- host side of liblzo_mi355x.so, in C like the reference.
 *
 * Implements the minilzo.h call surface (lzo_init, lzo1x_1_compress,
 * lzo1x_decompress, lzo1x_decompress_safe; reference lib/minilzo.c) and the
 * batch API of lzo_mi355x.h on top of the HIP kernels.  Every codec call runs
 * on the GPU; there is no CPU codec in this library.  A call made without a
 * usable GPU returns LZO_E_ERROR and says why on stderr once.
 *
 * Threading: callers are MDS commit/service threads, the MDSL
 * GC thread and client threads.  Each host thread gets, on each GPU it uses,
 * two HIP streams with their own device/pinned staging (grown on demand up to
 * one chunk, freed at thread exit), so concurrent calls never share device
 * state.  A host batch spreads over the GPUs on one helper thread per GPU
 * (batch_split.c), which use the calling thread's per-GPU resources.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <hip/hip_runtime_api.h>

#include "batch_split.h"
#include "lzo_mi355x.h"
#include "lzo_mi355x_kernels.h"
#include "minilzo.h"

/* Debug and experiment switches: ONE environment variable, POM_LZO_DEBUG,
 * a comma-separated list of key=value.  No product path
 * needs it; an unset key takes its default.  Keys: decoder=fast|win
 * (device batches), sc_copy=1, sc_combine=0, sc_lat=0, sc_lat_min=BYTES,
 * sc_trace=1, host_timing=1, slots=N, chunk_mb=N, dec_small_first=0, ooo=0, enc_lds_max=N, enc_waves=1|2,
 * enc_grid=N, fail_chunk=K (tests: a device's K-th chunk delivery fails).  The variable is read once, at the first use, into a private
 * copy; lzo_mi355x_debug_reload() reads it again (tests change it between
 * calls).  So the hot paths never call getenv.  Each (re)load publishes a new,
 * immutable copy through one atomic pointer, so a lookup on any thread reads
 * either the old or the new string whole, never one being rewritten (ADVICE
 * r5); the replaced copies are not freed (a reload is a test-time event and a
 * lookup may still be reading one). */
static pthread_mutex_t dbg_mu = PTHREAD_MUTEX_INITIALIZER;
static const char *dbg_cur;

static void dbg_load(int always)
{
    pthread_mutex_lock(&dbg_mu);
    if (always || !dbg_cur) {
        const char *e = getenv("POM_LZO_DEBUG");
        char *copy = strdup(e ? e : "");
        if (copy)
            __atomic_store_n(&dbg_cur, copy, __ATOMIC_RELEASE);
    }
    pthread_mutex_unlock(&dbg_mu);
}

void lzo_mi355x_debug_reload(void)
{
    dbg_load(1);
}

const char *pom_dbg_str(const char *key, char *buf, size_t n)
{
    const char *e = __atomic_load_n(&dbg_cur, __ATOMIC_ACQUIRE);
    if (!e) {
        dbg_load(0);                              /* first use */
        e = __atomic_load_n(&dbg_cur, __ATOMIC_ACQUIRE);
    }
    if (!e || !*e || !n)
        return NULL;
    const size_t kl = strlen(key);
    for (const char *p = e; *p;) {
        const char *end = strchr(p, ',');
        const size_t len = end ? (size_t)(end - p) : strlen(p);
        if (len > kl && strncmp(p, key, kl) == 0 && p[kl] == '=') {
            size_t vl = len - kl - 1;
            if (vl >= n)
                vl = n - 1;
            memcpy(buf, p + kl + 1, vl);
            buf[vl] = 0;
            return buf;
        }
        if (!end)
            break;
        p = end + 1;
    }
    return NULL;
}

long pom_dbg_int(const char *key, long dflt)
{
    char buf[32];
    const char *v = pom_dbg_str(key, buf, sizeof buf);
    return v && *v ? atol(v) : dflt;
}

#define ALIGN_UP(x, a) (((x) + (size_t)(a) - 1) & ~((size_t)(a) - 1))

/* ------------------------------------------------------------------------ */
/* GPU availability (checked once per process)                              */
/* ------------------------------------------------------------------------ */
static pthread_once_t gpu_once = PTHREAD_ONCE_INIT;
static int gpu_count;

static void gpu_probe(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        fprintf(stderr, "liblzo_mi355x: no usable GPU (hipGetDeviceCount=%d); "
                        "the MI355X LZO1X codec has no CPU fallback\n", n);
        n = 0;
    }
    gpu_count = n;
}

int lzo_mi355x_device_count(void)
{
    pthread_once(&gpu_once, gpu_probe);
    return gpu_count;
}

size_t lzo_mi355x_worst_compress(size_t n)
{
    return n + n / 16 + 64 + 3;
}

/* ------------------------------------------------------------------------ */
/* Per-thread, per-device streams and staging                               */
/* ------------------------------------------------------------------------ */
/* A staging slot: one stream with its device and pinned host buffers (grown
 * on demand; a host batch's chunks keep them bounded, see kChunkBudget). */
struct slot {
    hipStream_t stream;
    uint8_t *dmem;
    size_t dcap;
    uint8_t *hmem;
    size_t hcap;
};

/* A host thread's resources on one device: kSlots slots, so that several
 * chunks are in flight (copies and kernels of some while others are packed
 * or unpacked on the host). */
enum { kSlots = 4 };

struct dctx {
    int ready;
    struct slot s[kSlots];
};

enum { kMaxDev = 16 };

struct tctx {
    struct dctx dev[kMaxDev];
};

static pthread_key_t tkey;
static pthread_once_t tkey_once = PTHREAD_ONCE_INIT;

static void tctx_free(void *p)
{
    struct tctx *t = p;
    if (!t)
        return;
    for (int d = 0; d < kMaxDev; d++) {
        struct dctx *c = &t->dev[d];
        if (!c->ready)
            continue;
        hipSetDevice(d);
        for (int k = 0; k < kSlots; k++) {
            if (c->s[k].dmem)
                hipFree(c->s[k].dmem);
            if (c->s[k].hmem)
                hipHostFree(c->s[k].hmem);
            hipStreamDestroy(c->s[k].stream);
        }
    }
    free(t);
}

static void tkey_make(void)
{
    pthread_key_create(&tkey, tctx_free);
}

static struct tctx *tctx_get(void)
{
    if (lzo_mi355x_device_count() <= 0)
        return NULL;
    pthread_once(&tkey_once, tkey_make);
    struct tctx *t = pthread_getspecific(tkey);
    if (!t) {
        t = calloc(1, sizeof(*t));
        if (!t)
            return NULL;
        pthread_setspecific(tkey, t);
    }
    return t;
}

/* The calling thread's context on `device`, which must be its current device. */
static struct dctx *dctx_get(struct tctx *t, int device)
{
    if (device < 0 || device >= kMaxDev)
        return NULL;
    struct dctx *c = &t->dev[device];
    if (!c->ready) {
        for (int k = 0; k < kSlots; k++)
            if (hipStreamCreateWithFlags(&c->s[k].stream, hipStreamNonBlocking) != hipSuccess) {
                while (k-- > 0)
                    hipStreamDestroy(c->s[k].stream);
                return NULL;
            }
        c->ready = 1;
    }
    return c;
}

static int slot_reserve(struct slot *t, size_t dbytes, size_t hbytes)
{
    /* growth: +25%, or doubling up to 64 MiB (combined single calls grow
     * their groups step by step; each regrowth is a hipMalloc/hipHostMalloc) */
    const size_t kDoubleMax = (size_t)64 << 20;
    if (dbytes > t->dcap) {
        const size_t old = t->dcap;
        if (t->dmem)
            hipFree(t->dmem);
        t->dmem = NULL;
        t->dcap = 0;
        size_t want = ALIGN_UP(dbytes + dbytes / 4, 1 << 20);
        if (want < 2 * old && 2 * old <= kDoubleMax)
            want = 2 * old;
        if (hipMalloc((void **)&t->dmem, want) != hipSuccess)
            return -1;
        t->dcap = want;
    }
    if (hbytes > t->hcap) {
        const size_t old = t->hcap;
        if (t->hmem)
            hipHostFree(t->hmem);
        t->hmem = NULL;
        t->hcap = 0;
        size_t want = ALIGN_UP(hbytes + hbytes / 4, 1 << 20);
        if (want < 2 * old && 2 * old <= kDoubleMax)
            want = 2 * old;
        if (hipHostMalloc((void **)&t->hmem, want, hipHostMallocDefault) != hipSuccess)
            return -1;
        t->hcap = want;
    }
    return 0;
}

/* The slot single calls use: slot 0 on the calling thread's current device. */
static struct slot *single_slot(void)
{
    struct tctx *t = tctx_get();
    int dev = 0;
    if (!t || hipGetDevice(&dev) != hipSuccess)
        return NULL;
    struct dctx *c = dctx_get(t, dev);
    return c ? &c->s[0] : NULL;
}

/* ------------------------------------------------------------------------ */
/* Device-resident batch entry points                                       */
/* ------------------------------------------------------------------------ */
int lzo_mi355x_compress_dev(const uint8_t *src, const uint64_t *src_off,
                            const uint32_t *src_len, uint8_t *dst,
                            const uint64_t *dst_off, const uint32_t *dst_cap,
                            uint32_t *out_len, int32_t *status, uint32_t nblocks,
                            void *scratch, void *stream)
{
    /* blocks up to 16 MiB: the throughput encoder; larger ones are left
     * pending for the general encoder, whose other workgroups exit at once */
    hipStream_t s = (hipStream_t)stream;
    if (nblocks == 0)
        return 0;
    if (lzo_mi355x_launch_compress_fast(src, src_off, src_len, dst, dst_off, dst_cap, out_len,
                                        status, nblocks, scratch,
                                        scratch ? lzo_mi355x_compress_scratch(nblocks) : 0, s) != 0)
        return -1;
    return lzo_mi355x_launch_compress(src, src_off, src_len, dst, dst_off, dst_cap, out_len,
                                      status, nblocks, 1, s);
}

/* Scratch (256-byte aligned parts):
 *   [0]     fallback count u32
 *   [256]   op-set pool counters (LZO_MI355X_FAST_POOL_BYTES)
 *   then    op-set return ring, u64 per set
 *   then    the fast decoder's fallback list, u32 per block
 *   then    (more blocks than resident workgroups) the start order, u32 per block
 *   then    the op-slot sets, one per workgroup resident at once
 * Only the fallback list and the start order grow with nblocks (4 bytes a
 * block each). */
enum { SCR_POOL = 256, SCR_RING = SCR_POOL + LZO_MI355X_FAST_POOL_BYTES };

static size_t scr_sets(uint32_t nblocks)
{
    const uint32_t r = lzo_mi355x_fast_resident_blocks();
    return nblocks < r ? nblocks : r;
}

static size_t scr_head(uint32_t nblocks)
{
    return ALIGN_UP(SCR_RING + 8 * scr_sets(nblocks), 256);
}

static size_t scr_order_bytes(uint32_t nblocks)
{
    return nblocks > lzo_mi355x_fast_resident_blocks() ? ALIGN_UP(4 * (size_t)nblocks, 256) : 0;
}

static size_t scr_order_off(uint32_t nblocks)
{
    return scr_head(nblocks) + ALIGN_UP(4 * (size_t)nblocks, 256);
}

static size_t scr_ops_off(uint32_t nblocks)
{
    return scr_order_off(nblocks) + scr_order_bytes(nblocks);
}

size_t lzo_mi355x_decompress_scratch(uint32_t nblocks)
{
    return scr_ops_off(nblocks) + scr_sets(nblocks) * lzo_mi355x_fast_ops_bytes_per_block();
}

/* Which throughput decoder a batch uses: the op-set decoder
 * (lzo1x_decode_fast.hip: 16 blocks per CU) or the windowed one
 * (lzo1x_decode_win.hip: 2 blocks per CU, a 64 KiB LDS output ring, never
 * reads its own output back).  Debug key decoder=fast|win forces one;
 * single calls always use the windowed one (see single_call). */
enum { DEC_FAST = 0, DEC_WIN = 1 };
static int use_win_decoder(uint32_t nblocks)
{
    char buf[16];
    const char *e = pom_dbg_str("decoder", buf, sizeof buf);
    if (e)
        return strcmp(e, "win") == 0 ? DEC_WIN : DEC_FAST;
    /* default: the windowed decoder while the batch fits two workgroups per
     * CU (one round; lone blocks decode 1.3-1.5x faster there), the op-set
     * decoder for larger batches (16 blocks per CU) */
    const uint32_t cus = lzo_mi355x_fast_resident_blocks() / 16u;
    return nblocks <= 2u * (cus ? cus : 256u);
}

/* Single calls: the kernels write the output and its length/status straight
 * into the pinned host staging (hipHostMalloc, mapped into the device's
 * address space), so nothing is copied back but what was produced; the
 * caller reads it only after the stream synchronisation, which is what makes
 * the kernels' writes visible to the host.  debug key sc_copy=1: the round-2
 * path (device staging, one D2H copy of the whole room). */
static int sc_zero_copy(void)
{
    return pom_dbg_int("sc_copy", 0) != 1;
}

/* Throughput decoder over the whole batch, then the exact decoder over the blocks
 * it refused (malformed input, capacity/lookbehind errors, pathological
 * streams).  Without scratch every block takes the exact decoder.
 * unchecked: the exact decoder follows the unchecked lzo1x_decompress (the
 * fast decoder only ever finishes streams on which both agree). */
static int decompress_dev_with(const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len,
                               uint8_t *dst, const uint64_t *dst_off, const uint32_t *dst_cap,
                               uint32_t *out_len, int32_t *status, uint32_t nblocks, void *scratch,
                               int unchecked, int win, hipStream_t s);

static int decompress_dev(const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len,
                          uint8_t *dst, const uint64_t *dst_off, const uint32_t *dst_cap,
                          uint32_t *out_len, int32_t *status, uint32_t nblocks, void *scratch,
                          int unchecked, hipStream_t s)
{
    return decompress_dev_with(src, src_off, src_len, dst, dst_off, dst_cap, out_len, status,
                               nblocks, scratch, unchecked, use_win_decoder(nblocks), s);
}

static int decompress_dev_with(const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len,
                               uint8_t *dst, const uint64_t *dst_off, const uint32_t *dst_cap,
                               uint32_t *out_len, int32_t *status, uint32_t nblocks, void *scratch,
                               int unchecked, int win, hipStream_t s)
{
    if (nblocks == 0)
        return 0;
    if (!scratch)
        return lzo_mi355x_launch_decompress_exact(src, src_off, src_len, dst, dst_off, dst_cap,
                                                  out_len, status, NULL, NULL, nblocks, nblocks,
                                                  unchecked, s);
    uint8_t *scr = scratch;
    const uint32_t nsets = (uint32_t)scr_sets(nblocks);
    uint32_t *fb = (uint32_t *)scr, *ids = (uint32_t *)(scr + scr_head(nblocks));
    if (win) {
        /* the windowed decoder: no op sets,
         * only the fallback list */
        if (hipMemsetAsync(scr, 0, 256, s) != hipSuccess)
            return -1;
        if (lzo_mi355x_launch_decompress_win(src, src_off, src_len, dst, dst_off, dst_cap, out_len, status, fb,
                                             ids, nblocks, s) != 0)
            return -1;
    } else {
        if (hipMemsetAsync(scr, 0, SCR_RING + 8 * (size_t)nsets, s) != hipSuccess)
            return -1;
        if (lzo_mi355x_launch_decompress_fast(src, src_off, src_len, dst, dst_off, dst_cap,
                                              out_len, status, fb, ids,
                                              (uint32_t *)(scr + SCR_POOL), scr + SCR_RING,
                                              scr + scr_ops_off(nblocks), nsets, nblocks,
                                              scr_order_bytes(nblocks)
                                                  ? (uint32_t *)(scr + scr_order_off(nblocks))
                                                  : NULL,
                                              s) != 0)
            return -1;
    }
    const uint32_t ngrid = nblocks < 512 ? nblocks : 512;
    return lzo_mi355x_launch_decompress_exact(src, src_off, src_len, dst, dst_off, dst_cap,
                                              out_len, status, fb, ids, ngrid, nblocks, unchecked,
                                              s);
}

int lzo_mi355x_decompress_dev(const uint8_t *src, const uint64_t *src_off,
                              const uint32_t *src_len, uint8_t *dst,
                              const uint64_t *dst_off, const uint32_t *dst_cap,
                              uint32_t *out_len, int32_t *status, uint32_t nblocks,
                              void *scratch, void *stream)
{
    return decompress_dev(src, src_off, src_len, dst, dst_off, dst_cap, out_len, status, nblocks,
                          scratch, 0, (hipStream_t)stream);
}

int lzo_mi355x_decompress_fallbacks(const void *scratch, uint32_t *count, void *stream)
{
    /* the fallback count at scratch byte 0, once the stream has reached it */
    if (!scratch || !count)
        return -1;
    hipStream_t s = (hipStream_t)stream;
    if (hipMemcpyAsync(count, scratch, sizeof *count, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -1;
    return 0;
}

int lzo_mi355x_decoded_length_dev(const uint8_t *src, const uint64_t *src_off,
                                  const uint32_t *src_len, uint32_t *out_len,
                                  int32_t *status, uint32_t nblocks, void *stream)
{
    return lzo_mi355x_launch_decoded_length(src, src_off, src_len, out_len, status, nblocks, NULL,
                                            0xFFFFFFFFu, (hipStream_t)stream);
}

/* ------------------------------------------------------------------------ */
/* Host-resident batches: pack -> H2D -> kernels -> D2H -> unpack           */
/* ------------------------------------------------------------------------ */
/* Pack/unpack copies between caller buffers and the pinned staging: split
 * over up to kCopyThreads threads by bytes once a batch is large enough for
 * one memcpy stream to be the bottleneck (the host side of config C5). */
struct copy_job {
    uint8_t *dst;
    const uint8_t *src;
    size_t len;
};

struct copy_range {
    const struct copy_job *jobs;
    size_t lo, hi;
};

enum { kCopyThreads = 8 };
static const size_t kCopyParallelBytes = 8u << 20;

static void *copy_worker(void *arg)
{
    const struct copy_range *r = arg;
    for (size_t i = r->lo; i < r->hi; i++)
        if (r->jobs[i].len)
            memcpy(r->jobs[i].dst, r->jobs[i].src, r->jobs[i].len);
    return NULL;
}

static void copy_jobs(const struct copy_job *jobs, size_t n)
{
    size_t total = 0;
    for (size_t i = 0; i < n; i++)
        total += jobs[i].len;
    struct copy_range r[kCopyThreads];
    pthread_t th[kCopyThreads];
    int nt = total >= kCopyParallelBytes && n > 1 ? kCopyThreads : 1;
    /* contiguous job ranges of about total / nt bytes each */
    size_t i = 0, acc = 0;
    int k = 0;
    for (; k < nt && i < n; k++) {
        r[k].jobs = jobs;
        r[k].lo = i;
        const size_t goal = total / (size_t)nt * (size_t)(k + 1);
        while (i < n && (acc < goal || k == nt - 1)) {
            acc += jobs[i].len;
            i++;
        }
        r[k].hi = i;
    }
    int started = 0;
    for (int j = 1; j < k; j++)
        if (pthread_create(&th[j], NULL, copy_worker, &r[j]) == 0)
            started |= 1 << j;
        else
            copy_worker(&r[j]);
    if (k > 0)
        copy_worker(&r[0]);
    for (int j = 1; j < k; j++)
        if (started & (1 << j))
            pthread_join(th[j], NULL);
}

void pom_copy_parallel(uint8_t *const *dst, const uint8_t *const *src, const size_t *len, size_t n)
{
    struct copy_job *jobs = malloc(n * sizeof(*jobs));
    if (!jobs) {
        for (size_t i = 0; i < n; i++)
            if (len[i])
                memcpy(dst[i], src[i], len[i]);
        return;
    }
    for (size_t i = 0; i < n; i++) {
        jobs[i].dst = dst[i];
        jobs[i].src = src[i];
        jobs[i].len = len[i];
    }
    copy_jobs(jobs, n);
    free(jobs);
}

/* Staging layout of one chunk (identical on host and device, so one copy each
 * way):
 *   [src_off u64][dst_off u64][src_len u32][dst_cap u32][out_len u32][status i32]
 *   [packed offset u64]
 *   [src bytes, 16-B aligned per block][dst bytes, 16-B aligned per block]
 *   [device only: scratch of the kernels the batch runs][device only: packed output]
 * The kernels write each block into its capacity-sized dst slot; only the
 * produced bytes come back, packed (pack kernel), in one D2H copy into the
 * host's dst region.  Block i of the chunk is the caller's block ids[i]. */
struct layout {
    size_t nb;
    const size_t *ids;
    int collected;          /* produced bytes packed and their D2H queued */
    size_t packed;
    size_t o_srcoff, o_dstoff, o_srclen, o_dstcap, o_outlen, o_status, o_poff;
    size_t o_src, o_dst, o_scr, o_pack, htotal, dtotal;
};

static void layout_make(struct layout *L, const size_t *ids, size_t nb, const size_t *src_len,
                        const size_t *dst_cap, int compress)
{
    L->nb = nb;
    L->ids = ids;
    L->collected = 0;
    L->packed = 0;
    size_t o = 0;
    L->o_srcoff = o; o += 8 * nb;
    L->o_dstoff = o; o += 8 * nb;
    L->o_srclen = o; o += 4 * nb;
    L->o_dstcap = o; o += 4 * nb;
    L->o_outlen = o; o += 4 * nb;
    L->o_status = o; o += 4 * nb;
    L->o_poff = o; o += 8 * nb;
    o = ALIGN_UP(o, 256);
    L->o_src = o;
    size_t s = 0, d = 0;
    for (size_t i = 0; i < nb; i++) {
        s += ALIGN_UP(src_len[ids[i]], 16);
        d += ALIGN_UP(dst_cap[ids[i]], 16);
    }
    o += ALIGN_UP(s, 256);
    L->o_dst = o;
    o += ALIGN_UP(d, 256);
    L->htotal = o;
    L->o_scr = o;
    /* scratch of the one kernel family the batch runs */
    o += ALIGN_UP(compress ? lzo_mi355x_compress_scratch((uint32_t)nb)
                           : lzo_mi355x_decompress_scratch((uint32_t)nb), 256);
    L->o_pack = o;
    L->dtotal = o + ALIGN_UP(d, 256);
}

static void layout_fill(const struct layout *L, uint8_t *h, const uint8_t *const *src,
                        const size_t *src_len, const size_t *dst_cap)
{
    uint64_t *so = (uint64_t *)(h + L->o_srcoff);
    uint64_t *dof = (uint64_t *)(h + L->o_dstoff);
    uint32_t *sl = (uint32_t *)(h + L->o_srclen);
    uint32_t *dc = (uint32_t *)(h + L->o_dstcap);
    size_t s = 0, d = 0;
    struct copy_job *jobs = malloc(L->nb * sizeof(*jobs));
    for (size_t i = 0; i < L->nb; i++) {
        const size_t b = L->ids[i];
        so[i] = s;
        dof[i] = d;
        sl[i] = (uint32_t)src_len[b];
        dc[i] = (uint32_t)dst_cap[b];
        if (jobs) {
            jobs[i].dst = h + L->o_src + s;
            jobs[i].src = src[b];
            jobs[i].len = src_len[b];
        } else if (src_len[b]) {
            memcpy(h + L->o_src + s, src[b], src_len[b]);
        }
        s += ALIGN_UP(src_len[b], 16);
        d += ALIGN_UP(dst_cap[b], 16);
    }
    if (jobs) {
        copy_jobs(jobs, L->nb);
        free(jobs);
    }
}

enum op_kind { OP_COMPRESS, OP_DECOMPRESS, OP_CONCAT };

/* One host batch: the caller's arrays, the capacities the kernels use, and
 * the plan (device split, largest-first order). */
struct hbatch {
    enum op_kind kind;
    const uint8_t *const *src;
    const size_t *src_len;
    uint8_t *const *dst;
    size_t *dst_len;
    int *status;
    const size_t *cap;
    const size_t *cost;
    size_t budget;
    struct pom_plan plan;
    const int *devs;        /* plan device d runs on HIP device devs[d] */
    struct tctx *t;
    uint32_t enc_lds_max;   /* chunks of at most this many blocks: LDS dictionaries */
    int nslots;             /* chunks in flight per device (<= kSlots) */
    int ooo;                /* deliver chunks in completion order (compress batches) */
    pom_chunk_fn on_chunk;  /* called with each delivered chunk's block ids, or NULL */
    pom_chunk_fn pre_chunk; /* called with a chunk's block ids before its inputs are staged */
    void *cb_ctx;
};

/* debug key host_timing=1: per-batch and per-chunk wall times on stderr (diagnostic) */
#define g_timing (pom_dbg_int("host_timing", 0) == 1)

static double now_ms(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

/* The latency decoder's scratch: ONE buffer per device, shared by every
 * thread's host-batch chunks and combined single-call groups (ADVICE round
 * 3: per-thread, per-slot buffers of up to 1 GiB each pinned GBs of HBM).
 * A user holds the mutex while it launches, waits (on the GPU, through the
 * event) for the previous use's kernels, and records its own.  Groups needing
 * more than kLatMaxScratch (from ~1 MB of compressed input) take the windowed
 * decoder. */
static const size_t kLatMaxScratch = (size_t)256 << 20;
struct lat_scratch {
    pthread_mutex_t mu;
    void *buf;
    size_t cap;
    hipEvent_t done;            /* the last use's kernels (created with the buffer) */
};
static struct lat_scratch lat_s[kMaxDev];
static pthread_once_t lat_once = PTHREAD_ONCE_INIT;

static void lat_init(void)
{
    for (int d = 0; d < kMaxDev; d++)
        pthread_mutex_init(&lat_s[d].mu, NULL);
}

/* The device's scratch, at least `bytes`, locked, with stream s ordered
 * after its last use; NULL (unlocked) if the device or memory is missing. */
static struct lat_scratch *lat_acquire(size_t bytes, hipStream_t s)
{
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev || bytes > kLatMaxScratch)
        return NULL;
    pthread_once(&lat_once, lat_init);
    struct lat_scratch *L = &lat_s[dev];
    pthread_mutex_lock(&L->mu);
    if (!L->done && hipEventCreateWithFlags(&L->done, hipEventDisableTiming) != hipSuccess) {
        L->done = NULL;
        pthread_mutex_unlock(&L->mu);
        return NULL;
    }
    if (L->cap < bytes) {
        hipEventSynchronize(L->done);           /* (a never-recorded event is complete) */
        if (L->buf)
            hipFree(L->buf);
        L->buf = NULL;
        L->cap = 0;
        size_t want = ALIGN_UP(bytes + bytes / 4, (size_t)1 << 20);
        want = want < kLatMaxScratch ? want : kLatMaxScratch;
        if (hipMalloc(&L->buf, want) != hipSuccess) {
            L->buf = NULL;
            pthread_mutex_unlock(&L->mu);
            return NULL;
        }
        L->cap = want;
    }
    if (hipStreamWaitEvent(s, L->done, 0) != hipSuccess) {
        pthread_mutex_unlock(&L->mu);
        return NULL;
    }
    return L;
}

static void lat_release(struct lat_scratch *L, hipStream_t s)
{
    hipEventRecord(L->done, s);
    pthread_mutex_unlock(&L->mu);
}

static int use_lat_decoder(size_t z);

/* A decompress chunk of at most 8 blocks, each of at least sc_lat_min (debug key, default 2048)
 * compressed bytes, decodes on one latency-decoder pipeline (the whole GPU on
 * these few blocks; lzo1x_decode_lat.hip) with the exact decoder behind it for
 * the blocks it hands over.  1 launched, 0 not eligible (nothing launched),
 * -1 on an error. */
static int lat_chunk(struct slot *S, const struct layout *L, const uint8_t *h, uint8_t *d, hipStream_t s)
{
    const uint32_t nb = (uint32_t)L->nb;
    if (nb == 0 || nb > 8)
        return 0;
    const uint64_t *so = (const uint64_t *)(h + L->o_srcoff);
    const uint64_t *dof = (const uint64_t *)(h + L->o_dstoff);
    const uint32_t *sl = (const uint32_t *)(h + L->o_srclen);
    const uint32_t *dc = (const uint32_t *)(h + L->o_dstcap);
    for (uint32_t i = 0; i < nb; i++)
        if (!use_lat_decoder(sl[i]))
            return 0;
    (void)S;
    const size_t need = lzo_mi355x_decompress_lat_scratch_n(so, sl, dc, nb);
    if (need == 0 || need > kLatMaxScratch)
        return 0;
    uint8_t *scr = d + L->o_scr;
    uint32_t *fb = (uint32_t *)scr, *ids = (uint32_t *)(scr + scr_head(nb));
    uint32_t *ol = (uint32_t *)(d + L->o_outlen);
    int32_t *st = (int32_t *)(d + L->o_status);
    if (hipMemsetAsync(scr, 0, 256, s) != hipSuccess)
        return -1;
    struct lat_scratch *LS = lat_acquire(need, s);
    if (!LS)
        return 0;                               /* (the chunk's usual decoders) */
    const int lrc = lzo_mi355x_launch_decompress_lat_n(d + L->o_src, so, sl, d + L->o_dst, dof, dc, nb, ol, st,
                                                       fb, ids, 0, LS->buf, LS->cap, s);
    lat_release(LS, s);
    if (lrc != 0 ||
        lzo_mi355x_launch_decompress_exact(d + L->o_src, (const uint64_t *)(d + L->o_srcoff),
                                           (const uint32_t *)(d + L->o_srclen), d + L->o_dst,
                                           (const uint64_t *)(d + L->o_dstoff), (const uint32_t *)(d + L->o_dstcap),
                                           ol, st, fb, ids, nb, nb, 0, s) != 0)
        return -1;
    return 1;
}

/* Chunk on slot S: inputs into pinned staging, H2D, kernels, D2H of the
 * lengths -- all queued on the slot's stream, nothing waited for. */
static int chunk_launch(struct slot *S, struct layout *L, const struct hbatch *B)
{
    if (slot_reserve(S, L->dtotal, L->htotal) != 0)
        return -1;
    uint8_t *d = S->dmem, *h = S->hmem;
    hipStream_t s = S->stream;
    const uint32_t nb = (uint32_t)L->nb;
    const double t0 = g_timing ? now_ms() : 0;
    layout_fill(L, h, B->src, B->src_len, B->cap);
    if (g_timing)
        fprintf(stderr, "  chunk n=%u: fill %.2f ms (%zu B)\n", nb, now_ms() - t0, L->htotal);
    if (hipMemcpyAsync(d, h, L->o_dst, hipMemcpyHostToDevice, s) != hipSuccess)
        return -1;
    const uint8_t *dsrc = d + L->o_src;
    uint8_t *ddst = d + L->o_dst;
    const uint64_t *so = (const uint64_t *)(d + L->o_srcoff);
    const uint64_t *dof = (const uint64_t *)(d + L->o_dstoff);
    const uint32_t *sl = (const uint32_t *)(d + L->o_srclen);
    const uint32_t *dc = (const uint32_t *)(d + L->o_dstcap);
    uint32_t *ol = (uint32_t *)(d + L->o_outlen);
    int32_t *st = (int32_t *)(d + L->o_status);
    int rc;
    if (B->kind == OP_COMPRESS) {
        /* lzo_mi355x_compress_dev, with the general encoder's pass only when a
         * block of the chunk needs it: that kernel's workgroups take 64 KB of
         * LDS each, and behind the other slots' encoders a pass with nothing to
         * do waited ~0.75 ms for LDS to free up (C5 trace) */
        void *scr = nb <= B->enc_lds_max ? NULL : d + L->o_scr;
        int big = 0;
        for (size_t i = 0; i < L->nb; i++)
            big |= B->src_len[L->ids[i]] > LZO_MI355X_FAST_MAX_N;
        rc = lzo_mi355x_launch_compress_fast(dsrc, so, sl, ddst, dof, dc, ol, st, nb, scr,
                                             scr ? lzo_mi355x_compress_scratch(nb) : 0, s);
        if (rc == 0 && big)
            rc = lzo_mi355x_launch_compress(dsrc, so, sl, ddst, dof, dc, ol, st, nb, 1, s);
    }
    else if (B->kind == OP_DECOMPRESS) {
        const int lat = lat_chunk(S, L, h, d, s);
        rc = lat < 0 ? -1 : lat > 0 ? 0 : decompress_dev(dsrc, so, sl, ddst, dof, dc, ol, st, nb, d + L->o_scr, 0, s);
    }
    else
        rc = lzo_mi355x_launch_decompress_concat(dsrc, so, sl, ddst, dof, dc, ol, st, nb, s);
    if (rc != 0)
        return -1;
    return hipMemcpyAsync(h + L->o_outlen, d + L->o_outlen, 8 * L->nb, hipMemcpyDeviceToHost, s) ==
                   hipSuccess ? 0 : -1;
}

/* Once the chunk's kernels are done (waited for, or with `poll` only if they
 * already are), queues the pack kernel and the D2H of exactly the produced
 * bytes.  Returns 1 when queued, 0 when polling found the kernels running,
 * -1 on an error. */
static int chunk_collect(struct slot *S, struct layout *L, int poll)
{
    if (L->collected)
        return 1;
    uint8_t *d = S->dmem, *h = S->hmem;
    hipStream_t s = S->stream;
    if (poll) {
        const hipError_t q = hipStreamQuery(s);
        if (q == hipErrorNotReady)
            return 0;
        if (q != hipSuccess)
            return -1;
    } else if (hipStreamSynchronize(s) != hipSuccess) {
        return -1;
    }
    const uint32_t *hol = (const uint32_t *)(h + L->o_outlen);
    const uint32_t *hdc = (const uint32_t *)(h + L->o_dstcap);
    uint64_t *poff = (uint64_t *)(h + L->o_poff);
    size_t packed = 0;
    for (size_t i = 0; i < L->nb; i++) {
        poff[i] = packed;
        packed += ALIGN_UP((size_t)(hol[i] < hdc[i] ? hol[i] : hdc[i]), 16);
    }
    if (packed &&
        (hipMemcpyAsync(d + L->o_poff, poff, 8 * L->nb, hipMemcpyHostToDevice, s) != hipSuccess ||
         lzo_mi355x_launch_pack(d + L->o_dst, (const uint64_t *)(d + L->o_dstoff),
                                (const uint32_t *)(d + L->o_outlen),
                                (const uint32_t *)(d + L->o_dstcap),
                                (const uint64_t *)(d + L->o_poff), d + L->o_pack,
                                (uint32_t)L->nb, s) != 0 ||
         hipMemcpyAsync(h + L->o_dst, d + L->o_pack, packed, hipMemcpyDeviceToHost, s) !=
             hipSuccess))
        return -1;
    L->packed = packed;
    L->collected = 1;
    return 1;
}

/* Waits for the chunk's produced bytes and hands lengths, codes and bytes to
 * the caller's arrays.  The next chunk (nS/nL, may be NULL) is collected
 * first (its kernels waited for, its D2H queued), so that its copy runs
 * while this one is unpacked.  (Polling it with hipStreamQuery instead never
 * found it done here.) */
static int chunk_deliver(struct slot *S, struct layout *L, const struct hbatch *B,
                         struct slot *nS, struct layout *nL)
{
    const double t0 = g_timing ? now_ms() : 0;
    if (chunk_collect(S, L, 0) < 0 || hipStreamSynchronize(S->stream) != hipSuccess)
        return -1;
    if (nS && chunk_collect(nS, nL, 0) < 0)
        return -1;
    const double t1 = g_timing ? now_ms() : 0;
    const uint8_t *h = S->hmem;
    const uint32_t *hol = (const uint32_t *)(h + L->o_outlen);
    const int32_t *hst = (const int32_t *)(h + L->o_status);
    const uint64_t *poff = (const uint64_t *)(h + L->o_poff);
    struct copy_job *jobs = malloc(L->nb * sizeof(*jobs));
    for (size_t i = 0; i < L->nb; i++) {
        const size_t b = L->ids[i];
        const size_t n = hol[i] < B->cap[b] ? hol[i] : B->cap[b];
        if (jobs) {
            jobs[i].dst = B->dst[b];
            jobs[i].src = h + L->o_dst + poff[i];
            jobs[i].len = n;
        } else if (n) {
            memcpy(B->dst[b], h + L->o_dst + poff[i], n);
        }
        B->dst_len[b] = hol[i];
        B->status[b] = hst[i];
    }
    if (jobs) {
        copy_jobs(jobs, L->nb);
        free(jobs);
    }
    if (g_timing)
        fprintf(stderr, "  deliver n=%zu: wait %.2f (%zu B) unpack %.2f ms\n", L->nb, t1 - t0,
                L->packed, now_ms() - t1);
    return 0;
}

/* A host batch is cut into chunks of at most kChunkBudget bytes of input plus
 * output capacity (a larger block is a chunk of its own), pipelined through
 * the device's kSlots slots: chunk k is staged and its copies and kernels are
 * queued as soon as chunk k - kSlots has been waited for and unpacked, so the
 * copies, the kernels of several chunks and the host-side packing overlap.
 * The first chunk gets a quarter of the budget: for compress batches it holds
 * the largest blocks, whose long serial LZ chains start while the rest of the
 * batch is still being copied up; decode batches go smallest first (dev_run).  Debug key chunk_mb overrides the budget. */
static const size_t kChunkBudget = (size_t)128 << 20;
/* compress batches: their chains are long (a 536 KB ITB is ~6 ms on one CU),
 * so their chunks are delivered in completion order (hbatch.ooo): a chunk of
 * smaller blocks that finishes while the largest blocks' chunk still runs
 * frees its slot for the next chunk and is handed to on_chunk (the append
 * file) at once.  In launch order, 128 MiB chunks left the slots waiting on
 * the first chunk (C5 compress 13.4-14.7 against 16.4-17.7 GiB/s with 256
 * MiB); in completion order they compress as fast and the fused write gains
 * (profiles/r04e/c5_ooo/) */
static const size_t kChunkBudgetCompress = (size_t)128 << 20;
static const size_t kChunkBlocks = (size_t)1 << 20;
/* below this many bytes per device a batch stays on one device */
static const size_t kSplitMinBytes = (size_t)64 << 20;

/* Completion order (compress batches, hbatch.ooo): the first live slot whose
 * stream is done, polling every 20 us; a failed stream counts as done (its
 * delivery reports the error). */
static int wait_any_done(struct dctx *c, const int *live, int nslots)
{
    for (;;) {
        for (int i = 0; i < nslots; i++)
            if (live[i] && hipStreamQuery(c->s[i].stream) != hipErrorNotReady)
                return i;
        const struct timespec ts = {0, 20000};
        nanosleep(&ts, NULL);
    }
}

static int dev_run(void *arg, int d)
{
    const struct hbatch *B = arg;
    const int device = B->devs[d];
    int prev_dev = -1;
    if (hipGetDevice(&prev_dev) != hipSuccess)
        return -1;
    if (prev_dev != device && hipSetDevice(device) != hipSuccess)
        return -1;
    int rc = 0;
    struct dctx *c = dctx_get(B->t, device);
    if (!c) {
        rc = -1;
    } else {
        const size_t *ids = B->plan.by_dev + B->plan.dev_off[d];
        const size_t nids = B->plan.dev_off[d + 1] - B->plan.dev_off[d];
        /* decode batches go smallest first: a decoded chunk's D2H copy is the
         * long pole (PCIe), and the first chunk's kernels -- the smallest
         * blocks -- finish early, so the copies start early and run back to
         * back while the chunks of the largest blocks decode (debug key
         * dec_small_first=0: largest first, as compress batches) */
        size_t *rev = NULL;
        if (B->kind != OP_COMPRESS && nids > 1 && pom_dbg_int("dec_small_first", 1) != 0 &&
            (rev = malloc(nids * sizeof(*rev))) != NULL) {
            for (size_t i = 0; i < nids; i++)
                rev[i] = ids[nids - 1 - i];
            ids = rev;
        }
        struct layout L[kSlots];
        int live[kSlots] = {0};                /* slot holds a launched chunk */
        size_t from = 0;
        /* (tests: debug key fail_chunk=K makes this device's K-th delivery fail
         * as a failed GPU stream would) */
        const long fail_at = pom_dbg_int("fail_chunk", -1);
        long ndeliv = 0;
        for (int k = 0;; k++) {
            int cur = k % B->nslots;
            const int nxt = (k + 1) % B->nslots;
            const size_t *done_ids = NULL;     /* the chunk delivered now, for on_chunk */
            size_t done_nb = 0;
            int dj = -1;                       /* slot to deliver now, if any */
            if (!B->ooo) {
                if (live[cur])                 /* chunk k - nslots: wait, unpack */
                    dj = cur;
            } else {
                /* completion order: launch into a free slot; when there is
                 * none, or nothing is left to launch, deliver whichever chunk
                 * finishes first */
                cur = -1;
                for (int j = 0; j < B->nslots && cur < 0; j++)
                    if (!live[j])
                        cur = j;
                int any = 0;
                for (int j = 0; j < B->nslots; j++)
                    any |= live[j];
                if (any && (cur < 0 || from >= nids || rc != 0))
                    dj = wait_any_done(c, live, B->nslots);
            }
            if (dj >= 0) {
                const int ahead = !B->ooo && live[nxt] && nxt != dj;
                const int fail = fail_at >= 0 && ndeliv++ == fail_at;
                if (fail || chunk_deliver(&c->s[dj], &L[dj], B, ahead ? &c->s[nxt] : NULL, &L[nxt]) != 0) {
                    rc = -1;
                    for (int j = 0; j < B->nslots; j++)
                        hipStreamSynchronize(c->s[j].stream);
                } else {
                    done_ids = L[dj].ids;      /* (points into the plan, not the layout) */
                    done_nb = L[dj].nb;
                }
                live[dj] = 0;
                if (cur < 0)
                    cur = dj;
            }
            const int more = from < nids && rc == 0 && cur >= 0;
            if (more) {
                const size_t end = pom_chunk_end(ids, from, nids, B->cost,
                                                 k ? B->budget : B->budget / 4, kChunkBlocks);
                layout_make(&L[cur], ids + from, end - from, B->src_len, B->cap,
                            B->kind == OP_COMPRESS);
                /* the caller may produce the chunk's inputs now (e.g. read them),
                 * while the chunks in flight are copied and decoded */
                if (B->pre_chunk)
                    B->pre_chunk(B->cb_ctx, ids + from, end - from);
                if (chunk_launch(&c->s[cur], &L[cur], B) != 0) {
                    rc = -1;
                    hipStreamSynchronize(c->s[cur].stream);
                } else {
                    live[cur] = 1;
                }
                from = end;
            }
            /* the caller's per-chunk work runs while the launched chunks' copies
             * and kernels are in flight */
            if (done_ids && B->on_chunk) {
                const double tc = g_timing ? now_ms() : 0;
                B->on_chunk(B->cb_ctx, done_ids, done_nb);
                if (g_timing)
                    fprintf(stderr, "  on_chunk n=%zu: %.2f ms\n", done_nb, now_ms() - tc);
            }
            if (!(from < nids && rc == 0)) {
                int any = 0;
                for (int j = 0; j < B->nslots; j++)
                    any |= live[j];
                if (!any)
                    break;
            }
        }
        free(rev);
    }
    if (prev_dev != device)
        hipSetDevice(prev_dev);
    return rc;
}

/* Devices a host batch may use: POM_LZO_DEVICES ("0,2,3"; default every
 * visible device; parsed by pom_parse_devices, duplicates dropped).
 * Processes that run one rank per GPU set it to their own. */
static int batch_devices(int *devs)
{
    const int count = lzo_mi355x_device_count();
    int n = 0;
    const char *e = getenv("POM_LZO_DEVICES");
    if (e && *e) {
        n = pom_parse_devices(e, count, kMaxDev, devs);
    } else {
        for (int d = 0; d < count && d < kMaxDev; d++)
            devs[n++] = d;
    }
    /* the caller's current device first: a one-device batch runs there */
    int cur = -1;
    if (n > 1 && hipGetDevice(&cur) == hipSuccess)
        for (int i = 1; i < n; i++)
            if (devs[i] == cur) {
                devs[i] = devs[0];
                devs[0] = cur;
                break;
            }
    return n;
}

static int batch_common_cb(enum op_kind kind, const uint8_t *const *src, const size_t *src_len,
                           uint8_t *const *dst, size_t *dst_len, int *status, size_t nblocks,
                           pom_chunk_fn on_chunk, pom_chunk_fn pre_chunk, void *cb_ctx);

static int batch_common(enum op_kind kind, const uint8_t *const *src, const size_t *src_len,
                        uint8_t *const *dst, size_t *dst_len, int *status, size_t nblocks)
{
    return batch_common_cb(kind, src, src_len, dst, dst_len, status, nblocks, NULL, NULL, NULL);
}

/* lzo_mi355x_decompress_batch with pre_chunk(ctx, ids, nb) called before each
 * chunk's inputs are staged: the caller fills src[ids[i]] (src_len is known
 * up front) while earlier chunks are on the GPU.  Same threads as
 * pom_compress_batch_chunked. */
int pom_decompress_batch_chunked(const uint8_t *const *src, const size_t *src_len, uint8_t *const *dst,
                                 size_t *dst_len, int *status, size_t nblocks, pom_chunk_fn pre_chunk,
                                 void *ctx)
{
    return batch_common_cb(OP_DECOMPRESS, src, src_len, dst, dst_len, status, nblocks, NULL, pre_chunk, ctx);
}

/* lzo_mi355x_compress_batch with on_chunk(ctx, ids, nb) called as each chunk's
 * blocks (ids into the caller's arrays) are delivered -- from the thread
 * running that device's chunks, so concurrently for batches split over
 * several GPUs. */
int pom_compress_batch_chunked(const uint8_t *const *src, const size_t *src_len, uint8_t *const *dst,
                               size_t *dst_len, int *status, size_t nblocks, pom_chunk_fn on_chunk,
                               void *ctx)
{
    return batch_common_cb(OP_COMPRESS, src, src_len, dst, dst_len, status, nblocks, on_chunk, NULL, ctx);
}

static int batch_common_cb(enum op_kind kind, const uint8_t *const *src, const size_t *src_len,
                           uint8_t *const *dst, size_t *dst_len, int *status, size_t nblocks,
                           pom_chunk_fn on_chunk, pom_chunk_fn pre_chunk, void *cb_ctx)
{
    const double t0 = g_timing ? now_ms() : 0;
    struct tctx *t = tctx_get();
    if (!t)
        return LZO_E_ERROR;
    if (nblocks == 0)
        return LZO_E_OK;
    if (nblocks > 0xFFFFFFFFu)
        return LZO_E_ERROR;
    int devs[kMaxDev];
    const int ndev = batch_devices(devs);
    if (ndev <= 0)
        return LZO_E_ERROR;
    size_t *cap = malloc(nblocks * sizeof(size_t));
    size_t *cost = malloc(nblocks * sizeof(size_t));
    if (!cap || !cost) {
        free(cap);
        free(cost);
        return LZO_E_OUT_OF_MEMORY;
    }
    for (size_t b = 0; b < nblocks; b++) {
        if (src_len[b] > 0xFFFFFFF0u) {
            free(cap);
            free(cost);
            return LZO_E_ERROR;
        }
        cap[b] = kind == OP_COMPRESS ? lzo_mi355x_worst_compress(src_len[b]) : dst_len[b];
        if (cap[b] > 0xFFFFFFF0u)
            cap[b] = 0xFFFFFFF0u;
        cost[b] = src_len[b] + cap[b];
    }
    struct hbatch B = {kind, src, src_len, dst, dst_len, status, cap, cost,
                       kind == OP_COMPRESS ? kChunkBudgetCompress : kChunkBudget,
                       {0, 1, NULL, NULL}, devs, t, 0, kSlots, 0, on_chunk, pre_chunk, cb_ctx};
    B.ooo = kind == OP_COMPRESS && pom_dbg_int("ooo", 1) != 0;
    /* compress chunks that fit the LDS encoder's 4 blocks per CU at once use
     * it: a block alone on its CU finishes twice as fast as with the
     * dictionaries in HBM (that encoder wins only on full GPUs: 16 per CU) */
    B.enc_lds_max = (uint32_t)pom_dbg_int("enc_lds_max", (long)(lzo_mi355x_fast_resident_blocks() / 4));
    const long ns = pom_dbg_int("slots", kSlots);
    if (ns >= 1 && ns <= kSlots)
        B.nslots = (int)ns;
    const long mb = pom_dbg_int("chunk_mb", 0);
    if (mb > 0)
        B.budget = (size_t)mb << 20;
    int rc = LZO_E_OUT_OF_MEMORY;
    if (pom_plan_make(&B.plan, nblocks, cost, ndev, kSplitMinBytes) == 0) {
        /* blocks a failed device leaves untouched read as errors */
        for (size_t b = 0; b < nblocks; b++) {
            status[b] = LZO_E_ERROR;
            dst_len[b] = 0;
        }
        rc = pom_run_devices(B.plan.ndev, dev_run, &B) == 0 ? LZO_E_OK : LZO_E_ERROR;
        if (g_timing)
            fprintf(stderr, "pom host %s n=%zu devices=%d: %.2f ms\n",
                    kind == OP_COMPRESS ? "compress" : "decompress", nblocks, B.plan.ndev,
                    now_ms() - t0);
        pom_plan_free(&B.plan);
    }
    free(cap);
    free(cost);
    return rc;
}

int lzo_mi355x_compress_batch(const uint8_t *const *src, const size_t *src_len,
                              uint8_t *const *dst, size_t *dst_len, int *status,
                              size_t nblocks)
{
    return batch_common(OP_COMPRESS, src, src_len, dst, dst_len, status, nblocks);
}

int lzo_mi355x_decompress_batch(const uint8_t *const *src, const size_t *src_len,
                                uint8_t *const *dst, size_t *dst_len, int *status,
                                size_t nblocks)
{
    return batch_common(OP_DECOMPRESS, src, src_len, dst, dst_len, status, nblocks);
}

int lzo_mi355x_decompress_concat_batch(const uint8_t *const *src, const size_t *src_len,
                                       uint8_t *const *dst, size_t *dst_len, int *status,
                                       size_t nblocks)
{
    return batch_common(OP_CONCAT, src, src_len, dst, dst_len, status, nblocks);
}

/* ------------------------------------------------------------------------ */
/* minilzo.h call surface                                                   */
/* ------------------------------------------------------------------------ */

/* lib/minilzo.c:2567-2598: a zero version or a type-size mismatch is
 * LZO_E_ERROR; additionally the GPU must be usable. */
int __lzo_init_v2(unsigned v, int s1, int s2, int s3, int s4, int s5, int s6, int s7, int s8,
                  int s9)
{
    if (v == 0)
        return LZO_E_ERROR;
    int ok = (s1 == -1 || s1 == (int)sizeof(short)) && (s2 == -1 || s2 == (int)sizeof(int)) &&
             (s3 == -1 || s3 == (int)sizeof(long)) &&
             (s4 == -1 || s4 == (int)sizeof(lzo_uint32)) &&
             (s5 == -1 || s5 == (int)sizeof(lzo_uint)) &&
             (s6 == -1 || s6 == (int)lzo_sizeof_dict_t) &&
             (s7 == -1 || s7 == (int)sizeof(char *)) &&
             (s8 == -1 || s8 == (int)sizeof(lzo_voidp)) &&
             (s9 == -1 || s9 == (int)sizeof(lzo_callback_t));
    if (!ok)
        return LZO_E_ERROR;
    return lzo_mi355x_device_count() > 0 ? LZO_E_OK : LZO_E_ERROR;
}

unsigned lzo_version(void) { return LZO_VERSION; }
const char *lzo_version_string(void) { return LZO_VERSION_STRING; }
const char *lzo_version_date(void) { return LZO_VERSION_DATE; }
lzo_charp _lzo_version_string(void) { return (lzo_charp)LZO_VERSION_STRING; }
lzo_charp _lzo_version_date(void) { return (lzo_charp)LZO_VERSION_DATE; }
/* lib/minilzo.c:2306-2314 (minilzo builds return LZO_VERSION_STRING) */
lzo_bytep lzo_copyright(void) { return (lzo_bytep)LZO_VERSION_STRING; }

/* Host utilities of the reference's minilzo.c (lib/minilzo.c:2355-2500). */
int lzo_memcmp(const lzo_voidp a, const lzo_voidp b, lzo_uint len) { return memcmp(a, b, len); }
lzo_voidp lzo_memcpy(lzo_voidp dst, const lzo_voidp src, lzo_uint len) { return memcpy(dst, src, len); }
lzo_voidp lzo_memmove(lzo_voidp dst, const lzo_voidp src, lzo_uint len) { return memmove(dst, src, len); }
lzo_voidp lzo_memset(lzo_voidp buf, int c, lzo_uint len) { return memset(buf, c, len); }

lzo_uint32 lzo_adler32(lzo_uint32 c, const lzo_bytep buf, lzo_uint len)
{
    if (buf == NULL)
        return 1;
    uint32_t lo = c & 0xffffu, hi = (c >> 16) & 0xffffu;
    const unsigned char *p = buf;
    while (len > 0) {
        /* 5552 bytes keep both sums below 2^32 before the reduction */
        lzo_uint k = len < 5552 ? len : 5552;
        len -= k;
        for (lzo_uint i = 0; i < k; i++) {
            lo += p[i];
            hi += lo;
        }
        p += k;
        lo %= 65521u;
        hi %= 65521u;
    }
    return (hi << 16) | lo;
}

int _lzo_config_check(void)
{
    union {
        unsigned long a[2];
        unsigned char b[2 * sizeof(unsigned long)];
    } u;
    u.a[0] = u.a[1] = 0;
    u.b[0] = 128;
    lzo_uint v;
    memcpy(&v, u.b, sizeof v);
    return v == 128 ? LZO_E_OK : LZO_E_ERROR;       /* little-endian, as the codec assumes */
}

lzo_uintptr_t __lzo_ptr_linear(const lzo_voidp ptr) { return (lzo_uintptr_t)ptr; }

unsigned __lzo_align_gap(const lzo_voidp p, lzo_uint size)
{
    const lzo_uintptr_t a = (lzo_uintptr_t)p;
    return size ? (unsigned)(((a + size - 1) / size) * size - a) : 0u;
}

/* ---- single calls ------------------------------------------------------------
 * The minilzo.h entry points code one block per call, synchronously.  Calls
 * that arrive together from several threads on the same GPU (the MDS commit
 * threads, mds/txg.c:1010-1011, and the service threads that load ITBs,
 * mds/itb.c:2964) are COMBINED: the first caller becomes the leader and runs
 * every call queued behind it (of the same kind, up to kScGroup) as one
 * launch on its own stream; the others sleep until their result is in their
 * buffer.  A lone call is a group of one.  Debug key sc_combine=0 turns combining
 * off (every call its own launch, as in round 2).
 * Staging of a group of k calls (device and pinned host alike):
 *   [0, H)          header arrays: src_off u64[k], dst_off u64[k], src_len[k],
 *                   dst_cap[k], out_len[k], status[k], pre-scan length[k] and
 *                   status[k], the decoder's fallback list (count + k ids)
 *   [H, I)          the inputs, 256-byte aligned
 *   [I, J)          the outputs (each: worst case, the caller's capacity or a
 *                   guess); with zero copy they are written to the host side only
 * One H2D copy ([0, I)), one kernel, one synchronisation: the windowed decoder
 * refuses few valid streams, so the exact decoder runs only when a status says
 * a block was handed over.
 */
enum { kScGroup = 64 };
static const size_t kScGroupBytes = (size_t)256 << 20;

enum sc_kind { SC_COMPRESS, SC_SAFE, SC_UNCHECKED };

struct sc_req {
    enum sc_kind kind;
    const uint8_t *src;
    size_t src_len;
    uint8_t *dst;
    size_t room;
    size_t produced;
    int rc;
    int done;
    uint64_t group;             /* sequence number of the group that ran it */
    struct sc_req *next;
};

struct sc_queue {
    pthread_mutex_t mu;
    pthread_cond_t cv;
    struct sc_req *head, *tail;
    int leader;
    int last_k;                 /* size of the last group (a hint that callers come together) */
    uint64_t seq;               /* groups run so far */
    int ready;                  /* slot and stream below created */
    struct slot slot;           /* the groups' staging: one leader at a time per device */
};

static struct sc_queue sc_q[kMaxDev];
static __thread uint64_t sc_last_group[kMaxDev];   /* per device: group of this thread's last single call */
static pthread_once_t sc_once = PTHREAD_ONCE_INIT;

static void sc_init(void)
{
    for (int d = 0; d < kMaxDev; d++) {
        pthread_mutex_init(&sc_q[d].mu, NULL);
        /* the leader's ~50 us wait for company is a relative time: measure
         * it on CLOCK_MONOTONIC, which wall-clock adjustments do not move */
        pthread_condattr_t ca;
        pthread_condattr_init(&ca);
        pthread_condattr_setclock(&ca, CLOCK_MONOTONIC);
        pthread_cond_init(&sc_q[d].cv, &ca);
        pthread_condattr_destroy(&ca);
    }
}

static int sc_combine(void)
{
    return pom_dbg_int("sc_combine", 1) != 0;
}

/* header arrays of a group of k */
struct sc_hdr {
    uint64_t *src_off, *dst_off;
    uint32_t *src_len, *dst_cap, *out_len;
    int32_t *status;
    uint32_t *plen;
    int32_t *pstatus;
    uint32_t *fb;               /* the decoder's fallback list: count, then k ids */
};

static size_t sc_hdr_bytes(int k)
{
    return ALIGN_UP((size_t)k * 44 + 4, 256);
}

static struct sc_hdr sc_hdr_at(uint8_t *base, int k)
{
    struct sc_hdr x;
    x.src_off = (uint64_t *)base;
    x.dst_off = x.src_off + k;
    x.src_len = (uint32_t *)(x.dst_off + k);
    x.dst_cap = x.src_len + k;
    x.out_len = x.dst_cap + k;
    x.status = (int32_t *)(x.out_len + k);
    x.plen = (uint32_t *)(x.status + k);
    x.pstatus = (int32_t *)(x.plen + k);
    x.fb = (uint32_t *)(x.pstatus + k);
    return x;
}

/* One launch for the k calls g[0..k) (all of one kind) on the calling thread's
 * slot: fills each call's rc and produced length and copies its output. */
/* The staging of combined groups on the calling thread's device: the leader
 * flag gives one group at a time per device, so one slot serves every thread
 * (per-thread slots each grew to the groups their thread happened to lead,
 * and every regrowth is a hipMalloc / hipHostMalloc). */
static struct slot *sc_slot(struct sc_queue *q)
{
    if (!q)
        return single_slot();
    if (!q->ready) {
        if (hipStreamCreateWithFlags(&q->slot.stream, hipStreamNonBlocking) != hipSuccess)
            return NULL;
        q->ready = 1;
    }
    return &q->slot;
}

/* A decode whose compressed block is at least this long takes the latency
 * decoder (lzo1x_decode_lat.hip: the whole GPU on one block, 0.11-0.14 ms from
 * 32 KiB up to 536 KB, where the windowed decoder's one workgroup takes
 * 0.14-2.2 ms); shorter ones (equal at 12 KB) the windowed decoder, and so
 * does a combined group with any such call or more than 8 calls (see
 * lat_group).  Debug keys: sc_lat_min sets the threshold (bytes of compressed
 * input), sc_lat=0 turns it off. */
static int use_lat_decoder(size_t z)
{
    const long min_z = pom_dbg_int("sc_lat", 1) == 0 ? 0x7FFFFFFFL : pom_dbg_int("sc_lat_min", 2048L);
    return z >= (size_t)(min_z > 0 ? min_z : 2048L);
}


/* A group of k <= 8 decodes of at least sc_lat_min compressed bytes each
 * runs as ONE latency-decoder pipeline (lzo1x_decode_lat.hip: the blocks side
 * by side in every kernel).  Returns 1 when launched, 0 when the group does
 * not qualify (nothing launched), -1 on a launch error.  (Separate pipelines
 * on four streams were measured first: they did not overlap -- three 64 KiB
 * blocks 0.38 ms against 0.19 for one.) */
enum { kLatGroup = 8 };

static int lat_group(struct slot *t, struct sc_req **g, int k, const uint8_t *d, uint8_t *out,
                     const size_t *o_src, const size_t *o_out, uint32_t *olen, int32_t *ost, uint32_t *fb,
                     hipStream_t s)
{
    if (k > kLatGroup)
        return 0;
    uint64_t so[kLatGroup], doff[kLatGroup];
    uint32_t z[kLatGroup], cap[kLatGroup];
    for (int i = 0; i < k; i++) {
        if (!use_lat_decoder(g[i]->src_len) || g[i]->room > 0xFFFFFFFFu)
            return 0;
        so[i] = o_src[i];
        doff[i] = o_out[i];
        z[i] = (uint32_t)g[i]->src_len;
        cap[i] = (uint32_t)g[i]->room;
    }
    (void)t;
    const size_t need = lzo_mi355x_decompress_lat_scratch_n(so, z, cap, (uint32_t)k);
    if (need == 0 || need > kLatMaxScratch)
        return 0;                               /* out of its range: the windowed decoder */
    struct lat_scratch *LS = lat_acquire(need, s);
    if (!LS)
        return 0;
    const int rc = lzo_mi355x_launch_decompress_lat_n(d, so, z, out, doff, cap, (uint32_t)k, olen, ost, fb, fb + 1,
                                                      0, LS->buf, LS->cap, s);
    lat_release(LS, s);
    return rc == 0 ? 1 : -1;
}

static void sc_run_group(struct sc_req **g, int k, struct sc_queue *q)
{
    const enum sc_kind kind = g[0]->kind;
    const int trace = pom_dbg_int("sc_trace", 0) == 1;
    const double t0 = trace ? now_ms() : 0.0;
    for (int i = 0; i < k; i++)
        g[i]->rc = LZO_E_ERROR;
    struct slot *t = sc_slot(q);
    if (!t)
        return;
    const int zc = sc_zero_copy();
    const size_t H = sc_hdr_bytes(k);
    size_t o = H, o_out[kScGroup], o_src[kScGroup];
    for (int i = 0; i < k; i++) {
        o_src[i] = o;
        o += ALIGN_UP(g[i]->src_len, 256);
    }
    const size_t I = o;
    for (int i = 0; i < k; i++) {
        o_out[i] = o;
        o += ALIGN_UP(g[i]->room, 256);
    }
    const size_t J = o;
    if (slot_reserve(t, J, J) != 0)
        return;
    uint8_t *h = t->hmem, *d = t->dmem;
    hipStream_t s = t->stream;
    struct sc_hdr hh = sc_hdr_at(h, k), dh = sc_hdr_at(d, k);
    memset(h, 0, H);
    for (int i = 0; i < k; i++) {
        hh.src_off[i] = o_src[i];
        hh.dst_off[i] = o_out[i];
        hh.src_len[i] = (uint32_t)g[i]->src_len;
        hh.dst_cap[i] = (uint32_t)g[i]->room;
        hh.status[i] = -1;
        if (g[i]->src_len)
            memcpy(h + o_src[i], g[i]->src, g[i]->src_len);
    }
    if (hipMemcpyAsync(d, h, I, hipMemcpyHostToDevice, s) != hipSuccess)
        return;
    /* zero copy: outputs, out_len and status land in the pinned host staging */
    uint8_t *out = zc ? h : d;
    uint32_t *olen = zc ? hh.out_len : dh.out_len;
    int32_t *ost = zc ? hh.status : dh.status;
    int rc;
    if (kind == SC_COMPRESS) {
        /* no scratch: the LDS-dictionary encoder, faster for a few blocks; the
         * general encoder's pass only for a block over 16 MiB */
        int big = 0;
        for (int i = 0; i < k; i++)
            big |= g[i]->src_len > LZO_MI355X_FAST_MAX_N;
        rc = lzo_mi355x_launch_compress_fast(d, dh.src_off, dh.src_len, out, dh.dst_off, dh.dst_cap, olen,
                                             ost, (uint32_t)k, NULL, 0, s);
        if (rc == 0 && big)
            rc = lzo_mi355x_launch_compress(d, dh.src_off, dh.src_len, out, dh.dst_off, dh.dst_cap, olen, ost,
                                            (uint32_t)k, 1, s);
    } else {
        /* SC_UNCHECKED: decoded into the room; the unchecked decoder never
         * reports an output overrun (lib/minilzo.c:3676-3680), so
         * OUTPUT_OVERRUN here means the stream is longer than the room.
         * The windowed decoder never reads its output back (host memory);
         * its fallback list lives in the header (zeroed by the H2D copy). */
        const int lat = lat_group(t, g, k, d, out, o_src, o_out, olen, ost, dh.fb, s);
        rc = lat < 0   ? -1
             : lat > 0 ? 0
                       : lzo_mi355x_launch_decompress_win(d, dh.src_off, dh.src_len, out, dh.dst_off,
                                                          dh.dst_cap, olen, ost, dh.fb, dh.fb + 1,
                                                          (uint32_t)k, s);
    }
    /* (copy mode: lengths and statuses, then the outputs) */
    if (rc != 0 ||
        (!zc && (hipMemcpyAsync(h + k * 16, d + k * 16, (size_t)k * 16, hipMemcpyDeviceToHost, s) !=
                     hipSuccess ||
                 hipMemcpyAsync(h + I, d + I, J - I, hipMemcpyDeviceToHost, s) != hipSuccess)) ||
        hipStreamSynchronize(s) != hipSuccess)
        return;
    if (kind != SC_COMPRESS) {
        int handed = 0;
        for (int i = 0; i < k; i++)
            handed |= hh.status[i] == 0x7FFF0001;       /* (the throughput decoders' "exact decoder pending") */
        if (handed &&
            (lzo_mi355x_launch_decompress_exact(d, dh.src_off, dh.src_len, out, dh.dst_off, dh.dst_cap,
                                                olen, ost, dh.fb, dh.fb + 1, (uint32_t)k, (uint32_t)k,
                                                kind == SC_UNCHECKED, s) != 0 ||
             (!zc && (hipMemcpyAsync(h + k * 16, d + k * 16, (size_t)k * 16, hipMemcpyDeviceToHost, s) !=
                          hipSuccess ||
                      hipMemcpyAsync(h + I, d + I, J - I, hipMemcpyDeviceToHost, s) != hipSuccess)) ||
             hipStreamSynchronize(s) != hipSuccess))
            return;
    }
    int over = 0;
    for (int i = 0; i < k; i++)
        over |= kind == SC_UNCHECKED && hh.status[i] == LZO_E_OUTPUT_OVERRUN;
    if (over) {
        /* rare: the decoded lengths (inputs still on the GPU); a call whose
         * stream is longer than its room retries with that much room */
        if (lzo_mi355x_launch_decoded_length(d, dh.src_off, dh.src_len, dh.plen, dh.pstatus,
                                             (uint32_t)k, NULL, 0xFFFFFFFFu, s) != 0 ||
            hipMemcpyAsync(hh.plen, dh.plen, (size_t)k * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return;
    }
    for (int i = 0; i < k; i++) {
        struct sc_req *r = g[i];
        if (over && hh.status[i] == LZO_E_OUTPUT_OVERRUN && hh.plen[i] > r->room) {
            r->produced = hh.plen[i];
            r->rc = 1;
            continue;
        }
        const size_t n = hh.out_len[i] < r->room ? hh.out_len[i] : r->room;
        if (n)
            memcpy(r->dst, h + o_out[i], n);
        r->produced = hh.out_len[i];
        r->rc = hh.status[i];
    }
    if (trace)
        fprintf(stderr, "pom single-call group: kind %d, %d calls, %.3f ms\n", (int)kind, k, now_ms() - t0);
}

static int single_call(enum sc_kind kind, const uint8_t *src, size_t src_len, uint8_t *dst,
                       size_t room, size_t *produced)
{
    int dev = 0;
    if (src_len > 0xFFFFFFF0u || room > 0xFFFFFFF0u || lzo_mi355x_device_count() <= 0 ||
        hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev)
        return LZO_E_ERROR;
    struct sc_req r = {kind, src, src_len, dst, room, 0, LZO_E_ERROR, 0, 0, NULL};
    if (!sc_combine()) {
        struct sc_req *g = &r;
        sc_run_group(&g, 1, NULL);
        *produced = r.produced;
        return r.rc;
    }
    pthread_once(&sc_once, sc_init);
    struct sc_queue *q = &sc_q[dev];
    pthread_mutex_lock(&q->mu);
    if (q->tail)
        q->tail->next = &r;
    else
        q->head = &r;
    q->tail = &r;
    if (q->leader)
        pthread_cond_broadcast(&q->cv);         /* (a leader may be waiting for company) */
    while (!r.done) {
        if (q->leader) {
            pthread_cond_wait(&q->cv, &q->mu);
            continue;
        }
        /* lead: the queue's oldest calls of the oldest call's kind.  When this
         * thread's previous call was in the last group and that group had
         * company, the other callers are probably between two calls: give
         * them ~50 us to queue.  (A thread that was not in it -- a lone caller
         * after a burst of others -- does not wait: ADVICE round 3.) */
        q->leader = 1;
        if (q->last_k > 1 && q->head == q->tail && sc_last_group[dev] == q->seq) {
            struct timespec ts;
            clock_gettime(CLOCK_MONOTONIC, &ts);
            ts.tv_nsec += 50000;
            if (ts.tv_nsec >= 1000000000L) {
                ts.tv_sec++;
                ts.tv_nsec -= 1000000000L;
            }
            pthread_cond_timedwait(&q->cv, &q->mu, &ts);
        }
        struct sc_req *g[kScGroup];
        int k = 0;
        size_t bytes = 0;
        const enum sc_kind gk = q->head->kind;
        struct sc_req **pp = &q->head, *prev = NULL;
        while (*pp && k < kScGroup) {
            struct sc_req *x = *pp;
            const size_t xb = x->room + x->src_len;
            if (x->kind != gk || (k > 0 && bytes + xb > kScGroupBytes)) {
                prev = x;
                pp = &x->next;
                continue;
            }
            *pp = x->next;
            if (q->tail == x)
                q->tail = prev;
            x->next = NULL;
            g[k++] = x;
            bytes += xb;
        }
        pthread_mutex_unlock(&q->mu);
        sc_run_group(g, k, q);
        pthread_mutex_lock(&q->mu);
        q->seq++;
        for (int i = 0; i < k; i++) {
            g[i]->done = 1;
            g[i]->group = q->seq;
        }
        q->leader = 0;
        q->last_k = k;
        pthread_cond_broadcast(&q->cv);
    }
    pthread_mutex_unlock(&q->mu);
    sc_last_group[dev] = r.group;
    *produced = r.produced;
    return r.rc;
}

/* lib/minilzo.c:3159-3207.  The output is the reference's with a zero-filled
 * wrkmem (SURVEY.md finding 3), so wrkmem is not read. */
int lzo1x_1_compress(const lzo_bytep src, lzo_uint src_len, lzo_bytep dst, lzo_uintp dst_len,
                     lzo_voidp wrkmem)
{
    (void)wrkmem;
    size_t n = 0;
    const int rc = single_call(SC_COMPRESS, src, src_len, dst,
                               lzo_mi355x_worst_compress(src_len), &n);
    if (rc != LZO_E_ERROR)
        *dst_len = n;
    return rc;
}

/* lib/minilzo.c:3703-4190: *dst_len is the capacity in, the produced length out. */
int lzo1x_decompress_safe(const lzo_bytep src, lzo_uint src_len, lzo_bytep dst,
                          lzo_uintp dst_len, lzo_voidp wrkmem)
{
    (void)wrkmem;
    size_t n = 0;
    const int rc = single_call(SC_SAFE, src, src_len, dst, *dst_len, &n);
    if (rc != LZO_E_ERROR)
        *dst_len = n;
    return rc;
}

/* GPU pre-scan of one host-resident stream: decoded length and status. */
int lzo_mi355x_decoded_length(const uint8_t *src, unsigned long src_len, unsigned long *dst_len)
{
    struct slot *t = single_slot();
    if (!t || src_len > 0xFFFFFFF0u)
        return LZO_E_ERROR;
    const size_t o_src = sc_hdr_bytes(1);
    if (slot_reserve(t, o_src + src_len + 16, o_src + src_len + 16) != 0)
        return LZO_E_ERROR;
    uint8_t *h = t->hmem, *d = t->dmem;
    hipStream_t s = t->stream;
    struct sc_hdr hh = sc_hdr_at(h, 1), dh = sc_hdr_at(d, 1);
    memset(h, 0, o_src);
    hh.src_off[0] = o_src;
    hh.src_len[0] = (uint32_t)src_len;
    if (src_len)
        memcpy(h + o_src, src, src_len);
    if (hipMemcpyAsync(d, h, o_src + src_len, hipMemcpyHostToDevice, s) != hipSuccess ||
        lzo_mi355x_launch_decoded_length(d, dh.src_off, dh.src_len, dh.plen, dh.pstatus, 1, NULL,
                                         0xFFFFFFFFu, s) != 0 ||
        hipMemcpyAsync(h, d, o_src, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return LZO_E_ERROR;
    *dst_len = hh.plen[0];
    return hh.pstatus[0];
}

/* The unchecked decoder (lib/minilzo.c:3308-3699) that mds/itb.c:2964,
 * mdsl/gc.c:770 and api/api.c:6438 call.  It never learns the destination
 * size (mds/itb.c:2951-2964 passes an uninitialised *out_len): the GPU
 * decodes into a guessed room (16x the input, at least 256 KiB) and the
 * output comes back with its length in one round trip; only a block that
 * decodes to more than that takes a length pre-scan and a second decode. */
int lzo1x_decompress(const lzo_bytep src, lzo_uint src_len, lzo_bytep dst, lzo_uintp dst_len,
                     lzo_voidp wrkmem)
{
    (void)wrkmem;
    size_t room = (size_t)src_len * 16;
    if (room < ((size_t)256 << 10))
        room = (size_t)256 << 10;
    if (room > 0xFFFFFFF0u)
        room = 0xFFFFFFF0u;
    size_t n = 0;
    int rc = single_call(SC_UNCHECKED, src, src_len, dst, room, &n);
    if (rc == 1)                                   /* longer than the guess */
        rc = single_call(SC_UNCHECKED, src, src_len, dst, n, &n);
    if (rc != LZO_E_ERROR)
        *dst_len = n;
    return rc;
}
