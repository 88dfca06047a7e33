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
 * GC thread and client threads.  Each host thread gets its own HIP stream and
 * its own device/pinned staging (grown on demand, freed at thread exit), so
 * concurrent calls never share device state.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "lzo_mi355x.h"
#include "lzo_mi355x_kernels.h"
#include "minilzo.h"

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
/* Per-thread stream and staging                                            */
/* ------------------------------------------------------------------------ */
struct tctx {
    int ready;
    int device;
    hipStream_t stream;
    uint8_t *dmem;
    size_t dcap;
    uint8_t *hmem;
    size_t hcap;
};

static pthread_key_t tkey;
static pthread_once_t tkey_once = PTHREAD_ONCE_INIT;

static void tctx_free(void *p)
{
    struct tctx *t = p;
    if (!t)
        return;
    if (t->ready) {
        hipSetDevice(t->device);
        if (t->dmem)
            hipFree(t->dmem);
        if (t->hmem)
            hipHostFree(t->hmem);
        hipStreamDestroy(t->stream);
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
    if (!t->ready) {
        if (hipGetDevice(&t->device) != hipSuccess)
            return NULL;
        if (hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking) != hipSuccess)
            return NULL;
        t->ready = 1;
    }
    return t;
}

static int tctx_reserve(struct tctx *t, size_t dbytes, size_t hbytes)
{
    if (dbytes > t->dcap) {
        if (t->dmem)
            hipFree(t->dmem);
        t->dmem = NULL;
        t->dcap = 0;
        size_t want = ALIGN_UP(dbytes + dbytes / 4, 1 << 20);
        if (hipMalloc((void **)&t->dmem, want) != hipSuccess)
            return -1;
        t->dcap = want;
    }
    if (hbytes > t->hcap) {
        if (t->hmem)
            hipHostFree(t->hmem);
        t->hmem = NULL;
        t->hcap = 0;
        size_t want = ALIGN_UP(hbytes + hbytes / 4, 1 << 20);
        if (hipHostMalloc((void **)&t->hmem, want, hipHostMallocDefault) != hipSuccess)
            return -1;
        t->hcap = want;
    }
    return 0;
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

/* Scratch: the fast decoder's fallback list [count, block ids], then its
 * per-block op slots at a 256-byte boundary. */
static size_t fallback_bytes(uint32_t nblocks)
{
    return (4 * ((size_t)nblocks + 1) + 255) & ~(size_t)255;
}

size_t lzo_mi355x_decompress_scratch(uint32_t nblocks)
{
    return fallback_bytes(nblocks) + (size_t)nblocks * lzo_mi355x_fast_ops_bytes_per_block();
}

/* Fast decoder over the whole batch, then the exact decoder over the blocks
 * it refused (malformed input, capacity/lookbehind errors, pathological
 * streams).  Without scratch every block takes the exact decoder.
 * unchecked: the exact decoder follows the unchecked lzo1x_decompress (the
 * fast decoder only ever finishes streams on which both agree). */
static int decompress_dev(const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len,
                          uint8_t *dst, const uint64_t *dst_off, const uint32_t *dst_cap,
                          uint32_t *out_len, int32_t *status, uint32_t nblocks, void *scratch,
                          int unchecked, hipStream_t s)
{
    if (nblocks == 0)
        return 0;
    if (!scratch)
        return lzo_mi355x_launch_decompress_exact(src, src_off, src_len, dst, dst_off, dst_cap,
                                                  out_len, status, NULL, nblocks, nblocks,
                                                  unchecked, s);
    uint32_t *fb = (uint32_t *)scratch;
    if (hipMemsetAsync(fb, 0, 4, s) != hipSuccess)
        return -1;
    if (lzo_mi355x_launch_decompress_fast(src, src_off, src_len, dst, dst_off, dst_cap, out_len,
                                          status, fb, (uint8_t *)scratch + fallback_bytes(nblocks),
                                          nblocks, s) != 0)
        return -1;
    const uint32_t ngrid = nblocks < 512 ? nblocks : 512;
    return lzo_mi355x_launch_decompress_exact(src, src_off, src_len, dst, dst_off, dst_cap,
                                              out_len, status, fb, ngrid, nblocks, unchecked, s);
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

/* Staging layout (identical on host and device, so one copy each way):
 *   [src_off u64][dst_off u64][src_len u32][dst_cap u32][out_len u32][status i32]
 *   [packed offset u64]
 *   [src bytes, 16-B aligned per block][dst bytes, 16-B aligned per block]
 *   [decoder scratch]  [device only: packed output]
 * The kernels write each block into its capacity-sized dst slot; only the
 * produced bytes come back, packed (pack kernel), in one D2H copy into the
 * host's dst region. */
struct layout {
    size_t nb;
    size_t o_srcoff, o_dstoff, o_srclen, o_dstcap, o_outlen, o_status, o_poff;
    size_t o_src, o_dst, o_scr, o_pack, total, dtotal;
    size_t src_bytes, dst_bytes;
};

static void layout_make(struct layout *L, size_t nb, const size_t *src_len, const size_t *dst_cap)
{
    L->nb = nb;
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
    for (size_t b = 0; b < nb; b++) {
        s += ALIGN_UP(src_len[b], 16);
        d += ALIGN_UP(dst_cap[b], 16);
    }
    L->src_bytes = s;
    L->dst_bytes = d;
    o += ALIGN_UP(s, 256);
    L->o_dst = o;
    o += ALIGN_UP(d, 256);
    L->o_scr = o;
    const size_t scr_d = lzo_mi355x_decompress_scratch((uint32_t)nb);
    const size_t scr_c = lzo_mi355x_compress_scratch((uint32_t)nb);
    o += ALIGN_UP(scr_d > scr_c ? scr_d : scr_c, 256);
    L->total = o;
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
    for (size_t b = 0; b < L->nb; b++) {
        so[b] = s;
        dof[b] = d;
        sl[b] = (uint32_t)src_len[b];
        dc[b] = (uint32_t)dst_cap[b];
        if (jobs) {
            jobs[b].dst = h + L->o_src + s;
            jobs[b].src = src[b];
            jobs[b].len = src_len[b];
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

/* Runs one staged batch.  dst_cap: capacities used by the kernels.  On
 * return out_len/status of each block are in the pinned staging. */
static int run_staged(struct tctx *t, const struct layout *L, enum op_kind kind)
{
    uint8_t *d = t->dmem, *h = t->hmem;
    hipStream_t s = t->stream;
    const uint32_t nb = (uint32_t)L->nb;
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
    if (kind == OP_COMPRESS)
        rc = lzo_mi355x_compress_dev(dsrc, so, sl, ddst, dof, dc, ol, st, nb, d + L->o_scr, s);
    else if (kind == OP_DECOMPRESS)
        rc = decompress_dev(dsrc, so, sl, ddst, dof, dc, ol, st, nb, d + L->o_scr, 0, s);
    else
        rc = lzo_mi355x_launch_decompress_concat(dsrc, so, sl, ddst, dof, dc, ol, st, nb, s);
    if (rc != 0)
        return -1;
    if (hipMemcpyAsync(h + L->o_outlen, d + L->o_outlen, 8 * L->nb, hipMemcpyDeviceToHost, s) !=
            hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -1;
    /* packed offsets of the produced bytes, then one copy of exactly those */
    const uint32_t *hol = (const uint32_t *)(h + L->o_outlen);
    const uint32_t *hdc = (const uint32_t *)(h + L->o_dstcap);
    uint64_t *poff = (uint64_t *)(h + L->o_poff);
    size_t packed = 0;
    for (size_t b = 0; b < L->nb; b++) {
        poff[b] = packed;
        packed += ALIGN_UP((size_t)(hol[b] < hdc[b] ? hol[b] : hdc[b]), 16);
    }
    if (packed == 0)
        return 0;
    if (hipMemcpyAsync(d + L->o_poff, poff, 8 * L->nb, hipMemcpyHostToDevice, s) != hipSuccess)
        return -1;
    if (lzo_mi355x_launch_pack(d + L->o_dst, dof, ol, dc, (const uint64_t *)(d + L->o_poff),
                               d + L->o_pack, nb, s) != 0)
        return -1;
    if (hipMemcpyAsync(h + L->o_dst, d + L->o_pack, packed, hipMemcpyDeviceToHost, s) !=
        hipSuccess)
        return -1;
    return hipStreamSynchronize(s) == hipSuccess ? 0 : -1;
}

/* POM_HOST_TIMING=1: per-phase wall times of each host batch on stderr (diagnostic) */
static double now_ms(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

static int batch_common(enum op_kind kind, const uint8_t *const *src, const size_t *src_len,
                        uint8_t *const *dst, size_t *dst_len, int *status, size_t nblocks)
{
    static int timing = -1;
    if (timing < 0) {
        const char *e = getenv("POM_HOST_TIMING");
        timing = e && *e == '1';
    }
    double tm[5] = {0};
    if (timing)
        tm[0] = now_ms();
    struct tctx *t = tctx_get();
    if (!t)
        return LZO_E_ERROR;
    if (nblocks == 0)
        return LZO_E_OK;
    if (nblocks > 0xFFFFFFFFu)
        return LZO_E_ERROR;
    size_t *cap = malloc(nblocks * sizeof(size_t));
    if (!cap)
        return LZO_E_OUT_OF_MEMORY;
    for (size_t b = 0; b < nblocks; b++) {
        if (src_len[b] > 0xFFFFFFF0u) {
            free(cap);
            return LZO_E_ERROR;
        }
        cap[b] = kind == OP_COMPRESS ? lzo_mi355x_worst_compress(src_len[b]) : dst_len[b];
        if (cap[b] > 0xFFFFFFF0u)
            cap[b] = 0xFFFFFFF0u;
    }
    struct layout L;
    layout_make(&L, nblocks, src_len, cap);
    int rc = LZO_E_ERROR;
    if (tctx_reserve(t, L.dtotal, L.total) == 0) {
        if (timing)
            tm[1] = now_ms();
        layout_fill(&L, t->hmem, src, src_len, cap);
        if (timing)
            tm[2] = now_ms();
        if (run_staged(t, &L, kind) == 0) {
            if (timing)
                tm[3] = now_ms();
            const uint32_t *ol = (const uint32_t *)(t->hmem + L.o_outlen);
            const int32_t *st = (const int32_t *)(t->hmem + L.o_status);
            const uint64_t *poff = (const uint64_t *)(t->hmem + L.o_poff);
            struct copy_job *jobs = malloc(nblocks * sizeof(*jobs));
            for (size_t b = 0; b < nblocks; b++) {
                size_t n = ol[b] < cap[b] ? ol[b] : cap[b];
                if (jobs) {
                    jobs[b].dst = dst[b];
                    jobs[b].src = t->hmem + L.o_dst + poff[b];
                    jobs[b].len = n;
                } else if (n) {
                    memcpy(dst[b], t->hmem + L.o_dst + poff[b], n);
                }
                dst_len[b] = ol[b];
                status[b] = st[b];
            }
            if (jobs) {
                copy_jobs(jobs, nblocks);
                free(jobs);
            }
            rc = LZO_E_OK;
            if (timing) {
                tm[4] = now_ms();
                fprintf(stderr, "pom host %s n=%zu: reserve %.2f pack %.2f gpu %.2f unpack %.2f ms\n",
                        kind == OP_COMPRESS ? "compress" : "decompress", nblocks, tm[1] - tm[0],
                        tm[2] - tm[1], tm[3] - tm[2], tm[4] - tm[3]);
            }
        }
    }
    free(cap);
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

/* ---- single calls ------------------------------------------------------------
 * One block, one stream synchronisation: the header and the input go up, the
 * kernels run, and the header plus an output region the host sizes up front
 * come back in one go.  Staging (device and pinned host alike):
 *   [0, 256)        header: src_off u64, dst_off u64, src_len, dst_cap,
 *                   out_len, status, pre-scan length / status / capacity,
 *                   fallback list (2 words)
 *   [256, +G)       output (G: worst case, the caller's capacity, or a guess)
 *   then the input, then the fast decoder's scratch (device only)
 */
enum { SC_HDR = 256 };
struct sc_hdr {
    uint64_t src_off, dst_off;
    uint32_t src_len, dst_cap, out_len;
    int32_t status;
    uint32_t plen;
    int32_t pstatus;
    uint32_t pcap;
    uint32_t fb[2];
};

enum sc_kind { SC_COMPRESS, SC_SAFE, SC_UNCHECKED };

static int single_call(enum sc_kind kind, const uint8_t *src, size_t src_len, uint8_t *dst,
                       size_t room, size_t *produced)
{
    struct tctx *t = tctx_get();
    if (!t || src_len > 0xFFFFFFF0u || room > 0xFFFFFFF0u)
        return LZO_E_ERROR;
    const size_t o_src = SC_HDR + ALIGN_UP(room, 256);
    const size_t o_scr = o_src + ALIGN_UP(src_len, 256);
    const size_t dneed = o_scr + (kind == SC_COMPRESS ? 0 : lzo_mi355x_decompress_scratch(1));
    if (tctx_reserve(t, dneed, o_scr) != 0)
        return LZO_E_ERROR;
    uint8_t *h = t->hmem, *d = t->dmem;
    hipStream_t s = t->stream;
    struct sc_hdr *hh = (struct sc_hdr *)h;
    memset(hh, 0, sizeof(*hh));
    hh->src_off = o_src;
    hh->dst_off = SC_HDR;
    hh->src_len = (uint32_t)src_len;
    hh->dst_cap = (uint32_t)room;
    if (src_len)
        memcpy(h + o_src, src, src_len);
    struct sc_hdr *dh = (struct sc_hdr *)d;
    const uint64_t *so = &dh->src_off, *dof = &dh->dst_off;
    const uint32_t *sl = &dh->src_len;
    if (hipMemcpyAsync(d, h, sizeof(*hh), hipMemcpyHostToDevice, s) != hipSuccess ||
        (src_len && hipMemcpyAsync(d + o_src, h + o_src, src_len, hipMemcpyHostToDevice, s) !=
                        hipSuccess))
        return LZO_E_ERROR;
    int rc = 0;
    if (kind == SC_COMPRESS) {
        rc = lzo_mi355x_compress_dev(d, so, sl, d, dof, &dh->dst_cap, &dh->out_len, &dh->status, 1,
                                     NULL, s);   /* one block: the LDS dictionary is faster */
    } else if (kind == SC_SAFE) {
        rc = decompress_dev(d, so, sl, d, dof, &dh->dst_cap, &dh->out_len, &dh->status, 1,
                            d + o_scr, 0, s);
    } else {
        /* the unchecked decoder's own length, capped at the room (decoded
         * again with more room when it does not fit) */
        rc = lzo_mi355x_launch_decoded_length(d, so, sl, &dh->plen, &dh->pstatus, 1, &dh->pcap,
                                              (uint32_t)room, s);
        if (rc == 0)
            rc = decompress_dev(d, so, sl, d, dof, &dh->pcap, &dh->out_len, &dh->status, 1,
                                d + o_scr, 1, s);
    }
    if (rc != 0 || hipMemcpyAsync(h, d, o_src, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return LZO_E_ERROR;
    if (kind == SC_UNCHECKED && hh->plen > room) {
        *produced = hh->plen;                      /* needs more room: the caller retries */
        return 1;
    }
    const size_t n = hh->out_len < room ? hh->out_len : room;
    if (n)
        memcpy(dst, h + SC_HDR, n);
    *produced = hh->out_len;
    return hh->status;
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
    struct tctx *t = tctx_get();
    if (!t || src_len > 0xFFFFFFF0u)
        return LZO_E_ERROR;
    const size_t o_src = SC_HDR;
    if (tctx_reserve(t, o_src + src_len + 16, o_src + src_len + 16) != 0)
        return LZO_E_ERROR;
    uint8_t *h = t->hmem, *d = t->dmem;
    hipStream_t s = t->stream;
    struct sc_hdr *hh = (struct sc_hdr *)h, *dh = (struct sc_hdr *)d;
    memset(hh, 0, sizeof(*hh));
    hh->src_off = o_src;
    hh->src_len = (uint32_t)src_len;
    if (src_len)
        memcpy(h + o_src, src, src_len);
    if (hipMemcpyAsync(d, h, o_src + src_len, hipMemcpyHostToDevice, s) != hipSuccess ||
        lzo_mi355x_launch_decoded_length(d, &dh->src_off, &dh->src_len, &dh->plen, &dh->pstatus,
                                         1, NULL, 0xFFFFFFFFu, s) != 0 ||
        hipMemcpyAsync(h, d, sizeof(*hh), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return LZO_E_ERROR;
    *dst_len = hh->plen;
    return hh->pstatus;
}

/* The unchecked decoder (lib/minilzo.c:3308-3699) that mds/itb.c:2964,
 * mdsl/gc.c:770 and api/api.c:6438 call.  It never learns the destination
 * size (mds/itb.c:2951-2964 passes an uninitialised *out_len): the GPU
 * pre-scans the stream's decoded length in the same launch sequence and the
 * output comes back with it; only a block that decodes to more than the
 * guessed room (16x the input, at least 256 KiB) takes a second round trip. */
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
