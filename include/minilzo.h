/*
 * minilzo.h -- drop-in header for the MI355X LZO1X codec (liblzo_mi355x.so).
 *
 * Keeps the call surface Pomegranate compiles against
 * (include/hvfs_u.h:61 includes "minilzo.h"), so mds/itb.c, mds/txg.c,
 * mdsl/gc.c and api/api.c build unchanged against this library instead of
 * the vendored lib/minilzo.c.  Names, types and values follow the reference's
 * lib/minilzo.h and lib/lzoconf.h on LP64; nothing here is copied from them.
 *
 * Each entry point below replaces the reference function cited beside it.
 * All codec work runs on the GPU (HIP kernels for gfx950); there is no CPU
 * fallback: without a usable GPU, lzo_init() and every codec call return
 * LZO_E_ERROR.
 */
#ifndef POM_MINILZO_H
#define POM_MINILZO_H 1

#include <limits.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MINILZO_VERSION 0x2040            /* lib/minilzo.h:52 */
#define LZO_VERSION 0x2040                /* lib/lzoconf.h:46 */
#define LZO_VERSION_STRING "2.04"         /* lib/lzoconf.h:47 */
#define LZO_VERSION_DATE "Oct 31 2010"    /* lib/lzoconf.h:48 */

/* Integral types, lib/lzoconf.h:113-197 (LP64: lzo_uint is unsigned long). */
typedef unsigned long lzo_uint;
typedef long lzo_int;
typedef unsigned int lzo_uint32;
typedef int lzo_int32;
typedef unsigned long lzo_xint;
typedef unsigned char lzo_byte;
typedef unsigned char *lzo_bytep;
typedef char *lzo_charp;
typedef void *lzo_voidp;
typedef lzo_uint *lzo_uintp;
typedef lzo_int *lzo_intp;
typedef lzo_uint32 *lzo_uint32p;
typedef const unsigned char *lzo_cbytep;

/* Callback record whose size lzo_init() reports (lib/lzoconf.h:269-293). */
typedef struct lzo_callback_t lzo_callback_t;
typedef lzo_voidp (*lzo_alloc_func_t)(lzo_callback_t *self, lzo_uint items, lzo_uint size);
typedef void (*lzo_free_func_t)(lzo_callback_t *self, lzo_voidp ptr);
typedef void (*lzo_progress_func_t)(lzo_callback_t *, lzo_uint, lzo_uint, int);
struct lzo_callback_t {
    lzo_alloc_func_t nalloc;
    lzo_free_func_t nfree;
    lzo_progress_func_t nprogress;
    lzo_voidp user1;
    lzo_xint user2;
    lzo_xint user3;
};

/* Alignment helper used by callers to size wrkmem (api/api.c:1140,
 * lib/lzoconf.h:366). */
typedef union {
    void *vp;
    lzo_bytep bp;
    lzo_uint u;
    lzo_uint32 u32;
    unsigned long l;
} lzo_align_t;

/* Error codes, lib/lzoconf.h:309-318. */
#define LZO_E_OK 0
#define LZO_E_ERROR (-1)
#define LZO_E_OUT_OF_MEMORY (-2)
#define LZO_E_NOT_COMPRESSIBLE (-3)
#define LZO_E_INPUT_OVERRUN (-4)
#define LZO_E_OUTPUT_OVERRUN (-5)
#define LZO_E_LOOKBEHIND_OVERRUN (-6)
#define LZO_E_EOF_NOT_FOUND (-7)
#define LZO_E_INPUT_NOT_CONSUMED (-8)
#define LZO_E_NOT_YET_IMPLEMENTED (-9)

/* Work-memory sizes, lib/minilzo.h:79-81.  Callers allocate this much
 * (mds/txg.c:835, api/api.c:1140); the GPU codec does not read it: output is
 * defined as the reference's output with a zero-filled wrkmem. */
#define lzo_sizeof_dict_t ((unsigned)sizeof(lzo_bytep))
#define LZO1X_1_MEM_COMPRESS ((lzo_uint32)(16384L * lzo_sizeof_dict_t))
#define LZO1X_MEM_COMPRESS LZO1X_1_MEM_COMPRESS
#define LZO1X_MEM_DECOMPRESS (0)

/* Pointer-sized unsigned integer (lib/lzoconf.h:198-222 on LP64). */
typedef unsigned long lzo_uintptr_t;

/* Replaces lib/minilzo.c:2567-2598 (__lzo_init_v2).  Checks the caller's
 * type sizes like the reference, then that a gfx950 GPU is usable. */
int __lzo_init_v2(unsigned, int, int, int, int, int, int, int, int, int);
#define lzo_init()                                                                       \
    __lzo_init_v2(LZO_VERSION, (int)sizeof(short), (int)sizeof(int), (int)sizeof(long), \
                  (int)sizeof(lzo_uint32), (int)sizeof(lzo_uint), (int)lzo_sizeof_dict_t, \
                  (int)sizeof(char *), (int)sizeof(lzo_voidp), (int)sizeof(lzo_callback_t))

/* Version functions: replace lib/minilzo.c:2306-2344 (declared at
 * lib/lzoconf.h:338-342). */
unsigned lzo_version(void);
const char *lzo_version_string(void);
const char *lzo_version_date(void);
/* (the reference declares these `const lzo_charp` / `const lzo_bytep`: a
 * top-level const on a return type, which C ignores; the type is the same) */
lzo_charp _lzo_version_string(void);
lzo_charp _lzo_version_date(void);
lzo_bytep lzo_copyright(void);

/* Host utilities the reference's minilzo.c also exports (lib/lzoconf.h:344-372).
 * They touch no compressed data and run on the host, as in the reference. */
int lzo_memcmp(const lzo_voidp a, const lzo_voidp b, lzo_uint len);   /* lib/minilzo.c:2421 */
lzo_voidp lzo_memcpy(lzo_voidp dst, const lzo_voidp src, lzo_uint len);
lzo_voidp lzo_memmove(lzo_voidp dst, const lzo_voidp src, lzo_uint len);
lzo_voidp lzo_memset(lzo_voidp buf, int c, lzo_uint len);
/* Adler-32 with the reference's buf == NULL -> 1 rule (lib/minilzo.c:2355-2391). */
lzo_uint32 lzo_adler32(lzo_uint32 c, const lzo_bytep buf, lzo_uint len);
/* lib/minilzo.c:2522-2561: LZO_E_OK when the byte order and unaligned access
 * the library assumes hold. */
int _lzo_config_check(void);
/* lib/minilzo.c:2251-2287. */
lzo_uintptr_t __lzo_ptr_linear(const lzo_voidp ptr);
unsigned __lzo_align_gap(const lzo_voidp p, lzo_uint size);
#define LZO_PTR_ALIGN_UP(p, size) ((p) + (lzo_uint)__lzo_align_gap((const lzo_voidp)(p), (lzo_uint)(size)))

/* Replaces lib/minilzo.c:3159-3207 (lzo1x_1_compress).  Output is
 * byte-identical to the reference with a zero-filled wrkmem; dst must hold
 * src_len + src_len/16 + 67 bytes, as with the reference. */
int lzo1x_1_compress(const lzo_bytep src, lzo_uint src_len, lzo_bytep dst,
                     lzo_uintp dst_len, lzo_voidp wrkmem);

/* Replaces lib/minilzo.c:3308-3699 (lzo1x_decompress, unchecked).  Like the
 * reference it ignores the incoming *dst_len; the decoded length is found on
 * the GPU first, and malformed input returns an LZO_E_* code instead of
 * overrunning memory. */
int lzo1x_decompress(const lzo_bytep src, lzo_uint src_len, lzo_bytep dst,
                     lzo_uintp dst_len, lzo_voidp wrkmem);

/* Replaces lib/minilzo.c:3703-4190 (lzo1x_decompress_safe): *dst_len is the
 * capacity in and the produced length out; return codes match bit for bit. */
int lzo1x_decompress_safe(const lzo_bytep src, lzo_uint src_len, lzo_bytep dst,
                          lzo_uintp dst_len, lzo_voidp wrkmem);

#ifdef __cplusplus
}
#endif

#endif /* POM_MINILZO_H */
