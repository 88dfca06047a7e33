// lzo1x_decode_quad.hip -- the quarter-wave LZO1X decoder for MI355X (gfx950):
// FOUR blocks per workgroup, 16 lanes (a quarter wave) per block, three waves
// with one job each.
//
// The grammar is lib/minilzo.c:3308-3699.  Every
// per-instruction cost of a serial LZ decoder (reading the control bytes,
// decoding, bounds checks, loop control) is paid once per wave instruction
// for four blocks at a time: each quarter of a wave runs its own block, and
// the quarters step in lockstep with per-quarter lane masks.
//
//  * PARSER wave: per quarter, one LZO1X instruction per step -- a literal
//    run, then the match with its 0-3 trailing literals -- decoded from the
//    block's compressed bytes staged in LDS.  It writes the literal bytes
//    into the block's 8 KiB LDS output ring itself and publishes each match
//    (cut into pieces of at most 1 KiB) as an 8-byte record.  It never runs
//    more than kLag output bytes ahead of the executor.
//  * EXECUTOR wave: per quarter, one record pass per step: up to 128 bytes of
//    a match, 8 per lane, read from the ring (a match shorter than 128 back
//    repeats its last period: byte t of the match is the byte (t mod d) of
//    the d bytes before it) and written exactly.  It stores completed 1 KiB
//    chunks of the ring to HBM and closes the block.
//  * LOADER wave: stages the compressed input ahead of the parser, and copies
//    the far matches (more than kFarT back: outside what the ring keeps) from
//    the block's own output in HBM into the ring before the executor reaches
//    them -- the only HBM reads of the output, all off the two chains.
//
// Ring invariants (R = kRing, per quarter, positions are output offsets):
// every write lands at a position below exec + kLag (exec: the executor's
// position, every byte below it final), so it overwrites a slot whose old
// position is below exec + kLag - R = exec - 6144; near sources are at most
// kFarT = 6000 back, and chunks are stored to HBM by then.  Far sources lie
// below exec + kLag - kFarT, which the executor has stored and waited for.
//
// A block this decoder does not finish exactly (malformed input, look-behind
// or capacity errors, EOF not at the end of the input, a destination not
// 16-byte aligned, empty or >= 16 MiB input or capacity) goes to the fallback
// list for lzo1x_decode_exact_kernel, which returns the reference's output
// and LZO_E_* code.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "lzo_mi355x_kernels.h"

namespace {

constexpr uint32_t kWave = 64;
constexpr uint32_t kQ = 4;                       // blocks (quarters) per workgroup
constexpr uint32_t kQL = 16;                     // lanes per quarter
constexpr uint32_t kRing = 8192;                 // output ring per block
constexpr uint32_t kRingMask = kRing - 1;
constexpr uint32_t kGuard = 16;                  // ring copies: [guard][ring][mirror]
constexpr uint32_t kRingStride = kGuard + kRing + 16;
constexpr uint32_t kStage = 512;                 // compressed-input ring per block
constexpr uint32_t kStageMask = kStage - 1;
constexpr uint32_t kStageStride = kStage + 16;   // + mirror of its first 16 bytes
constexpr uint32_t kStageChunk = 128;            // loader staging granule (8 B per lane)
constexpr uint32_t kNeed = 160;                  // input bytes a parser step may read past ip
constexpr uint32_t kRec = 64;                    // record ring per block
constexpr uint32_t kFarQ = 32;                   // far-copy queue per block
constexpr uint32_t kLag = 2048;                  // parser writes below exec + kLag
constexpr uint32_t kFarT = 6000;                 // matches further back are far copies
constexpr uint32_t kPiece = 1024;                // longest match record
constexpr uint32_t kSync = 512;                  // literal bytes between records at most (then a SYNC)
constexpr uint32_t kPass = kQL * 8;              // bytes per executor / literal pass
constexpr uint32_t kChunk = 1024;                // ring -> HBM granule
constexpr uint32_t kMaxLen = (1u << 24) - 1024;  // z and capacity limit (24-bit positions)
constexpr int32_t kFallback = 0x7FFF0001;
static_assert(kLag + kFarT < kRing - 128, "near sources survive the writes of the lag window");
static_assert(kFarT > kLag + 2 * kChunk, "far sources are stored before they are read");

// record kinds (high byte of word 0; low 24 bits: output position)
constexpr uint32_t RK_NEAR = 0, RK_FAR = 1, RK_SYNC = 2, RK_END = 3, RK_ERR = 4;

// instruction-start states
constexpr uint32_t ST_A = 0;                     // top of the loop (t < 16: literal run)
constexpr uint32_t ST_B = 1;                     // after a literal run (t < 16: 3-byte M1)
constexpr uint32_t ST_C = 2;                     // after 1-3 trailing literals (t < 16: 2-byte M1)
constexpr uint32_t ST_F = 3;                     // the first byte (lib/minilzo.c:3357)

struct __attribute__((aligned(16))) QuadLds {
    uint8_t ring[kQ][kRingStride];
    uint8_t stage[kQ][kStageStride];
    uint2 rec[kQ][kRec];
    uint2 farq[kQ][kFarQ];
    uint2 sel[8][8];                             // v_perm selectors, period d < 8, phase r
    uint32_t rec_pub[kQ];                        // parser -> executor: records published
    uint32_t rec_head[kQ];                       // executor -> parser: records consumed
    uint32_t expos[kQ];                          // executor: gen << 24 | position (bytes below final)
    uint32_t flushed[kQ];                        // executor: gen << 24 | bytes stored and drained
    uint32_t far_pub[kQ];                        // parser -> loader: far records published
    uint32_t far_done[kQ];                       // loader -> executor, parser: far records copied
    uint32_t pip[kQ];                            // parser: gen << 24 | ip (kIpDone: block parsed)
    uint32_t stg[kQ];                            // loader: gen << 24 | input bytes staged
    uint32_t bq[kQ][4];                          // parser -> others: block of generation g (at g mod 4)
    uint32_t live;                               // waves still running (exit of the loader)
};
static_assert(sizeof(QuadLds) * 4 <= 160 * 1024, "four workgroups (16 blocks) per CU");
constexpr uint32_t kIpDone = 0xFFFFFFu;

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint32_t lds_off(const void* p)
{
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// Hand-offs between the waves go through LDS only: one wave's LDS accesses
// execute in order, so a counter stored after the data it covers (and after
// an lgkmcnt wait) is never seen before that data; the readers' own LDS reads
// come after their counter read.  (Release/acquire atomics would also wait for
// the executor's HBM stores, which no other wave reads through these counters.)
// (compiler fences keep the plain LDS accesses on their side of these)
__device__ __forceinline__ uint32_t ld_acq(const uint32_t* p)
{
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    const uint32_t v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    return v;
}
__device__ __forceinline__ void lds_drain()
{
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0xC07F);          // lgkmcnt(0)
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
__device__ __forceinline__ void st_rel(uint32_t* p, uint32_t v)
{
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
// wave-wide OR of a lane predicate: any quarter (lane) that...
__device__ __forceinline__ bool any(bool p) { return __ballot(p) != 0; }

// Misaligned LDS accesses: gfx950 runs LDS in unaligned mode, so b128 / b64 /
// b32 / b16 at any byte address are exact (scripts/probe/lds_misaligned_probe.hip).
// The compiler assumes natural alignment for its own accesses, so these are
// written out.  LDS accesses of one wave complete in order, so the compiler's
// own lgkmcnt waits stay correct.
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint2 rd8(uint32_t a)
{
    v2u x;
    asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(x) : "v"(a) : "memory");
    return make_uint2(x.x, x.y);
}
__device__ __forceinline__ void rd8x3(uint32_t a, uint32_t b, uint32_t c, uint2& x, uint2& y, uint2& z)
{
    v2u p, q, r;
    asm volatile("ds_read_b64 %0, %3\n\tds_read_b64 %1, %4\n\tds_read_b64 %2, %5\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(p), "=&v"(q), "=&v"(r) : "v"(a), "v"(b), "v"(c) : "memory");
    x = make_uint2(p.x, p.y);
    y = make_uint2(q.x, q.y);
    z = make_uint2(r.x, r.y);
}
__device__ __forceinline__ uint4 rd16(uint32_t a)
{
    v4u x;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(x) : "v"(a) : "memory");
    return make_uint4(x.x, x.y, x.z, x.w);
}
__device__ __forceinline__ void wr8(uint32_t a, uint2 v)
{
    const v2u t = {v.x, v.y};
    asm volatile("ds_write_b64 %0, %1" : : "v"(a), "v"(t) : "memory");
}
__device__ __forceinline__ void wr4(uint32_t a, uint32_t v) { asm volatile("ds_write_b32 %0, %1" : : "v"(a), "v"(v) : "memory"); }
__device__ __forceinline__ void wr2(uint32_t a, uint32_t v) { asm volatile("ds_write_b16 %0, %1" : : "v"(a), "v"(v) : "memory"); }
__device__ __forceinline__ void wr1(uint32_t a, uint32_t v) { asm volatile("ds_write_b8 %0, %1" : : "v"(a), "v"(v) : "memory"); }

// Exactly the first nb (1..8) bytes of v at LDS address a.
__device__ __forceinline__ void wr_exact(uint32_t a, uint2 v, uint32_t nb)
{
    if (nb >= 8) {
        wr8(a, v);
        return;
    }
    uint64_t x = ((uint64_t)v.y << 32) | v.x;
    if (nb & 4) {
        wr4(a, (uint32_t)x);
        a += 4;
        x >>= 32;
    }
    if (nb & 2) {
        wr2(a, (uint32_t)x);
        a += 2;
        x >>= 16;
    }
    if (nb & 1)
        wr1(a, (uint32_t)x);
}

// The first nb (1..8) bytes of v at output position p of a ring (base: the
// ring's LDS offset, guard included): also into the guard / mirror copy when
// within 8 bytes of either end, so 8- and 16-byte reads never wrap.
__device__ __forceinline__ void ring_put(uint32_t base, uint32_t p, uint2 v, uint32_t nb)
{
    const uint32_t a = p & kRingMask;
    wr_exact(base + kGuard + a, v, nb);
    // bytes past the end belong at the start (the head lands in the guard);
    // the first 8 bytes are mirrored past the end for reads that cross it
    if (a + nb > kRing || a < 8)
        wr_exact(base + kGuard + (a < 8 ? a + kRing : a - kRing), v, nb);
}
__device__ __forceinline__ uint32_t ring_at(uint32_t base, uint32_t p) { return base + kGuard + (p & kRingMask); }

// Per-block buffers of a quarter.  Global memory accesses of a quarter use
// its own lanes' addresses (flat, not a buffer descriptor: the four blocks
// of a wave have different bases).
struct Blk {
    const uint8_t* in;
    uint8_t* out;
    uint32_t z, cap;
    bool ok;                                     // eligible for this decoder
};

__device__ __forceinline__ Blk blk_info(uint32_t b, uint32_t nblocks, const uint8_t* src, const uint64_t* src_off,
                                        const uint32_t* src_len, uint8_t* dst, const uint64_t* dst_off,
                                        const uint32_t* dst_cap)
{
    Blk k;
    const uint32_t bb = b < nblocks ? b : 0u;
    k.in = src + src_off[bb];
    k.out = dst + dst_off[bb];
    k.z = src_len[bb];
    k.cap = dst_cap[bb];
    k.ok = b < nblocks && k.z > 0 && k.z < kMaxLen && k.cap < kMaxLen && ((uintptr_t)k.out & 15u) == 0;
    return k;
}

// 8 bytes of the block's compressed input at position p (aligned dwords,
// clamped to the block: bytes past z read as whatever lies in its last dword).
__device__ __forceinline__ uint2 in8(const Blk& k, uint32_t p)
{
    const uintptr_t a = (uintptr_t)k.in + p;
    const uintptr_t last = ((uintptr_t)k.in + k.z - 1) & ~(uintptr_t)3;
    const uintptr_t a0 = a & ~(uintptr_t)3;
    const uint32_t sh = (uint32_t)(a & 3);
    const uintptr_t c0 = a0 < last ? a0 : last, c1 = a0 + 4 < last ? a0 + 4 : last, c2 = a0 + 8 < last ? a0 + 8 : last;
    const uint32_t w0 = *(const uint32_t*)c0, w1 = *(const uint32_t*)c1, w2 = *(const uint32_t*)c2;
    return make_uint2(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh));
}

// 8 bytes of the block's own output at position p, read from L2 (agent-scope
// loads bypass this CU's vector L1: the executor stored these bytes).
__device__ __forceinline__ uint2 out8(const Blk& k, uint32_t p)
{
    const uintptr_t a = (uintptr_t)k.out + p;
    const uint32_t* a0 = (const uint32_t*)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t w0 = __hip_atomic_load((uint32_t*)a0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t w1 = __hip_atomic_load((uint32_t*)(a0 + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t w2 = sh ? __hip_atomic_load((uint32_t*)(a0 + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    return make_uint2(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh));
}

__device__ __forceinline__ void close_block(uint32_t b, bool ok, uint32_t len, uint32_t* out_len, int32_t* status,
                                            uint32_t* fallback, uint32_t* fallback_ids)
{
    if (ok) {
        out_len[b] = len;
        status[b] = 0;
    } else {
        out_len[b] = 0xFA110000u;
        status[b] = kFallback;
        const uint32_t at = atomicAdd(&fallback[0], 1u);
        fallback_ids[at] = b;
    }
}

// Blocks: quarter q of workgroup w starts with block w * 4 + q; each next
// one is a ticket the parser draws from a counter in the caller's scratch
// (fallback[1], zero on entry) and passes to the other waves through
// S.bq[q][g mod 4] -- quarters that drew small blocks take more of them, so a
// batch of mixed sizes (C4: 4-256 KiB) finishes together.

struct Args {
    const uint8_t* src;
    const uint64_t* src_off;
    const uint32_t* src_len;
    uint8_t* dst;
    const uint64_t* dst_off;
    const uint32_t* dst_cap;
    uint32_t* out_len;
    int32_t* status;
    uint32_t* fallback;
    uint32_t* fallback_ids;
    uint32_t nblocks;
};

// ---------------------------------------------------------------------------
// Parser wave
// ---------------------------------------------------------------------------
enum { PH_DEC = 0, PH_LIT = 1, PH_PUB = 2, PH_TRL = 3, PH_END = 4, PH_FIN = 5 };
constexpr uint32_t kBadRun = 0xFFFFFFFFu;

// Zero bytes from input position at0 on (length extensions of long runs and
// matches, lib/minilzo.c:3371-3377, :3464-3470), for the lanes with go; the
// count, or kBadRun past the input or past 2^24 bytes.  While it waits for
// the loader, the quarter publishes at as its input position: the zeros
// before it are no longer needed.
__device__ uint32_t zero_run(QuadLds& S, uint32_t q, uint32_t stgb, uint32_t gt, uint32_t zr, uint32_t z,
                             uint32_t at0, bool go, bool lead)
{
    uint32_t zc = 0;
    for (uint32_t spin = 0; any(go); spin++) {
        const uint32_t at = at0 + zc;
        if (go && (at >= z || zc > (1u << 24) || spin > (1u << 22))) {
            go = false;
            zc = kBadRun;
        }
        const uint32_t c = ld_acq(&S.stg[q]);
        const uint32_t staged = (c & 0xFF000000u) == gt ? c & 0xFFFFFFu : 0u;
        const bool wait = go && staged < umin(at + 8, zr);
        if (any(wait)) {
            if (wait && lead)
                st_rel(&S.pip[q], gt | at);
            __builtin_amdgcn_s_sleep(1);
        }
        const bool rd = go && !wait;
        const uint2 v = rd ? rd8(stgb + (at & kStageMask)) : make_uint2(0, 0);
        const uint64_t x = ((uint64_t)v.y << 32) | v.x;
        const uint32_t nz = x ? (uint32_t)__builtin_ctzll(x) >> 3 : 8u;
        if (rd) {
            zc += nz;
            go = nz == 8;
        }
    }
    return zc;
}

__device__ void parser_wave(QuadLds& S, const Args& A)
{
    const uint32_t l = lane_id(), q = l >> 4, j = l & 15;
    const uint32_t w = blockIdx.x;
    const uint32_t ringb = lds_off(S.ring[q]);
    const uint32_t stgb = lds_off(S.stage[q]);
    const bool lead = j == 0;                    // the quarter's lane for records and counters

    uint32_t g = 0, b = w * kQ + q;
    Blk k = blk_info(b, A.nblocks, A.src, A.src_off, A.src_len, A.dst, A.dst_off, A.dst_cap);
    uint32_t ph = b < A.nblocks ? (k.ok ? PH_DEC : PH_END) : PH_FIN;
    bool err = !k.ok;
    uint32_t st = ST_F, ip = 0, op = 0;
    uint32_t lit_rem = 0, lit_src = 0;
    uint32_t m_dst = 0, m_rem = 0, m_d = 0, m_s = 0;
    uint32_t rcnt = 0, fcnt = 0, last_pub = 0;
    // caches of the other waves' counters
    uint32_t c_stg = 0, c_ex = 0, c_head = 0, c_fdone = 0;
    uint32_t idle = 0;

    for (;;) {
        if (!any(ph != PH_FIN))
            break;
        c_stg = ld_acq(&S.stg[q]);
        c_ex = ld_acq(&S.expos[q]);
        c_head = ld_acq(&S.rec_head[q]);
        c_fdone = ld_acq(&S.far_done[q]);
        const uint32_t gt = (g & 0xFFu) << 24;
        // input staged for this generation, and how far the executor is
        const uint32_t staged = (c_stg & 0xFF000000u) == gt ? c_stg & 0xFFFFFFu : 0u;
        const uint32_t zr = k.z + 16;                // (the loader stages past z, clamped)
        const uint32_t exo = (c_ex & 0xFF000000u) == gt ? c_ex & 0xFFFFFFu : 0u;
        const bool exgen = (c_ex & 0xFF000000u) == gt;  // the executor is on this block
        const uint32_t room = exgen ? exo + kLag : 0u;  // writes end at or below this
        bool progress = false;

        // ---- P1: a literal run at ip (state A or F) ------------------------
        // lib/minilzo.c:3357-3414
        {
            const bool want = ph == PH_DEC && (st == ST_A || st == ST_F);
            const bool can = want && staged >= umin(ip + kNeed, zr);
            uint4 v = make_uint4(0, 0, 0, 0);
            if (any(can))
                v = rd16(stgb + (ip & kStageMask));
            const uint32_t t = v.x & 0xFFu, b1 = (v.x >> 8) & 0xFFu;
            const bool first_long = st == ST_F && t > 17;
            const bool run = can && (t < 16 || first_long);
            // t == 0: 15 + 255 * (zero bytes) + the next byte; zero bytes are rare (runs of 270+)
            const bool ext0 = run && !first_long && t == 0 && b1 == 0;
            uint32_t len = first_long ? t - 17 : t ? t + 3 : b1 + 18;
            uint32_t adv = t || first_long ? 1u : 2u;
            if (any(ext0)) {
                const uint32_t zc = zero_run(S, q, stgb, gt, zr, k.z, ip + 1, ext0, lead);
                if (ext0) {
                    const uint32_t at = ip + 1 + zc;
                    const bool bad = zc == kBadRun || at >= k.z;
                    if (bad)
                        err = true;
                    else {
                        // the non-zero byte is staged: zero_run read it
                        const uint32_t nz = rd8(stgb + (at & kStageMask)).x & 0xFFu;
                        len = 15 + 255 * zc + nz + 3;
                        adv = 2 + zc;
                    }
                }
            }
            if (run && !err) {
                if (ip + adv + len > k.z || op + len > k.cap)
                    err = true;                  // (input or output overrun: the exact decoder)
                else {
                    lit_src = ip + adv;
                    lit_rem = len;
                    ip += adv + len;
                    st = first_long && len < 4 ? ST_C : ST_B;
                    ph = PH_LIT;
                    progress = true;
                }
            }
            if (run && err)
                ph = PH_END;
            // the first byte is 16 or 17: a match at the top of the loop (:3367)
            if (can && st == ST_F && !run)
                st = ST_A;
        }

        // ---- P2: one pass of the literal run, written into the ring --------
        {
            const uint32_t n = umin(lit_rem, kPass);
            const bool can = ph == PH_LIT && staged >= umin(lit_src + n + 16, zr) && op + n <= room;
            if (any(can)) {
                const uint32_t t0 = 8 * j;
                const bool mine = can && t0 < n;
                const uint2 v = mine ? rd8(stgb + ((lit_src + t0) & kStageMask)) : make_uint2(0, 0);
                if (mine)
                    ring_put(ringb, op + t0, v, umin(8u, n - t0));
                if (can) {
                    op += n;
                    lit_src += n;
                    lit_rem -= n;
                    ph = lit_rem ? PH_LIT : PH_DEC;
                    progress = true;
                }
            }
            // a long literal stretch tells the executor where it stands
            const bool sync = (ph == PH_LIT || ph == PH_DEC || ph == PH_TRL) && op >= last_pub + kSync &&
                              rcnt - c_head < kRec;
            if (any(sync)) {
                if (sync && lead)
                    S.rec[q][rcnt % kRec] = make_uint2(op | (RK_SYNC << 24), 0);
                if (sync) {
                    rcnt++;
                    last_pub = op;
                }
            }
        }

        // ---- P3: the match at ip (lib/minilzo.c:3416-3668) -----------------
        {
            const bool want = ph == PH_DEC && st != ST_F;
            const bool can = want && staged >= umin(ip + kNeed, zr);
            uint4 v = make_uint4(0, 0, 0, 0);
            if (any(can))
                v = rd16(stgb + (ip & kStageMask));
            const uint32_t t = v.x & 0xFFu, b1 = (v.x >> 8) & 0xFFu, b2 = (v.x >> 16) & 0xFFu,
                           b3 = v.x >> 24, b4 = v.y & 0xFFu;
            uint32_t L, d, ilen, le;
            bool eof = false, ext0 = false;
            if (t >= 64) {                       // M2
                L = (t >> 5) + 1;
                d = 1 + ((t >> 2) & 7) + (b1 << 3);
                ilen = 2;
                le = t;
            } else if (t >= 32) {                // M3
                const bool x = (t & 31) == 0;
                ext0 = x && b1 == 0;
                L = x ? 33 + b1 : (t & 31) + 2;
                le = x ? b2 | (b3 << 8) : b1 | (b2 << 8);
                d = 1 + (le >> 2);
                ilen = x ? 4 : 3;
            } else if (t >= 16) {                // M4 (distance 0: EOF)
                const bool x = (t & 7) == 0;
                ext0 = x && b1 == 0;
                L = x ? 9 + b1 : (t & 7) + 2;
                le = x ? b2 | (b3 << 8) : b1 | (b2 << 8);
                const uint32_t raw = ((t & 8) << 11) + (le >> 2);
                eof = raw == 0;
                d = raw + 0x4000;
                ilen = x ? 4 : 3;
            } else if (st == ST_B) {             // M1 after a literal run
                L = 3;
                d = 1 + 0x800 + (t >> 2) + (b1 << 2);
                ilen = 2;
                le = t;
            } else {                             // M1 after trailing literals (ST_C), or ST_A
                L = 2;
                d = 1 + (t >> 2) + (b1 << 2);
                ilen = 2;
                le = t;
            }
            (void)b4;
            // state A with t < 16 was a literal run (P1); it only gets here when
            // P1 could not run it this step
            const bool match = can && (st != ST_A || t >= 16);
            if (any(match && ext0)) {
                const bool m3 = t < 64 && t >= 32;
                const bool go = match && ext0;
                const uint32_t zc = zero_run(S, q, stgb, gt, zr, k.z, ip + 1, go, lead);
                if (go) {
                    // t, zc zeros, the length byte, the two distance bytes: zero_run
                    // stopped at the length byte, so 8 bytes from it are staged
                    const uint32_t at = ip + 1 + zc;
                    const bool bad = zc == kBadRun || at + 3 > k.z;
                    const uint2 u = bad ? make_uint2(0, 0) : rd8(stgb + (at & kStageMask));
                    const uint32_t nb = u.x & 0xFFu;
                    L = (m3 ? 31 : 7) + 255 * zc + nb + 2;
                    le = ((u.x >> 8) & 0xFFu) | (((u.x >> 16) & 0xFFu) << 8);
                    const uint32_t raw = ((t & 8) << 11) + (le >> 2);
                    eof = !m3 && raw == 0;
                    d = m3 ? 1 + (le >> 2) : raw + 0x4000;
                    ilen = bad ? 0xFFFFFFF0u : 4 + zc;  // (bad: refused below)
                }
            }
            const uint32_t s = le & 3;
            if (match) {
                if (ilen > k.z || ip + ilen > k.z) {
                    err = true;
                } else if (eof) {
                    // EOF: the input must end exactly here (LZO_E_OK); anything
                    // else is for the exact decoder to report
                    ip += ilen;
                    err = err || ip != k.z;
                } else if (d > op || op + L + s > k.cap || ip + ilen + s > k.z) {
                    err = true;                  // look-behind, output or input overrun
                } else {
                    m_dst = op;
                    m_rem = L;
                    m_d = d;
                    m_s = s;
                    ip += ilen;
                    ph = PH_PUB;
                    progress = true;
                }
                if (eof || err)
                    ph = PH_END;
            }
        }

        // ---- P4: publish the next piece of the match -----------------------
        {
            const uint32_t n = umin(m_rem, kPiece);
            const bool far = m_d > kFarT;
            const bool can = ph == PH_PUB && m_dst + n <= room && rcnt - c_head < kRec &&
                             (!far || fcnt - c_fdone < kFarQ);
            if (any(can)) {
                if (can && lead) {
                    S.rec[q][rcnt % kRec] = make_uint2(m_dst | ((far ? RK_FAR : RK_NEAR) << 24), n | (m_d << 16));
                    if (far)
                        S.farq[q][fcnt % kFarQ] = make_uint2(m_dst | ((g & 0xFFu) << 24), n | (m_d << 16));
                }
                if (can) {
                    rcnt++;
                    fcnt += far ? 1u : 0u;
                    m_dst += n;
                    m_rem -= n;
                    last_pub = m_dst;
                    if (m_rem == 0) {
                        op = m_dst;
                        ph = m_s ? PH_TRL : PH_DEC;
                        st = ST_A;
                    }
                    progress = true;
                }
            }
        }

        // ---- P5: the 1-3 trailing literals (lib/minilzo.c:3650-3668) -------
        {
            const bool can = ph == PH_TRL && op + m_s <= room && staged >= umin(ip + 8, zr);
            if (any(can)) {
                const uint2 v = can && j == 0 ? rd8(stgb + (ip & kStageMask)) : make_uint2(0, 0);
                if (can && j == 0)
                    ring_put(ringb, op, v, m_s);
                if (can) {
                    ip += m_s;
                    op += m_s;
                    st = ST_C;
                    ph = PH_DEC;
                    progress = true;
                }
            }
        }

        // ---- P6: the end of the block: the END record, then the next block --
        {
            const bool can = ph == PH_END && rcnt - c_head < kRec;
            if (any(can)) {
                if (can && lead)
                    S.rec[q][rcnt % kRec] = make_uint2(op | ((err ? RK_ERR : RK_END) << 24), 0);
                // the next block: a ticket (one atomic per quarter), passed on in bq
                uint32_t tk = 0;
                if (can && lead)
                    tk = atomicAdd(&A.fallback[1], 1u);
                tk = (uint32_t)__shfl((int)tk, (int)(q * kQL), (int)kWave);
                if (can) {
                    rcnt++;
                    g++;
                    b = gridDim.x * kQ + tk;
                    b = b < A.nblocks ? b : A.nblocks;
                    if (lead)
                        S.bq[q][g & 3] = b;
                    k = blk_info(b, A.nblocks, A.src, A.src_off, A.src_len, A.dst, A.dst_off, A.dst_cap);
                    err = !k.ok;
                    ph = b < A.nblocks ? (k.ok ? PH_DEC : PH_END) : PH_FIN;
                    st = ST_F;
                    ip = op = 0;
                    lit_rem = m_rem = 0;
                    last_pub = 0;
                    progress = true;
                }
            }
        }

        // ---- publish -------------------------------------------------------
        lds_drain();                             // (the ring bytes and records first)
        if (lead) {
            st_rel(&S.far_pub[q], fcnt);
            st_rel(&S.rec_pub[q], rcnt);
            const uint32_t need = ph == PH_LIT ? lit_src : ip;   // the lowest input byte still to read
            st_rel(&S.pip[q], ph == PH_FIN ? 0xFF000000u | kIpDone : ((g & 0xFFu) << 24) | umin(need, kIpDone - 1));
        }
        if (!any(progress)) {
            if (++idle > (1u << 24))
                break;                           // (never: a lost handshake ends the wave, the blocks stay unclosed)
            __builtin_amdgcn_s_sleep(1);
        } else
            idle = 0;
    }
    if (l == 0)
        atomicSub(&S.live, 1u);
}

// ---------------------------------------------------------------------------
// Executor wave
// ---------------------------------------------------------------------------
__device__ void executor_wave(QuadLds& S, const Args& A)
{
    const uint32_t l = lane_id(), q = l >> 4, j = l & 15;
    const uint32_t w = blockIdx.x;
    const uint32_t ringb = lds_off(S.ring[q]);
    const bool lead = j == 0;

    uint32_t g = 0, b = w * kQ + q;
    Blk k = blk_info(b, A.nblocks, A.src, A.src_off, A.src_len, A.dst, A.dst_off, A.dst_cap);
    bool fin = b >= A.nblocks;
    uint32_t head = 0, pass = 0, fseen = 0;      // records consumed, pass offset in the record, far records passed
    uint32_t pos = 0, stored = 0, drained = 0;   // bytes final, stored to HBM, stored and waited for
    uint32_t c_pub = 0, c_fdone = 0;
    uint32_t idle = 0;

    for (;;) {
        if (!any(!fin))
            break;
        c_pub = ld_acq(&S.rec_pub[q]);
        c_fdone = ld_acq(&S.far_done[q]);
        const bool has = !fin && head != c_pub;
        uint2 r = make_uint2(0, 0);
        if (any(has))
            r = rd8(lds_off(&S.rec[q][head % kRec]));
        const uint32_t kind = r.x >> 24, dst = r.x & 0xFFFFFFu, L = r.y & 0xFFFFu, d = r.y >> 16;
        bool progress = false;

        // ---- near match: one pass of up to 128 bytes ------------------------
        {
            const bool act = has && kind == RK_NEAR;
            if (any(act)) {
                const uint32_t t0 = pass + 8 * j;
                const bool mine = act && t0 < L;
                const uint32_t base = dst - d;
                // byte t of the match = byte (t mod d) of the d bytes before it
                // (d >= kPass: no byte of a pass reads another of the same pass)
                uint32_t r0 = t0;
                if (d < kPass) {
                    const float rc = __builtin_amdgcn_rcpf((float)d);
                    const uint32_t qq = (uint32_t)((float)t0 * rc);
                    r0 = t0 - qq * d;
                    r0 = r0 >= d ? r0 - d : r0;
                }
                const uint32_t sa = ring_at(ringb, base + r0);
                const uint32_t sb = ring_at(ringb, d < 8 ? base : base + r0 - d);   // (d < 8: the pattern)
                const uint32_t ss = lds_off(&S.sel[d < 8 ? d : 0][d < 8 ? r0 & 7 : 0]);
                uint2 va, vb, sel;
                if (any(mine))
                    rd8x3(sa, sb, ss, va, vb, sel);
                uint2 v;
                if (d >= 8) {
                    const uint32_t wl = d - r0;  // bytes of va before the period wraps
                    if (d >= kPass || wl >= 8)
                        v = va;
                    else {
                        // bytes [0, wl) from va, [wl, 8) from vb
                        const uint64_t ma = (1ull << (8 * wl)) - 1;
                        const uint64_t xa = ((uint64_t)va.y << 32) | va.x, xb = ((uint64_t)vb.y << 32) | vb.x;
                        const uint64_t x = (xa & ma) | (xb & ~ma);
                        v = make_uint2((uint32_t)x, (uint32_t)(x >> 32));
                    }
                } else {
                    // period 1-7: the d bytes before the match (vb), expanded from phase r0
                    v.x = __builtin_amdgcn_perm(vb.y, vb.x, sel.x);
                    v.y = __builtin_amdgcn_perm(vb.y, vb.x, sel.y);
                }
                if (mine)
                    ring_put(ringb, dst + t0, v, umin(8u, L - t0));
                if (act) {
                    pass += kPass;
                    if (pass >= L) {
                        pass = 0;
                        head++;
                        pos = dst + L;
                    } else
                        pos = dst + pass;
                    progress = true;
                }
            }
        }
        // ---- far match (the loader copies it), sync --------------------------
        {
            const bool far_ready = has && kind == RK_FAR && c_fdone > fseen;
            const bool sync = has && kind == RK_SYNC;
            if (far_ready || sync) {
                head++;
                pos = far_ready ? dst + L : dst;
                fseen += far_ready ? 1u : 0u;
                progress = true;
            }
        }
        // ---- store completed chunks to HBM ---------------------------------
        {
            const bool fl = !fin && (pos & ~(kChunk - 1)) > stored;
            if (any(fl)) {
                // the chunks stored before are complete now: the loader may read them
                __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
                drained = stored;
                for (uint32_t c = 0; any(fl && stored + c < (pos & ~(kChunk - 1))); c += kChunk) {
                    const bool doit = fl && stored + c < (pos & ~(kChunk - 1));
#pragma unroll
                    for (uint32_t i = 0; i < kChunk / 256; i++) {
                        const uint32_t p = stored + c + 256 * i + 16 * j;
                        const uint4 v = doit ? rd16(ring_at(ringb, p)) : make_uint4(0, 0, 0, 0);
                        if (doit)
                            *(uint4*)(k.out + p) = v;
                    }
                }
                if (fl)
                    stored = pos & ~(kChunk - 1);
            }
        }
        // ---- end of the block ------------------------------------------------
        {
            const bool end = has && (kind == RK_END || kind == RK_ERR);
            if (any(end)) {
                const bool ok = kind == RK_END;
                if (end && ok) {
                    // the last, partial chunk: whole 16-byte pieces, then the tail
                    for (uint32_t p0 = stored; any(end && p0 < dst); p0 += 256) {
                        const uint32_t p = p0 + 16 * j;
                        if (end && p < dst) {
                            const uint4 v = rd16(ring_at(ringb, p));
                            const uint32_t nb = umin(16u, dst - p);
                            uint8_t* o = k.out + p;
                            if (nb == 16)
                                *(uint4*)o = v;
                            else {
                                uint32_t wv[4] = {v.x, v.y, v.z, v.w};
                                for (uint32_t i = 0; i < nb; i++)
                                    o[i] = (uint8_t)(wv[i >> 2] >> (8 * (i & 3)));
                            }
                        }
                    }
                }
                if (end && lead)
                    close_block(b, ok, dst, A.out_len, A.status, A.fallback, A.fallback_ids);
                if (end) {
                    head++;
                    g++;
                    b = S.bq[q][g & 3];              // (written before the END record was published)
                    k = blk_info(b, A.nblocks, A.src, A.src_off, A.src_len, A.dst, A.dst_off, A.dst_cap);
                    fin = b >= A.nblocks;
                    pos = stored = drained = pass = 0;
                    progress = true;
                }
                __builtin_amdgcn_s_waitcnt(0x0F70);   // (the next block's chunks are new lines)
            }
        }
        lds_drain();
        if (lead) {
            st_rel(&S.expos[q], ((g & 0xFFu) << 24) | pos);
            st_rel(&S.flushed[q], ((g & 0xFFu) << 24) | drained);
            st_rel(&S.rec_head[q], head);
        }
        if (!any(progress)) {
            if (++idle > (1u << 24))
                break;
            __builtin_amdgcn_s_sleep(1);
        } else
            idle = 0;
    }
    if (l == 0)
        atomicSub(&S.live, 1u);
}

// ---------------------------------------------------------------------------
// Loader wave
// ---------------------------------------------------------------------------
__device__ void loader_wave(QuadLds& S, const Args& A)
{
    const uint32_t l = lane_id(), q = l >> 4, j = l & 15;
    const uint32_t w = blockIdx.x;
    const uint32_t ringb = lds_off(S.ring[q]);
    const uint32_t stgb = lds_off(S.stage[q]);
    const bool lead = j == 0;

    uint32_t lg = 0, ld = 0;                     // staging: generation, bytes staged
    Blk k = blk_info(w * kQ + q, A.nblocks, A.src, A.src_off, A.src_len, A.dst, A.dst_off, A.dst_cap);
    uint32_t fdone = 0;                          // far records copied
    uint32_t fg = 0xFFFFFFFFu;                   // generation of the far block cached in fk
    Blk fk = k;
    uint32_t idle = 0;

    for (;;) {
        if (ld_acq(&S.live) <= 1 && !any(fdone != ld_acq(&S.far_pub[q])))
            break;                               // parser and executor are done
        const uint32_t pip = ld_acq(&S.pip[q]);
        const uint32_t fpub = ld_acq(&S.far_pub[q]);
        const uint32_t ex = ld_acq(&S.expos[q]);
        const uint32_t fl = ld_acq(&S.flushed[q]);
        bool progress = false;

        // the parser moved to the next block: stage that one from its start
        const uint32_t pg = pip >> 24;
        if (pg != (lg & 0xFFu) && pip != (0xFF000000u | kIpDone)) {
            lg++;
            ld = 0;
            k = blk_info(S.bq[q][lg & 3], A.nblocks, A.src, A.src_off, A.src_len, A.dst, A.dst_off, A.dst_cap);
            progress = true;
        }
        const bool pdone = (pip & 0xFFFFFFu) == kIpDone || pg != (lg & 0xFFu);
        const uint32_t pipv = pip & 0xFFFFFFu;
        // ---- staging: up to two chunks per quarter ------------------------
        const uint32_t zend = k.ok ? k.z + 16 : 0u;
        uint2 sv[2];
        bool sdo[2];
#pragma unroll
        for (uint32_t c = 0; c < 2; c++) {
            const uint32_t at = ld + c * kStageChunk;
            sdo[c] = !pdone && k.ok && at < zend && at + kStageChunk <= pipv + kStage;
            sv[c] = sdo[c] ? in8(k, at + 8 * j) : make_uint2(0, 0);
        }
        // ---- far copies: one record per quarter ---------------------------
        const bool fhas = fdone != fpub;
        uint2 fr = make_uint2(0, 0);
        if (any(fhas))
            fr = rd8(lds_off(&S.farq[q][fdone % kFarQ]));
        const uint32_t fdst = fr.x & 0xFFFFFFu, fgen = fr.x >> 24, fL = fr.y & 0xFFFFu, fd = fr.y >> 16;
        // the source must be stored (and drained) by the executor of that block
        const bool fgo = fhas && (fl >> 24) == fgen && (ex >> 24) == fgen && fdst - fd + fL <= (fl & 0xFFFFFFu);
        if (any(fgo)) {
            // the far record's block: generation fgen (mod 256) of this quarter
            if (fgo && (fg & 0xFFu) != fgen) {
                uint32_t gg = fg == 0xFFFFFFFFu ? 0u : fg;
                while ((gg & 0xFFu) != fgen)
                    gg++;
                fg = gg;
                fk = blk_info(S.bq[q][fg & 3], A.nblocks, A.src, A.src_off, A.src_len, A.dst, A.dst_off,
                              A.dst_cap);
            }
        }
        uint2 fv[kPiece / kPass];
#pragma unroll
        for (uint32_t i = 0; i < kPiece / kPass; i++) {
            const uint32_t t0 = i * kPass + 8 * j;
            fv[i] = fgo && t0 < fL ? out8(fk, fdst - fd + t0) : make_uint2(0, 0);
        }
        // ---- write what arrived -------------------------------------------
#pragma unroll
        for (uint32_t c = 0; c < 2; c++) {
            if (sdo[c]) {
                const uint32_t a = (ld + c * kStageChunk + 8 * j) & kStageMask;
                wr8(stgb + a, sv[c]);
                if (a < 16)
                    wr8(stgb + kStage + a, sv[c]);
            }
        }
#pragma unroll
        for (uint32_t i = 0; i < kPiece / kPass; i++) {
            const uint32_t t0 = i * kPass + 8 * j;
            if (fgo && t0 < fL)
                ring_put(ringb, fdst + t0, fv[i], umin(8u, fL - t0));
        }
        const uint32_t nst = (sdo[0] ? 1u : 0u) + (sdo[1] ? 1u : 0u);
        if (nst) {
            ld += nst * kStageChunk;
            progress = true;
        }
        if (fgo) {
            fdone++;
            progress = true;
        }
        lds_drain();
        if (lead) {
            st_rel(&S.stg[q], ((lg & 0xFFu) << 24) | umin(ld, 0xFFFFFFu));
            st_rel(&S.far_done[q], fdone);
        }
        if (!any(progress)) {
            if (++idle > (1u << 24))
                break;
            __builtin_amdgcn_s_sleep(2);
        } else
            idle = 0;
    }
}

__global__ __launch_bounds__(3 * kWave, 3) void lzo1x_decode_quad_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off, const uint32_t* __restrict__ src_len,
    uint8_t* __restrict__ dst, const uint64_t* __restrict__ dst_off, const uint32_t* __restrict__ dst_cap,
    uint32_t* __restrict__ out_len, int32_t* __restrict__ status, uint32_t* __restrict__ fallback,
    uint32_t* __restrict__ fallback_ids, uint32_t nblocks)
{
    __shared__ QuadLds S;
    const uint32_t t = threadIdx.x;
    if (t < kQ) {
        S.bq[t][0] = blockIdx.x * kQ + t;
        S.rec_pub[t] = S.rec_head[t] = S.far_pub[t] = S.far_done[t] = 0;
        S.expos[t] = S.flushed[t] = 0;
        S.pip[t] = 0;
        S.stg[t] = 0;
    }
    if (t == 0)
        S.live = 3;
    if (t < 64) {
        // v_perm selectors: byte i of the expansion of a period-d pattern from
        // phase r is pattern byte (r + i) mod d
        const uint32_t d = t >> 3, r = t & 7;
        uint32_t s0 = 0, s1 = 0;
        if (d >= 1 && r < d) {
            for (uint32_t i = 0; i < 8; i++) {
                const uint32_t v = (r + i) % d;
                if (i < 4)
                    s0 |= v << (8 * i);
                else
                    s1 |= v << (8 * (i - 4));
            }
        }
        S.sel[d][r] = make_uint2(s0, s1);
    }
    __syncthreads();
    Args A{src, src_off, src_len, dst, dst_off, dst_cap, out_len, status, fallback, fallback_ids, nblocks};
    const uint32_t wave = __builtin_amdgcn_readfirstlane(t >> 6);
    if (wave == 0)
        parser_wave(S, A);
    else if (wave == 1)
        executor_wave(S, A);
    else
        loader_wave(S, A);
}

}  // namespace

// Workgroups of the quarter decoder: four blocks each, four per CU resident.
extern "C" int lzo_mi355x_launch_decompress_quad(const uint8_t* src, const uint64_t* src_off,
                                                 const uint32_t* src_len, uint8_t* dst,
                                                 const uint64_t* dst_off, const uint32_t* dst_cap,
                                                 uint32_t* out_len, int32_t* status, uint32_t* fallback,
                                                 uint32_t* fallback_ids, uint32_t nblocks, hipStream_t stream)
{
    if (nblocks == 0)
        return 0;
    static int cus[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64)
        dev = 0;
    if (!cus[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        cus[dev] = n;
    }
    const uint32_t want = (nblocks + kQ - 1) / kQ, resident = 4u * (uint32_t)cus[dev];
    const uint32_t grid = want < resident ? want : resident;
    hipLaunchKernelGGL(lzo1x_decode_quad_kernel, dim3(grid), dim3(3 * kWave), 0, stream, src, src_off, src_len,
                       dst, dst_off, dst_cap, out_len, status, fallback, fallback_ids, nblocks);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
