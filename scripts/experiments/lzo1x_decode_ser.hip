// lzo1x_decode_ser.hip -- the table-walk LZO1X decoder for MI355X (gfx950):
// one workgroup of two waves per block, 16 blocks per CU.
//
// The block's compressed stream is taken in WINDOWS of at most 256 bytes and
// 64 instructions (lib/minilzo.c:3308-3699 is the grammar, SURVEY.md Appendix
// A.2).  The WALKER wave (wave 1) prepares window i while the EXECUTOR wave
// (wave 0) runs window i - 1; one barrier per window hands the slot over.
//
// Walker:
//  1. STAGE: the window's 384 input bytes into LDS (one dwordx2 per lane).
//  2. TABLE: every lane decodes the instructions that would start at its 4
//     positions, once as state A (top of the loop: t < 16 is a literal run)
//     and once as state B/C (after literals: t < 16 is an M1 match), into one
//     byte each: the instruction's length including its trailing literals and
//     the state after it.  Rare instructions (a zero length-extension byte,
//     literal runs over 61 bytes, EOF, the first byte) get 0, "decode slowly".
//  3. WALK: from the window's first instruction start the wave follows the
//     table, one LDS read per instruction; the list of starts goes to LDS.
// Executor:
//  4. DECODE: lane k decodes instruction k (match length, distance, literal
//     count and source); an inclusive scan gives every instruction's output
//     position, and the capacity / look-behind checks are lane-parallel.
//  5. EXECUTE: one pass per instruction in order.  A pass moves up to 64
//     bytes, one per lane, into an 8 KiB LDS output ring: match bytes from
//     the ring (a period-d match reads byte l mod d of its period) or from a
//     far-source slot read at the window's start (more than 8 KiB back),
//     trailing literal bytes from the staged input, in the same ds_read_u8.
//     Long matches, further far sources and long literal runs take a pass
//     loop.
//  6. FLUSH: completed 1 KiB pieces of the ring go to HBM, one dwordx4 store
//     per lane.
//
// A block this decoder does not finish exactly (malformed input, look-behind
// or capacity errors, EOF not at the end of the input, a destination not
// 16-byte aligned, empty or >= 16 MiB input) is appended to the fallback list
// for lzo1x_decode_exact_kernel, which returns the reference's output and
// LZO_E_* code.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "lzo_mi355x_kernels.h"   // (built by scripts/experiments/Makefile, outside the product library)

namespace {

constexpr uint32_t kWave = 64;
constexpr uint32_t kRing = 8192;                 // recent output kept in LDS
constexpr uint32_t kRingMask = kRing - 1;
constexpr uint32_t kWin = 256;                   // table positions per window
constexpr uint32_t kStage = 384;                 // staged input bytes per window (256 + a 64-byte pass + 64)
constexpr uint32_t kChunk = 1024;                // ring -> HBM store granule (16 B per lane)
constexpr uint32_t kRoom = kRing - kChunk;       // unstored output the ring may hold
constexpr uint32_t kFastSpan = 4096;             // windows up to this output take the one-pass path
constexpr int32_t kFallback = 0x7FFF0001;

// LDS: ring | stage x2 | far-source slots | walk table (u8 [2][256]) |
// start lists x2 (u16 [64]) | window records x2 | control | trash (2 B a lane)
constexpr uint32_t kFarSlots = 4;                // far sources read ahead per window
constexpr uint32_t kStageOff = kRing;            // + kStage * (window & 1)
constexpr uint32_t kFarOff = kStageOff + 2 * kStage;
constexpr uint32_t kTabOff = kFarOff + 64 * kFarSlots;
constexpr uint32_t kListOff = kTabOff + 2 * kWin;   // + 128 * (window & 1)
constexpr uint32_t kCtlOff = kListOff + 2 * 2 * kWave;   // 2 x {P, n, eof_k, state}, then done
constexpr uint32_t kTrashOff = kCtlOff + 48;
constexpr uint32_t kLdsBytes = kTrashOff + 2 * kWave;
static_assert(kLdsBytes * 16 <= 160 * 1024, "16 blocks per CU");
static_assert(kCtlOff % 16 == 0 && kTrashOff % 16 == 0, "aligned control words");

// instruction-start states
constexpr uint32_t ST_A = 0;                     // top of the loop
constexpr uint32_t ST_B = 1;                     // after a literal run (t < 16: 3-byte M1)
constexpr uint32_t ST_C = 2;                     // after 1-3 trailing literals (t < 16: 2-byte M1)
constexpr uint32_t ST_F = 3;                     // first byte of the stream (lib/minilzo.c:3357)

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ uint32_t lane_read(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
// Inclusive prefix sum over the wave: DPP row shifts, then the row totals.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);   // row_shr:8
    const uint32_t r0 = lane_read(v, 15), r1 = lane_read(v, 31), r2 = lane_read(v, 47);
    const uint32_t row = lane_id() >> 4;
    v += (row >= 1 ? r0 : 0u) + (row >= 2 ? r1 : 0u) + (row >= 3 ? r2 : 0u);
    return v;
}

// The compressed block as a range-checked buffer: loads past its last dword
// return 0, so staging and slow decodes need no branches on the block end.
struct Src {
    __amdgpu_buffer_rsrc_t rs;
    uint32_t sh;                                 // in & 3
    uint32_t z;                                  // compressed length
    const uint8_t* base;                         // in & ~3
};

__device__ __forceinline__ Src make_src(const uint8_t* in, uint32_t z)
{
    const uint32_t lo = uni((uint32_t)(uintptr_t)in);
    const uint32_t hi = uni((uint32_t)((uintptr_t)in >> 32));
    const uintptr_t base = (((uintptr_t)hi << 32) | lo) & ~(uintptr_t)3;
    const uint32_t sh = lo & 3u;
    const uint32_t bytes = ((sh + z - 1) & ~3u) + 4u;
    return {__builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)bytes, 0x00020000), sh, z,
            (const uint8_t*)base};
}

// 4 input bytes from position pos (any alignment); bytes past z are whatever
// the last dword holds or 0 -- every caller checks positions against z.
__device__ __forceinline__ uint32_t src_dword(const Src& S, uint32_t pos)
{
    const uint32_t a = pos + S.sh;
    const uint32_t a0 = a & ~3u;
    const uint32_t w0 = __builtin_amdgcn_raw_buffer_load_b32(S.rs, a0, 0, 0);
    const uint32_t w1 = __builtin_amdgcn_raw_buffer_load_b32(S.rs, a0 + 4, 0, 0);
    return __builtin_amdgcn_alignbyte(w1, w0, a & 3u);
}

__device__ __forceinline__ uint32_t src_byte(const Src& S, uint32_t pos)
{
    return pos < S.z ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(S.rs, pos + S.sh, 0, 0) : 0u;
}

// One instruction decoded the slow way (any state, any extension), reading
// the input byte by byte.  kind: 0 ok, 1 EOF (ending exactly at z), 2 refuse.
struct Ins {
    uint32_t L, d, lit, lsrc, next, nst, kind;
};

__device__ __noinline__ Ins decode_slow(Src S, uint32_t p, uint32_t s)
{
    Ins x{0, 0, 0, 0, 0, ST_A, 2};
    const uint32_t z = S.z;
    uint32_t q = p;
    if (q >= z)
        return x;
    uint32_t t = src_byte(S, q++);
    // a length extension: zero bytes count 255 each, then base + the first
    // non-zero byte (lib/minilzo.c:3372-3382, 3503-3513, 3547-3557)
    auto ext = [&](uint32_t base, uint32_t& n) -> bool {
        uint32_t v = 0;
        for (;;) {
            if (q >= z || v > (1u << 24))
                return false;
            const uint32_t b = src_byte(S, q++);
            if (b) {
                n = v + base + b;
                return true;
            }
            v += 255;
        }
    };
    if (s == ST_F) {
        if (t > 17) {                            // :3357-3365
            x.lit = t - 17;
            x.lsrc = q;
            x.next = q + x.lit;
            x.nst = x.lit >= 4 ? ST_B : ST_C;
            x.kind = x.next < z ? 0 : 2;
            return x;
        }
        s = ST_A;
    }
    uint32_t w;
    if (t < 16) {
        if (s == ST_A) {                         // literal run, :3367-3414
            uint32_t n = t;
            if (n == 0 && !ext(15, n))
                return x;
            x.lit = n + 3;
            x.lsrc = q;
            x.next = q + x.lit;
            x.nst = ST_B;
            x.kind = x.next < z ? 0 : 2;
            return x;
        }
        const uint32_t b1 = src_byte(S, q++);   // M1, :3418-3443 (B), :3588-3613 (C)
        x.L = s == ST_B ? 3u : 2u;
        x.d = (s == ST_B ? 0x801u : 1u) + (t >> 2) + (b1 << 2);
        w = t;
    } else if (t >= 64) {                        // M2, :3447-3498
        const uint32_t b1 = src_byte(S, q++);
        x.L = (t >> 5) + 1;
        x.d = 1 + ((t >> 2) & 7) + (b1 << 3);
        w = t;
    } else if (t >= 32) {                        // M3, :3500-3537
        uint32_t n = t & 31;
        if (n == 0 && !ext(31, n))
            return x;
        x.L = n + 2;
        w = src_byte(S, q) | (src_byte(S, q + 1) << 8);
        q += 2;
        x.d = 1 + (w >> 2);
    } else {                                     // M4 / EOF, :3538-3587
        uint32_t n = t & 7;
        if (n == 0 && !ext(7, n))
            return x;
        x.L = n + 2;
        w = src_byte(S, q) | (src_byte(S, q + 1) << 8);
        q += 2;
        const uint32_t dd = ((t & 8) << 11) + (w >> 2);
        if (dd == 0) {                           // :3565-3566 / 3580-3581
            x.L = 0;
            x.next = q;
            x.kind = q == z ? 1 : 2;             // the fast path only ends exactly at z
            return x;
        }
        x.d = dd + 0x4000;
    }
    const uint32_t T = w & 3;                    // trailing literals, :3650-3667
    x.lit = T;
    x.lsrc = q;
    x.next = q + T;
    x.nst = T ? ST_C : ST_A;
    x.kind = x.next < z ? 0 : 2;
    return x;
}

// Table entry of the instruction starting with bytes t b1 b2 b3, for state A
// (a) or B/C (!a): length with trailing literals | next state << 6, or 0.
__device__ __forceinline__ uint32_t table_entry(uint32_t t, uint32_t b1, uint32_t b2, uint32_t b3, bool a)
{
    const bool lo = t < 16, m2 = t >= 64, m3 = t >= 32 && t < 64, m4 = t >= 16 && t < 32;
    const bool ext = (m3 && (t & 31) == 0) || (m4 && (t & 7) == 0);
    const uint32_t w = ext ? (b2 | (b3 << 8)) : (b1 | (b2 << 8));
    const bool eof = m4 && (t & 8) == 0 && (w >> 2) == 0;
    const uint32_t ilen = (m2 || lo) ? 2u : (ext ? 4u : 3u);
    const uint32_t T = ((m2 || lo) ? t : w) & 3u;
    const uint32_t eN = (ext && b1 == 0) || eof ? 0u : (ilen + T) | ((T ? ST_C : ST_A) << 6);
    // state A, t < 16: a literal run of t + 3 (1-byte header) or 18 + b1 (2-byte header)
    const uint32_t runlen = t ? t + 4u : 20u + b1;
    const uint32_t eA = (t == 0 && (b1 == 0 || b1 > 43)) ? 0u : runlen | (ST_B << 6);
    return (a && lo) ? eA : eN;
}

// Instruction fields from its first four bytes (callers know the table entry
// is not 0, so there is no EOF, zero extension byte or long run here).
__device__ __forceinline__ void decode_fast(uint32_t t, uint32_t b1, uint32_t b2, uint32_t b3, uint32_t s,
                                            uint32_t p, uint32_t& L, uint32_t& d, uint32_t& lit,
                                            uint32_t& lsrc)
{
    const bool lo = t < 16, m2 = t >= 64, m3 = t >= 32 && t < 64, m4 = t >= 16 && t < 32;
    const bool run = lo && s == ST_A;
    const bool ext = (m3 && (t & 31) == 0) || (m4 && (t & 7) == 0);
    const uint32_t w = ext ? (b2 | (b3 << 8)) : (b1 | (b2 << 8));
    const uint32_t ilen = (m2 || lo) ? 2u : (ext ? 4u : 3u);
    const uint32_t T = ((m2 || lo) ? t : w) & 3u;
    L = run ? 0u
            : m2 ? (t >> 5) + 1u
            : m3 ? (ext ? 31u + b1 : (t & 31u)) + 2u
            : m4 ? (ext ? 7u + b1 : (t & 7u)) + 2u
            : (s == ST_B ? 3u : 2u);
    d = m2 ? 1u + ((t >> 2) & 7u) + (b1 << 3)
           : m3 ? 1u + (w >> 2)
           : m4 ? ((t & 8u) << 11) + (w >> 2) + 0x4000u
           : (s == ST_B ? 0x801u : 1u) + (t >> 2) + (b1 << 2);
    lit = run ? (t ? t + 3u : 18u + b1) : T;
    lsrc = p + (run ? (t ? 1u : 2u) : ilen);
}

struct Out {
    uint8_t* out;
    uint32_t stored;                             // output bytes stored to HBM (a kChunk multiple until the end)
};

// Ring -> HBM: every whole chunk below `upto`.
__device__ __forceinline__ void flush_to(uint8_t* lds, Out& O, uint32_t upto)
{
    const uint32_t l = lane_id();
    for (; O.stored + kChunk <= upto; O.stored += kChunk) {
        const uint4 v = *(const uint4*)(lds + ((O.stored + 16 * l) & kRingMask));
        *(uint4*)(O.out + O.stored + 16 * l) = v;
    }
}

// The last bytes [stored, end): whole 16-byte pieces, then the lane that
// holds the end writes its bytes one by one.
__device__ void flush_tail(uint8_t* lds, Out& O, uint32_t end)
{
    flush_to(lds, O, end & ~(kChunk - 1));
    const uint32_t l = lane_id();
    const uint32_t a = O.stored + 16 * l;
    if (a + 16 <= end) {
        *(uint4*)(O.out + a) = *(const uint4*)(lds + (a & kRingMask));
    } else if (a < end) {
        for (uint32_t i = a; i < end; i++)
            O.out[i] = lds[i & kRingMask];
    }
    O.stored = end;
}

// Make room in the ring for output up to `end`.
__device__ __forceinline__ void room_for(uint8_t* lds, Out& O, uint32_t at, uint32_t end)
{
    if (end - O.stored > kRoom)
        flush_to(lds, O, at & ~(kChunk - 1));
}

// A byte of the block's own output that lies below O.stored, read through L2
// (the vector L1 holds no stale line of it): agent-scope load of its dword.
__device__ __forceinline__ uint32_t out_byte(const Out& O, uint32_t pos)
{
    const uint32_t w = __hip_atomic_load((uint32_t*)(O.out + (pos & ~3u)), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    return (w >> (8 * (pos & 3u))) & 0xFFu;
}

// ---- the row executor (ROWS): output rows of 256 bytes, 4 per lane ---------
// Every byte of a row gets an ORIGIN: an LDS byte (ring or staged input,
// kLdsF), an input position (kInF), or an output position; an output position
// inside the row is followed by pointer doubling until none is left, then one
// gather and one ds_write_b32 per lane move the row.
constexpr uint32_t kLdsF = 0x80000000u;          // origin: LDS byte address
constexpr uint32_t kInF = 0x40000000u;           // origin: compressed-input position
constexpr uint32_t kLowM = 0x3FFFFFFFu;
constexpr uint32_t kRowMax = 1u << 28;           // output positions the origins can carry
constexpr uint32_t kRowB = 4 * kWave;            // bytes per row
constexpr uint32_t kTabB = 4 * kRowB;            // the row's origin table (u32 a byte)

__device__ __forceinline__ uint32_t bperm(uint32_t lane4, uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)lane4, (int)v);
}

__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }

// Inclusive running maximum over the wave.
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v)
{
    v = umax(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true));
    v = umax(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true));
    v = umax(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true));
    v = umax(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true));
    const uint32_t r0 = lane_read(v, 15), r1 = lane_read(v, 31), r2 = lane_read(v, 47);
    const uint32_t row = lane_id() >> 4;
    v = row >= 1 ? umax(v, r0) : v;
    v = row >= 2 ? umax(v, r1) : v;
    v = row >= 3 ? umax(v, r2) : v;
    return v;
}

// The window's output [op, op + span) in rows.  Lane k holds instruction k:
// its match [ok_, ok_ + L) from d back, then lit literal bytes from lsrc.
// (diagnostics, STAMPS) cycles: 3 row set-up (flush, starts, scan,
// descriptors), 5 doubling, 6 LDS gather and row write, 7 HBM / input
// loads; counts: 10 rows, 11 doubling rounds, 12 rows with HBM or input
// bytes, 15 rows with 3+ instructions in a lane's 4 bytes
template <bool STAMPS>
__device__ __forceinline__ void row_exec(uint8_t* lds, Out& O, const Src& S, uint32_t P, uint32_t so,
                                         bool act, uint32_t ok_, uint32_t L, uint32_t d, uint32_t lit,
                                         uint32_t lsrc, uint32_t op, uint32_t span, uint64_t (&acc)[16],
                                         uint64_t& tmark)
{
#define RSTAMP(ph)                                                  \
    do {                                                            \
        if (STAMPS) {                                               \
            const uint64_t now_ = __builtin_amdgcn_s_memtime();     \
            acc[ph] += now_ - tmark;                                \
            tmark = now_;                                           \
        }                                                           \
    } while (0)
#define RCOUNT(i, v)                                                \
    do {                                                            \
        if (STAMPS)                                                 \
            acc[i] += (v);                                          \
    } while (0)
    const uint32_t l = lane_id();
    const uint32_t end = op + span;
    const uint32_t lS = ok_ + L;                 // the literal part's output start
    const bool lst = lit != 0 && lsrc >= P && lsrc + lit <= P + kStage;
    // literal origin = ((litb + p) & kLowM) | (litb & ~kLowM)
    const uint32_t litb = lst ? ((so + (lsrc - P) - lS) & kLowM) | kLdsF : ((lsrc - lS) & kLowM) | kInF;
    const bool mk1 = act && L != 0, mk2 = act && lit != 0;
    uint8_t* const mark = lds + kFarOff;         // segment starts of the row (u8 [256])
    uint32_t carry = 0;                          // segment covering the row's first byte
    for (uint32_t R0 = op & ~15u; R0 < end; R0 += kRowB) {
        // Ring slots: the row [R0, R0 + kRowB), then kTabB bytes of dead slots
        // (output already in HBM) that hold the row's origin table; output
        // from R0 + kRowB + kTabB - kRing up is in the ring, older in HBM.
        if (R0 + kRowB + kTabB - O.stored > kRing)
            flush_to(lds, O, R0 & ~(kChunk - 1));
        const uint32_t lim = R0 + kRowB + kTabB - kRing;   // (mod 2^32: compare o + kRing)
        // segment ids (2k + 1 match of k, 2k + 2 its literals; 0 = a byte this
        // window does not write) by a running maximum over the row's starts
        const bool s1 = mk1 && ok_ - R0 < kRowB, s2 = mk2 && lS - R0 < kRowB;
        uint32_t g[4] = {carry, carry, carry, carry};
        if (__ballot(s1 || s2)) {
            // (a row inside one long segment has no start: every byte is carry)
            *(uint32_t*)(mark + 4 * l) = 0;
            if (s1)
                mark[ok_ - R0] = (uint8_t)(2 * l + 1);
            if (s2)
                mark[lS - R0] = (uint8_t)(2 * l + 2);
            const uint32_t mv = *(const uint32_t*)(mark + 4 * l);
            const uint32_t h0 = mv & 0xFFu;
            const uint32_t h1 = umax(h0, (mv >> 8) & 0xFFu);
            const uint32_t h2 = umax(h1, (mv >> 16) & 0xFFu);
            const uint32_t h3 = umax(h2, mv >> 24);
            const uint32_t inc = wave_incl_max(h3);
            const uint32_t pre = umax(carry, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x138, 0xF, 0xF, true));
            carry = umax(carry, lane_read(inc, 63));
            g[0] = umax(pre, h0);
            g[1] = umax(pre, h1);
            g[2] = umax(pre, h2);
            g[3] = umax(pre, h3);
        }
        const uint32_t pb = R0 + 4 * l;
        uint32_t k[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            g[j] = pb + j < end ? g[j] : 0u;
            k[j] = g[j] ? (g[j] - 1) >> 1 : 0u;
        }
        // descriptors of the bytes' instructions: those of bytes 0 and 3 always,
        // of bytes 1 and 2 when a third instruction starts inside the lane's 4
        uint32_t D[4], B[4];
        D[0] = bperm(4 * k[0], d);
        B[0] = bperm(4 * k[0], litb);
        D[3] = bperm(4 * k[3], d);
        B[3] = bperm(4 * k[3], litb);
        D[1] = k[1] == k[0] ? D[0] : D[3];
        B[1] = k[1] == k[0] ? B[0] : B[3];
        D[2] = k[2] == k[3] ? D[3] : D[0];
        B[2] = k[2] == k[3] ? B[3] : B[0];
        const bool n1 = k[1] != k[0] && k[1] != k[3], n2 = k[2] != k[0] && k[2] != k[3];
        RCOUNT(10, 1);
        if (__ballot(n1 || n2)) {
            RCOUNT(15, 1);
            const uint32_t x1 = bperm(4 * k[1], d), y1 = bperm(4 * k[1], litb);
            const uint32_t x2 = bperm(4 * k[2], d), y2 = bperm(4 * k[2], litb);
            D[1] = n1 ? x1 : D[1];
            B[1] = n1 ? y1 : B[1];
            D[2] = n2 ? x2 : D[2];
            B[2] = n2 ? y2 : B[2];
        }
        // a match byte copies the byte d back (a period shorter than the match
        // resolves through the doubling below: reducing it to its last
        // repetition by a modulo measured slower, 0.87 against 0.84 ms on C2)
        uint32_t o[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t p = pb + j;
            const uint32_t om = p - D[j], ol = ((B[j] + p) & kLowM) | (B[j] & ~kLowM);
            // (bitwise selects: a conditional here becomes an exec-masked branch)
            const uint32_t mz = 0u - (uint32_t)(g[j] != 0), mo = 0u - (g[j] & 1u);
            o[j] = ((kLdsF | (p & kRingMask)) & ~mz) | (((om & mo) | (ol & ~mo)) & mz);
        }
        RSTAMP(3);
        // pointer doubling over the row's own bytes, through the origin table
        const uint32_t tb = (R0 + kRowB) & kRingMask;
        for (;;) {
            bool q[4];
            bool any = false;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                q[j] = (o[j] & (kLdsF | kInF)) == 0 && o[j] >= R0;
                any = any || q[j];
            }
            if (!__ballot(any))
                break;
            RCOUNT(11, 1);
            *(uint4*)(lds + ((tb + 16 * l) & kRingMask)) = make_uint4(o[0], o[1], o[2], o[3]);
            uint32_t nx[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t t = q[j] ? o[j] - R0 : 4 * l + j;
                nx[j] = *(const uint32_t*)(lds + ((tb + 4 * t) & kRingMask));
            }
#pragma unroll
            for (int j = 0; j < 4; j++)
                o[j] = q[j] ? nx[j] : o[j];
        }
        RSTAMP(5);
        // gather: LDS (ring or stage), else HBM (output older than the ring
        // keeps, read through L2 once this wave's stores landed) or the
        // compressed input
        uint32_t v[4];
        bool gl = false;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const bool lo = (o[j] & kLdsF) != 0;
            const bool hbm = !lo && !(o[j] & kInF) && o[j] + kRing < lim + kRing;
            v[j] = lds[lo ? (o[j] & kLowM) : (o[j] & kRingMask)];
            gl = gl || (o[j] & kInF) || hbm;
        }
        RSTAMP(6);
        if (__ballot(gl)) {
            RCOUNT(12, 1);
            // every lane loads 4 dwords (the output's first dword where it has
            // nothing to fetch), then waits once
            __builtin_amdgcn_s_waitcnt(0x0F70);             // vmcnt(0): this wave's stores landed
            uint32_t w[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const bool in = (o[j] & kInF) != 0;
                const bool hb = !(o[j] & (kLdsF | kInF)) && o[j] + kRing < lim + kRing;
                const uint32_t a = in ? (o[j] & kLowM) + S.sh : (hb ? o[j] : 0u);
                const uint8_t* base = in ? S.base : O.out;
                w[j] = __hip_atomic_load((const uint32_t*)(base + (a & ~3u)), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const bool in = (o[j] & kInF) != 0;
                const bool hb = !(o[j] & (kLdsF | kInF)) && o[j] + kRing < lim + kRing;
                const uint32_t a = in ? (o[j] & kLowM) + S.sh : o[j];
                const uint32_t x = (w[j] >> (8 * (a & 3u))) & 0xFFu;
                v[j] = (in || hb) ? x : v[j];
            }
            RSTAMP(7);
        }
        *(uint32_t*)(lds + (pb & kRingMask)) = v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24);
        RSTAMP(6);
    }
#undef RSTAMP
#undef RCOUNT
}

// General execution of one instruction: a match of L bytes from d back at
// output position x, then lit literal bytes from input position lsrc, in
// passes of up to 64 bytes with the ring flushed as it fills.
__device__ __forceinline__ void exec_slow(uint8_t* lds, Out& O, const Src& S, uint32_t P, uint32_t so,
                                          uint32_t x, uint32_t L, uint32_t d, uint32_t lit, uint32_t lsrc)
{
    const uint32_t l = lane_id();
    if (L && d > kRing) {
        // far: passes of 64 bytes read from HBM, below O.stored (room_for
        // keeps it kRoom behind); this wave's stores land first
        for (uint32_t j = 0; j < L; j += kWave) {
            const uint32_t c = L - j < kWave ? L - j : kWave;
            const uint32_t at = x + j;
            room_for(lds, O, at, at + c);
            __builtin_amdgcn_s_waitcnt(0x0F70);                // vmcnt(0)
            const uint32_t v = l < c ? out_byte(O, at - d + l) : 0u;
            lds[l < c ? ((at + l) & kRingMask) : kTrashOff + 2 * l] = (uint8_t)v;
        }
        x += L;
    } else if (L && d < kWave) {
        // period d < 64: byte j is byte j mod d of the period right before x,
        // so one read serves every pass; passes are a multiple of d long
        // (l mod d and 64 / d by v_rcp_f32: (l + 0.5) / d stays >= 1/126 off
        // an integer, far beyond its error)
        const float rd = __builtin_amdgcn_rcpf((float)d);
        const uint32_t rm = l - d * (uint32_t)(((float)l + 0.5f) * rd);
        const uint32_t step = d * uni((uint32_t)(64.5f * rd));
        const uint8_t v = lds[(x - d + rm) & kRingMask];
        for (uint32_t j = 0; j < L; j += step) {
            const uint32_t c = L - j < step ? L - j : step;
            const uint32_t at = x + j;
            room_for(lds, O, at, at + c);
            lds[l < c ? ((at + l) & kRingMask) : kTrashOff + 2 * l] = v;
        }
        x += L;
    } else if (L) {
        // 64 <= d <= kRing: groups of g = min(d / 64, 4) passes of 64 bytes
        // read only bytes older than the group: reads first, then writes
        const uint32_t g = d >= 4 * kWave ? 4u : d / kWave;
        for (uint32_t j = 0; j < L; j += g * kWave) {
            const uint32_t at = x + j;
            const uint32_t cg = L - j < g * kWave ? L - j : g * kWave;
            room_for(lds, O, at, at + cg);
            uint8_t v[4];
#pragma unroll
            for (uint32_t i = 0; i < 4; i++)
                v[i] = lds[(at + i * kWave + l - d) & kRingMask];
#pragma unroll
            for (uint32_t i = 0; i < 4; i++) {
                const uint32_t o = i * kWave + l;
                lds[o < cg ? ((at + o) & kRingMask) : kTrashOff + 2 * l] = v[i];
            }
        }
        x += L;
    }
    for (uint32_t j = 0; j < lit; j += kWave) {
        const uint32_t c = lit - j < kWave ? lit - j : kWave;
        const uint32_t at = x + j;
        room_for(lds, O, at, at + c);
        const uint32_t q = lsrc + j;
        uint32_t v;
        if (q + c <= P + kStage && q >= P)
            v = lds[so + (q - P) + l];
        else
            v = src_byte(S, q + l);
        lds[l < c ? ((at + l) & kRingMask) : kTrashOff + 2 * l] = (uint8_t)v;
    }
}

__device__ __forceinline__ void close_block(uint32_t b, bool ok, uint32_t len, uint32_t* out_len,
                                            int32_t* status, uint32_t* fallback, uint32_t* fallback_ids)
{
    if (lane_id() != 0)
        return;
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

// The two waves of a block's workgroup, one window apart:
//  * the WALKER (wave 1) stages window i, builds its table and walks it,
//    leaving the list of instruction starts and {P, n, eof_k, state};
//  * the EXECUTOR (wave 0) decodes and executes window i - 1 meanwhile.
// One barrier per window hands the slot over.
//
// (diagnostics) per-phase cycle stamps, 16 x u64 per block: 0 stage + table,
// 1 walk (walker), 2 decode + scan + checks, 3 one-pass instructions, 4 slow
// near matches, 5 far matches, 6 literal-only slow passes, 7 far loads and
// flushes, 13 executor's barrier waits; counts: 8 windows, 9 instructions,
// 10 slow near, 11 far, 12 slow literals
template <bool STAMPS, bool ROWS>
__global__ __launch_bounds__(2 * kWave, 8) void lzo1x_decode_ser_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ src_len, uint8_t* __restrict__ dst,
    const uint64_t* __restrict__ dst_off, const uint32_t* __restrict__ dst_cap,
    uint32_t* __restrict__ out_len, int32_t* __restrict__ status,
    uint32_t* __restrict__ fallback, uint32_t* __restrict__ fallback_ids, uint32_t nblocks,
    uint64_t* __restrict__ dbg)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
    uint64_t acc[16] = {};
    uint64_t tmark = STAMPS ? __builtin_amdgcn_s_memtime() : 0;
#define STAMP(ph)                                                   \
    do {                                                            \
        if (STAMPS) {                                               \
            const uint64_t now_ = __builtin_amdgcn_s_memtime();     \
            acc[ph] += now_ - tmark;                                \
            tmark = now_;                                           \
        }                                                           \
    } while (0)
#define COUNT(i, v)                                                 \
    do {                                                            \
        if (STAMPS)                                                 \
            acc[i] += (v);                                          \
    } while (0)
    const uint32_t b = blockIdx.x;
    if (b >= nblocks)
        return;
    const uint32_t l = lane_id();
    const uint32_t wave = uni(threadIdx.x >> 6);
    const uint32_t z = src_len[b];
    Out O{dst + dst_off[b], 0};
    const uint32_t cap = dst_cap[b];
    if (z == 0 || z >= (1u << 24) || ((uintptr_t)O.out & 15u)) {
        if (wave == 0)
            close_block(b, false, 0, out_len, status, fallback, fallback_ids);
        return;
    }
    const Src S = make_src(src + src_off[b], z);
    uint32_t* const ctl = (uint32_t*)(lds + kCtlOff);
    if (threadIdx.x == 0)
        ctl[8] = 0;                              // done: the executor closed the block
    __syncthreads();

    // walker state
    uint32_t p = 0, s = ST_F;                    // next instruction start and its state
    bool wdone = false;
    // executor state
    uint32_t op = 0;                             // output position
    bool ok = true;

    for (uint32_t i = 0;; i++) {
        if (wave == 1) {
            if (!wdone) {
                // ---- walker: window i into slot i & 1 ----------------------------
                const uint32_t so = kStageOff + kStage * (i & 1u);
                const uint32_t P = p & ~3u;
                if (l < kStage / 8) {
                    const uint32_t w0 = src_dword(S, P + 8 * l), w1 = src_dword(S, P + 8 * l + 4);
                    *(uint2*)(lds + so + 8 * l) = make_uint2(w0, w1);
                }
                {
                    const uint32_t d0 = *(const uint32_t*)(lds + so + 4 * l);
                    const uint32_t d1 = *(const uint32_t*)(lds + so + 4 * l + 4);
                    uint32_t ea = 0, en = 0;
#pragma unroll
                    for (uint32_t j = 0; j < 4; j++) {
                        const uint32_t w = __builtin_amdgcn_alignbyte(d1, d0, j);
                        const uint32_t t = w & 0xFF, b1 = (w >> 8) & 0xFF, b2 = (w >> 16) & 0xFF, b3 = w >> 24;
                        ea |= table_entry(t, b1, b2, b3, true) << (8 * j);
                        en |= table_entry(t, b1, b2, b3, false) << (8 * j);
                    }
                    *(uint32_t*)(lds + kTabOff + 4 * l) = ea;
                    *(uint32_t*)(lds + kTabOff + kWin + 4 * l) = en;
                }
                STAMP(0);
                // walk: lane k keeps the k-th start (r | state << 10).  The
                // table steps run in a tight loop with the position and state
                // in VGPRs (uniform values): VALU work plus one scalar test a
                // step, not a SALU chain; instructions the table does not hold
                // (state F, zero extension bytes, long runs, EOF) are decoded
                // byte by byte between runs of table steps
                uint32_t n = 0, mine = 0, eof_k = kWave, state = 0;
                uint32_t r = p - P;
                for (;;) {
                    uint32_t e = 1;
                    if (s != ST_F) {
                        // (one exit, one scalar test a step: a loop with several
                        // exits gets flow blocks full of SALU copies)
                        uint32_t rv = __builtin_amdgcn_mov_dpp(r, 0xE4, 0xF, 0xF, false);   // (VGPR copies)
                        uint32_t sv = __builtin_amdgcn_mov_dpp(s, 0xE4, 0xF, 0xF, false);
                        uint32_t nv = __builtin_amdgcn_mov_dpp(n, 0xE4, 0xF, 0xF, false);
                        uint64_t go;
                        do {
                            mine = l == nv ? (rv | (sv << 10)) : mine;
                            e = lds[kTabOff + (sv == ST_A ? 0u : kWin) + rv];
                            const bool t = e != 0;
                            rv += e & 63u;
                            sv = t ? e >> 6 : sv;
                            nv += t ? 1u : 0u;
                            go = __ballot(t && rv < kWin && nv < kWave);
                        } while (go);
                        r = uni(rv);
                        s = uni(sv);
                        n = uni(nv);
                        e = uni(e);
                        if (e != 0)
                            break;               // 64 starts, or past the window
                    } else {
                        mine = l == n ? (r | (s << 10)) : mine;
                    }
                    // (the call returns in VGPRs: keep the walk's state scalar)
                    const Ins x = decode_slow(S, P + r, s);
                    const uint32_t kind = uni(x.kind), nx = uni(x.next), ns = uni(x.nst);
                    n++;
                    if (kind != 0) {
                        state = kind;            // 1 EOF, 2 refuse
                        eof_k = n - 1;
                        break;
                    }
                    r = nx - P;
                    s = ns;
                    if (n >= kWave || r >= kWin)
                        break;
                }
                if (state == 0 && P + r >= z)
                    state = 2;                   // past the input without EOF
                p = P + r;
                if (l < n)
                    *(uint16_t*)(lds + kListOff + 2 * kWave * (i & 1u) + 2 * l) = (uint16_t)mine;
                if (l == 0)
                    *(uint4*)(ctl + 4 * (i & 1u)) = make_uint4(P, n, eof_k, state);
                wdone = state != 0;
                STAMP(1);
            }
        } else if (i > 0) {
            // ---- executor: window i - 1 from slot (i - 1) & 1 ----------------------
            const uint32_t j = (i - 1) & 1u;
            const uint4 c = *(const uint4*)(ctl + 4 * j);
            const uint32_t P = c.x, n = c.y, eof_k = c.z, state = c.w;
            const uint32_t so = kStageOff + kStage * j;
            bool last = state != 0;
            if (state == 2)
                ok = false;
            COUNT(8, 1);
            COUNT(9, n);
            uint32_t L = 0, d = 0, lit = 0, lsrc = 0;
            const bool act = ok && l < n && l != eof_k;
            if (act) {
                const uint32_t mine = *(const uint16_t*)(lds + kListOff + 2 * kWave * j + 2 * l);
                const uint32_t rk = mine & 1023u, sk = mine >> 10;
                const uint32_t a = rk & ~3u;
                const uint32_t d0 = *(const uint32_t*)(lds + so + a);
                const uint32_t d1 = *(const uint32_t*)(lds + so + a + 4);
                const uint32_t w = __builtin_amdgcn_alignbyte(d1, d0, rk & 3u);
                const uint32_t t = w & 0xFF, b1 = (w >> 8) & 0xFF, b2 = (w >> 16) & 0xFF, b3 = w >> 24;
                const bool slow = sk == ST_F || table_entry(t, b1, b2, b3, sk == ST_A) == 0;
                if (slow) {
                    const Ins x = decode_slow(S, P + rk, sk);
                    L = x.L;
                    d = x.d;
                    lit = x.lit;
                    lsrc = x.lsrc;
                } else {
                    decode_fast(t, b1, b2, b3, sk, P + rk, L, d, lit, lsrc);
                }
            }
            const uint32_t tot = L + lit;
            const uint32_t incl = wave_incl_scan(tot);
            const uint32_t span = lane_read(incl, 63);
            const uint32_t ok_ = incl - tot + op;            // this instruction's output position
            // capacity (NEED_OP) and look-behind (TEST_LB), lane-parallel
            const bool bad = act && (op + incl > cap || (L != 0 && d > ok_));
            if (__ballot(bad) != 0 || op + span > cap || (ROWS && op + span >= kRowMax))
                ok = false;
            STAMP(2);
            if (ok && ROWS) {
                row_exec<STAMPS>(lds, O, S, P, so, act, ok_, L, d, lit, lsrc, op, span, acc, tmark);
                op += span;
            } else if (ok) {
                const bool small = span <= kFastSpan && tot <= kWave &&
                                   (lit == 0 || (lsrc >= P && lsrc + lit <= P + kStage));
                if (span <= kFastSpan)
                    room_for(lds, O, op, op + span);
                // Far sources (more than the ring back) of small instructions:
                // read now, one slot of 64 bytes each (kFarSlots per window),
                // one round trip per window instead of one per instruction.
                // They lie below O.stored (room_for), once this wave's stores
                // have landed.
                const bool farc = act && small && L != 0 && d > kRing;
                const uint64_t farm = __ballot(farc);
                uint32_t slot = kFarSlots;
                if (farm) {
                    slot = __builtin_amdgcn_mbcnt_hi((uint32_t)(farm >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)farm, 0u));
                    __builtin_amdgcn_s_waitcnt(0x0F70);             // vmcnt(0): stores landed
                    if (farc && slot < kFarSlots) {
                        const uint32_t sp = ok_ - d;
                        const uint32_t sh = sp & 3u;
                        const uint32_t* q = (const uint32_t*)(O.out + (sp & ~3u));
                        uint32_t w[17];
#pragma unroll
                        for (int x = 0; x < 17; x++)
                            w[x] = __hip_atomic_load(q + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        uint4* dst4 = (uint4*)(lds + kFarOff + 64 * slot);
#pragma unroll
                        for (int x = 0; x < 4; x++)
                            dst4[x] = make_uint4(__builtin_amdgcn_alignbyte(w[4 * x + 1], w[4 * x], sh),
                                                 __builtin_amdgcn_alignbyte(w[4 * x + 2], w[4 * x + 1], sh),
                                                 __builtin_amdgcn_alignbyte(w[4 * x + 3], w[4 * x + 2], sh),
                                                 __builtin_amdgcn_alignbyte(w[4 * x + 4], w[4 * x + 3], sh));
                    }
                }
                const bool far1 = farc && slot < kFarSlots;
                const bool one = small && (L == 0 || d <= kRing || far1);
                const uint64_t onem = __ballot(act && one);
                STAMP(7);
                // per-lane pass constants of the one-pass instructions: match
                // bytes from (Xv + (l mod d)) & (ring mask, or none for a far
                // slot), literal bytes from the staged input
                const uint32_t M = (L != 0 && d < kWave) ? (4096u + d - 1u) / d : 0u;   // l mod d = l - d * (l * M >> 12)
                const uint32_t Xv = far1 ? kFarOff + 64 * slot : ok_ - d;
                const uint32_t Dv = far1 ? 0u : d, Mv = far1 ? 0u : M;
                const uint32_t Rv = far1 ? 0xFFFFu : kRingMask;
                const uint32_t Yv = so + (lsrc - P) - L;
                struct Pass {
                    uint32_t a, w;
                };
                // (readlanes are VALU; scalar unpacking would load the CU's one SALU)
                auto pass_of = [&](uint32_t k) -> Pass {
                    const uint32_t Z = lane_read(ok_, k), X = lane_read(Xv, k), Y = lane_read(Yv, k);
                    const uint32_t dk = lane_read(Dv, k), Mk = lane_read(Mv, k), rmask = lane_read(Rv, k);
                    const uint32_t Lk = lane_read(L, k), Lt = lane_read(tot, k);
                    const uint32_t rm = l - __umul24(dk, __umul24(l, Mk) >> 12);
                    // (bitwise selects: a conditional here becomes an exec-masked branch)
                    const uint32_t ma = 0u - (uint32_t)(l < Lk), mw = 0u - (uint32_t)(l < Lt);
                    Pass q;
                    q.a = (((X + rm) & rmask) & ma) | ((Y + l) & ~ma);
                    q.w = (((Z + l) & kRingMask) & mw) | ((kTrashOff + 2 * l) & ~mw);
                    return q;
                };
                uint32_t k = 0;
                while (k < n) {
                    // one-pass instructions k .. e1 - 1: groups of four (addresses
                    // first, then the dependent read -> write chain; LDS keeps the
                    // wave's order), then one at a time
                    const uint64_t no = ~onem >> k;
                    const uint32_t e1 = no ? k + (uint32_t)__builtin_ctzll(no) : n;
                    const uint32_t end = e1 < n ? e1 : n;
                    for (; k + 4 <= end; k += 4) {
                        const Pass q0 = pass_of(k), q1 = pass_of(k + 1), q2 = pass_of(k + 2), q3 = pass_of(k + 3);
                        lds[q0.w] = lds[q0.a];
                        lds[q1.w] = lds[q1.a];
                        lds[q2.w] = lds[q2.a];
                        lds[q3.w] = lds[q3.a];
                    }
                    for (; k < end; k++) {
                        const Pass q0 = pass_of(k);
                        lds[q0.w] = lds[q0.a];
                    }
                    if (k >= n)
                        break;
                    const uint32_t tk = lane_read(tot, k);
                    if (tk != 0) {
                        STAMP(3);
                        const uint32_t Lk = lane_read(L, k), dk = lane_read(d, k);
                        exec_slow(lds, O, S, P, so, lane_read(ok_, k), Lk, dk, lane_read(lit, k),
                                  lane_read(lsrc, k));
                        if (STAMPS) {                // (constant indices: acc stays in registers)
                            if (Lk == 0) {
                                STAMP(6);
                                COUNT(12, 1);
                            } else if (dk > kRing) {
                                STAMP(5);
                                COUNT(11, 1);
                            } else {
                                STAMP(4);
                                COUNT(10, 1);
                            }
                        }
                    }
                    k++;
                }
                STAMP(3);
                op += span;
            }
            if (!ok)
                last = true;
            if (last) {
                if (ok)
                    flush_tail(lds, O, op);
                close_block(b, ok, op, out_len, status, fallback, fallback_ids);
                if (l == 0)
                    ctl[8] = 1;
            }
        }
        __syncthreads();
        STAMP(13);
        if (ctl[8])
            break;
    }
    if (STAMPS && l == 0) {
        if (wave == 0) {
            for (int x = 2; x < 16; x++)
                dbg[(size_t)b * 16 + x] = acc[x];   // (14, 15: row executor counts)
        } else {
            dbg[(size_t)b * 16 + 0] = acc[0];
            dbg[(size_t)b * 16 + 1] = acc[1];
        }
    }
#undef STAMP
#undef COUNT
}

}  // namespace

extern "C" int lzo_mi355x_launch_decompress_ser(const uint8_t* src, const uint64_t* src_off,
                                                const uint32_t* src_len, uint8_t* dst,
                                                const uint64_t* dst_off, const uint32_t* dst_cap,
                                                uint32_t* out_len, int32_t* status,
                                                uint32_t* fallback, uint32_t* fallback_ids,
                                                uint32_t nblocks, hipStream_t stream)
{
    if (nblocks == 0)
        return 0;
    hipLaunchKernelGGL((lzo1x_decode_ser_kernel<false, false>), dim3(nblocks), dim3(2 * kWave), 0, stream, src,
                       src_off, src_len, dst, dst_off, dst_cap, out_len, status, fallback, fallback_ids,
                       nblocks, nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Diagnostic: the same decoder with per-phase cycle stamps (see the kernel).
extern "C" int lzo_mi355x_debug_decompress_ser_stamps(const uint8_t* src, const uint64_t* src_off,
                                                      const uint32_t* src_len, uint8_t* dst,
                                                      const uint64_t* dst_off, const uint32_t* dst_cap,
                                                      uint32_t* out_len, int32_t* status,
                                                      uint32_t* fallback, uint32_t* fallback_ids,
                                                      uint32_t nblocks, uint64_t* stamps,
                                                      hipStream_t stream)
{
    if (nblocks == 0)
        return 0;
    hipLaunchKernelGGL((lzo1x_decode_ser_kernel<true, false>), dim3(nblocks), dim3(2 * kWave), 0, stream, src,
                       src_off, src_len, dst, dst_off, dst_cap, out_len, status, fallback, fallback_ids,
                       nblocks, stamps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The same walker with the row executor (POM_DECODER=row).
extern "C" int lzo_mi355x_launch_decompress_row(const uint8_t* src, const uint64_t* src_off,
                                                const uint32_t* src_len, uint8_t* dst,
                                                const uint64_t* dst_off, const uint32_t* dst_cap,
                                                uint32_t* out_len, int32_t* status,
                                                uint32_t* fallback, uint32_t* fallback_ids,
                                                uint32_t nblocks, hipStream_t stream)
{
    if (nblocks == 0)
        return 0;
    hipLaunchKernelGGL((lzo1x_decode_ser_kernel<false, true>), dim3(nblocks), dim3(2 * kWave), 0, stream,
                       src, src_off, src_len, dst, dst_off, dst_cap, out_len, status, fallback,
                       fallback_ids, nblocks, nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int lzo_mi355x_debug_decompress_row_stamps(const uint8_t* src, const uint64_t* src_off,
                                                      const uint32_t* src_len, uint8_t* dst,
                                                      const uint64_t* dst_off, const uint32_t* dst_cap,
                                                      uint32_t* out_len, int32_t* status,
                                                      uint32_t* fallback, uint32_t* fallback_ids,
                                                      uint32_t nblocks, uint64_t* stamps,
                                                      hipStream_t stream)
{
    if (nblocks == 0)
        return 0;
    hipLaunchKernelGGL((lzo1x_decode_ser_kernel<true, true>), dim3(nblocks), dim3(2 * kWave), 0, stream,
                       src, src_off, src_len, dst, dst_off, dst_cap, out_len, status, fallback,
                       fallback_ids, nblocks, stamps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
