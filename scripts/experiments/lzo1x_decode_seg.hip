// lzo1x_decode_seg.hip -- the segment-row LZO1X decoder for MI355X (gfx950):
// ONE wave per block, 9.9 KB of LDS, 16 blocks per CU.
//
// The grammar is lib/minilzo.c:3308-3699.  The block
// is decoded window by window; a window is at most 64 LZO1X instructions (a
// match with its 0-3 trailing literals, or a literal run), one per lane.
//
//  1. PIECE: 256 instruction-start positions of the compressed stream (plus a
//     64-byte reach for their literals) are staged in LDS, and every
//     (position, class) node gets its successor in a u16 table: class A is the
//     top of the loop (t < 16 starts a literal run), class N follows literals
//     (t < 16 is an M1 match; B and C move the same bytes).  Instructions the
//     table does not hold -- zero length-extension bytes, EOF, runs past the
//     reach or the input -- are RARE: 0.
//  2. WALK: from the window's first node the wave follows the table, one LDS
//     read per instruction; lane k keeps the k-th node.
//  3. DECODE: lane k decodes its instruction with its exact state (B or C for
//     an M1, from lane k-1), a prefix sum gives output positions, and the
//     capacity and look-behind checks are lane-parallel.
//  4. FAR COPIES: matches more than kFarT back are copied from the block's own
//     output in HBM straight into their places in the 8 KiB LDS output ring,
//     all of a window in one load round trip.
//  5. ROWS: the window's output in rows of 64 bytes, one per lane.  Every
//     segment (the match or the literal part of an instruction) marks its
//     start in the row; a running maximum gives each byte its segment, whose
//     descriptor (8 bytes, in the table's place) gives the byte's source: a
//     staged literal, or the ring byte d back -- for a match shorter than d,
//     the congruent byte of the last period before the row.  One LDS read and
//     one write per byte; bytes whose source lies in the same row (d < 64)
//     follow in sub-passes.
//  6. FLUSH: whole 1 KiB chunks of the ring go to HBM, 16 bytes per lane.
// Rare instructions are decoded and executed on their own (byte-serial decode
// from HBM, 64-byte passes).
//
// A block this decoder does not finish exactly (malformed input, look-behind
// or capacity errors, EOF not at the end of the input, a destination not
// 16-byte aligned, empty or >= 16 MiB input) goes to the fallback list for
// lzo1x_decode_exact_kernel, which returns the reference's output and LZO_E_*
// code.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "lzo_mi355x_kernels.h"

namespace {

constexpr uint32_t kWave = 64;
constexpr uint32_t kRing = 8192;                 // recent output kept in LDS
constexpr uint32_t kRingMask = kRing - 1;
constexpr uint32_t kPiece = 256;                 // instruction starts per piece
constexpr uint32_t kReach = 320;                 // a table instruction ends by here
constexpr uint32_t kStage = 336;                 // staged input bytes (kReach + dword reads)
constexpr uint32_t kChunk = 1024;                // ring -> HBM granule (16 B per lane)
constexpr uint32_t kFarT = 4096;                 // matches from further back: far copies
constexpr uint32_t kFarSpan = 3072;              // largest window output with far copies
constexpr uint32_t kRoom = kRing - kChunk;       // unstored output the slow path lets the ring hold
constexpr int32_t kFallback = 0x7FFF0001;

#ifndef POM_SEG_ROWS
#define POM_SEG_ROWS 4
#endif
constexpr int kRows = POM_SEG_ROWS;              // rows of 64 bytes per group
constexpr uint32_t kGroup = kRows * kWave;       // output bytes per row group

// LDS: ring | stage | jump table (u16 [512] while parsing; u64 [129] segment
// descriptors while executing) | step table (u8 [512] while parsing; then 4
// rows of marks and the trash, the target of masked-out lanes)
constexpr uint32_t kStageOff = kRing;
constexpr uint32_t kJumpOff = kStageOff + kStage;
constexpr uint32_t kJumpBytes = 1040;
constexpr uint32_t kStepOff = kJumpOff + kJumpBytes;
constexpr uint32_t kStepBytes = 512;
constexpr uint32_t kMarkOff = kStepOff;
constexpr uint32_t kTrashOff = kMarkOff + 4 * kWave;
constexpr uint32_t kLdsBytes = kStepOff + kStepBytes;
static_assert(kLdsBytes * 16 <= 160 * 1024, "16 blocks per CU");
static_assert(kJumpOff % 16 == 0 && kStepOff % 16 == 0, "table alignment");
static_assert(2 * 2 * kPiece <= kJumpBytes && 8 * (2 * kWave + 1) <= kJumpBytes, "jump table / descriptors");
static_assert(kTrashOff + kWave <= kStepOff + kStepBytes, "marks and trash over the step table");

// jump entries: target node (10 bits) | steps taken (3 bits) | stopped
constexpr uint32_t kJStop = 1u << 13;

// exact instruction-start states
constexpr uint32_t ST_A = 0;                     // top of the loop
constexpr uint32_t ST_B = 1;                     // after a literal run (t < 16: 3-byte M1)
constexpr uint32_t ST_C = 2;                     // after 1-3 trailing literals (t < 16: 2-byte M1)
constexpr uint32_t ST_F = 3;                     // first byte of the stream (lib/minilzo.c:3357)

// descriptor flags (high word of a match segment's descriptor): d in bits
// 0-15, or for kPerS d in bits 0-7 and floor(65536 / d) + 1 in bits 8-24
constexpr uint32_t kPerS = 1u << 30;             // d < min(L, 256): repeats a period of d
constexpr uint32_t kFar = 1u << 31;              // copied before the rows

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ uint32_t lane_read(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }

// Inclusive prefix sum over the wave: DPP row shifts, then the row totals.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}

// Inclusive running maximum over the wave (values >= 0).
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v)
{
    v = umax(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true));
    v = umax(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true));
    v = umax(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true));
    v = umax(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true));
    v = umax(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));
    v = umax(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false));
    return v;
}

// The compressed block as a range-checked buffer: loads past its last dword
// return 0, so staging and slow decodes need no branches on the block end.
struct Src {
    __amdgpu_buffer_rsrc_t rs;
    uint32_t sh;                                 // in & 3
    uint32_t z;                                  // compressed length
};

__device__ __forceinline__ Src make_src(const uint8_t* in, uint32_t z)
{
    const uint32_t lo = uni((uint32_t)(uintptr_t)in);
    const uint32_t hi = uni((uint32_t)((uintptr_t)in >> 32));
    const uintptr_t base = (((uintptr_t)hi << 32) | lo) & ~(uintptr_t)3;
    const uint32_t sh = lo & 3u;
    const uint32_t bytes = ((sh + z - 1) & ~3u) + 4u;
    return {__builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)bytes, 0x00020000), sh, z};
}

__device__ __forceinline__ uint32_t src_byte(const Src& S, uint32_t pos)
{
    return pos < S.z ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(S.rs, pos + S.sh, 0, 0) : 0u;
}

// One instruction decoded byte by byte from HBM, any state, any extension.
// kind: 0 ok, 1 EOF (ending exactly at z), 2 refuse.
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
            x.kind = q == z ? 1 : 2;             // this decoder only ends exactly at z
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

// Step entries of the instructions starting at piece position r with bytes
// t b1 b2 b3, for class A (.x) and class N (.y): the instruction's length
// with its literals (at most 63) | the next class << 6; 0 for a rare
// instruction or one that ends past lim (the reach, or the input end).
__device__ __forceinline__ uint2 step_pair(uint32_t t, uint32_t b1, uint32_t b2, uint32_t b3, uint32_t r,
                                           uint32_t lim)
{
    const bool lo = t < 16, m2 = t >= 64, m3 = t >= 32 && t < 64, m4 = t >= 16 && t < 32;
    const bool ext = (m3 && (t & 31) == 0) || (m4 && (t & 7) == 0);
    const uint32_t w = ext ? (b2 | (b3 << 8)) : (b1 | (b2 << 8));
    const bool eof = m4 && (t & 8) == 0 && (w >> 2) == 0;
    const uint32_t ilen = (m2 || lo) ? 2u : (ext ? 4u : 3u);
    const uint32_t T = ((m2 || lo) ? t : w) & 3u;
    const uint32_t lN = ilen + T;
    const bool rN = (ext && b1 == 0) || eof || r + lN > lim;
    const uint32_t eN = rN ? 0u : lN | (T ? 0x40u : 0u);
    // class A, t < 16: a literal run of t + 3 (1-byte header) or 18 + b1 (2-byte header)
    const uint32_t lR = t ? t + 4u : 20u + b1;
    const bool rR = (t == 0 && b1 == 0) || lR > 63 || r + lR > lim;
    const uint32_t eR = rR ? 0u : lR | 0x40u;
    return make_uint2(lo ? eR : eN, eN);
}

// The jump entry of one step from node (r, c) with step entry e.
__device__ __forceinline__ uint32_t jump1(uint32_t r, uint32_t e, uint32_t node)
{
    const uint32_t nr = r + (e & 63u);
    const uint32_t tgt = (nr << 1) | (e >> 6);
    return e == 0 ? (node | kJStop) : (tgt | (1u << 10) | (nr >= kPiece ? kJStop : 0u));
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

// Make room in the ring for output up to `end` (the slow path).
__device__ __forceinline__ void room_for(uint8_t* lds, Out& O, uint32_t at, uint32_t end)
{
    if (end - O.stored > kRoom)
        flush_to(lds, O, at & ~(kChunk - 1));
}

// The dword of the block's own output holding byte pos (below O.stored, once
// this wave's stores have landed), read through L2: agent-scope load.
__device__ __forceinline__ uint32_t out_dword(const Out& O, uint32_t pos)
{
    return __hip_atomic_load((uint32_t*)(O.out + (pos & ~3u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One instruction the table does not hold: a match of L bytes from d back at
// output position x, then lit literal bytes from input position lsrc, in
// 64-byte passes with the ring flushed as it fills.  P: the staged piece.
__device__ void exec_slow(uint8_t* lds, Out& O, const Src& S, uint32_t P, uint32_t x, uint32_t L,
                          uint32_t d, uint32_t lit, uint32_t lsrc)
{
    const uint32_t l = lane_id();
    const uint32_t trash = kTrashOff + l;
    if (L && d > kRing) {
        // far: passes of 64 bytes read from HBM, below O.stored (room_for
        // keeps it kRoom behind); this wave's stores land first
        for (uint32_t j = 0; j < L; j += kWave) {
            const uint32_t c = L - j < kWave ? L - j : kWave;
            const uint32_t at = x + j;
            room_for(lds, O, at, at + c);
            __builtin_amdgcn_s_waitcnt(0x0F70);                // vmcnt(0)
            const uint32_t q = at - d + l;
            const uint32_t v = l < c ? (out_dword(O, q) >> (8 * (q & 3u))) : 0u;
            lds[l < c ? ((at + l) & kRingMask) : trash] = (uint8_t)v;
        }
        x += L;
    } else if (L && d < kWave) {
        // period d < 64: byte j is byte j mod d of the period right before x,
        // so one read serves every pass; passes are a multiple of d long
        const float rd = __builtin_amdgcn_rcpf((float)d);
        const uint32_t rm = l - d * (uint32_t)(((float)l + 0.5f) * rd);
        const uint32_t step = d * uni((uint32_t)(64.5f * rd));
        const uint8_t v = lds[(x - d + rm) & kRingMask];
        for (uint32_t j = 0; j < L; j += step) {
            const uint32_t c = L - j < step ? L - j : step;
            const uint32_t at = x + j;
            room_for(lds, O, at, at + c);
            lds[l < c ? ((at + l) & kRingMask) : trash] = v;
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
                lds[o < cg ? ((at + o) & kRingMask) : trash] = v[i];
            }
        }
        x += L;
    }
    // literals: 4 bytes a lane (256 per pass) from HBM unless staged
    for (uint32_t j = 0; j < lit; j += 4 * kWave) {
        const uint32_t c = lit - j < 4 * kWave ? lit - j : 4 * kWave;
        const uint32_t at = x + j;
        room_for(lds, O, at, at + c);
        const uint32_t q = lsrc + j;
        const bool staged = q >= P && q + c <= P + kReach;
        uint8_t v[4];
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) {
            const uint32_t o = i * kWave + l;
            v[i] = staged ? lds[kStageOff + (q - P) + (o < c ? o : 0u)] : (uint8_t)src_byte(S, q + o);
        }
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) {
            const uint32_t o = i * kWave + l;
            lds[o < c ? ((at + o) & kRingMask) : trash] = v[i];
        }
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

// (diagnostics, STAMPS) per-phase s_memtime cycle sums, 16 x u64 per block:
// 0 stage + tables, 1 walk + expansion, 2 decode + checks, 3 far copies,
// 4 rows, 5 rare instructions; counts: 8 windows, 9 instructions, 10 row
// groups, 11 sub-passes, 12 far batches, 13 rare instructions, 14 groups with
// segment starts
template <bool STAMPS>
__global__ __launch_bounds__(kWave, 4) void lzo1x_decode_seg_kernel(
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
            __builtin_amdgcn_s_waitcnt(0);                          \
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
    const uint32_t z = src_len[b];
    Out O{dst + dst_off[b], 0};
    const uint32_t cap = dst_cap[b];
    if (z == 0 || z >= (1u << 24) || ((uintptr_t)O.out & 15u)) {
        close_block(b, false, 0, out_len, status, fallback, fallback_ids);
        return;
    }
    const Src S = make_src(src + src_off[b], z);
    const uint32_t trash = kTrashOff + l;
    const uint16_t* const jump = (const uint16_t*)(lds + kJumpOff);

    uint32_t p = 0, st = ST_F;                   // next instruction start and its exact state
    uint32_t op = 0;                             // output position
    bool ok = true;
    // input words of piece pfP (lanes < kStage / 8): the next piece is loaded
    // while the current window executes
    uint32_t pfP = 0xFFFFFFFFu, pf0 = 0, pf1 = 0, pf2 = 0;
    for (;;) {
        uint32_t n = 0, cur = 0;
        bool rare = true;
        const uint32_t P = p & ~3u;
        if (st != ST_F) {
            // ---- 1. piece: stage, step table, 4-step jump table -----------------
            if (l < kStage / 8) {
                if (P != pfP) {
                    const uint32_t a0 = (S.sh + P + 8 * l) & ~3u;   // (P is dword aligned)
                    pf0 = __builtin_amdgcn_raw_buffer_load_b32(S.rs, a0, 0, 0);
                    pf1 = __builtin_amdgcn_raw_buffer_load_b32(S.rs, a0 + 4, 0, 0);
                    pf2 = __builtin_amdgcn_raw_buffer_load_b32(S.rs, a0 + 8, 0, 0);
                }
                *(uint2*)(lds + kStageOff + 8 * l) =
                    make_uint2(__builtin_amdgcn_alignbyte(pf1, pf0, S.sh), __builtin_amdgcn_alignbyte(pf2, pf1, S.sh));
            }
            pfP = P;
            {
                // lane l: nodes 8l .. 8l + 7 (positions 4l .. 4l + 3, both classes)
                const uint32_t lim = z - P < kReach ? z - P : kReach;
                const uint32_t d0 = *(const uint32_t*)(lds + kStageOff + 4 * l);
                const uint32_t d1 = *(const uint32_t*)(lds + kStageOff + 4 * l + 4);
                uint32_t e8[8], jv[8];
#pragma unroll
                for (uint32_t j = 0; j < 4; j++) {
                    const uint32_t w = __builtin_amdgcn_alignbyte(d1, d0, j);
                    const uint32_t r = 4 * l + j;
                    const uint2 sp = step_pair(w & 0xFF, (w >> 8) & 0xFF, (w >> 16) & 0xFF, w >> 24, r, lim);
                    e8[2 * j] = sp.x;
                    e8[2 * j + 1] = sp.y;
                    jv[2 * j] = jump1(r, sp.x, 2 * r);
                    jv[2 * j + 1] = jump1(r, sp.y, 2 * r + 1);
                }
                *(uint2*)(lds + kStepOff + 8 * l) =
                    make_uint2(e8[0] | (e8[1] << 8) | (e8[2] << 16) | (e8[3] << 24),
                               e8[4] | (e8[5] << 8) | (e8[6] << 16) | (e8[7] << 24));
                *(uint4*)(lds + kJumpOff + 16 * l) = make_uint4(jv[0] | (jv[1] << 16), jv[2] | (jv[3] << 16),
                                                                jv[4] | (jv[5] << 16), jv[6] | (jv[7] << 16));
                // two doublings in place (a wave's LDS reads all issue before its
                // writes): 2, then 4 steps, stopping at a rare node or the exit
#pragma unroll
                for (int round = 0; round < 2; round++) {
                    uint32_t nx[8];
#pragma unroll
                    for (int i = 0; i < 8; i++)
                        nx[i] = jump[(jv[i] & kJStop) ? 0u : (jv[i] & 1023u)];
#pragma unroll
                    for (int i = 0; i < 8; i++) {
                        const uint32_t s2 = ((jv[i] >> 10) & 7u) + ((nx[i] >> 10) & 7u);
                        jv[i] = (jv[i] & kJStop) ? jv[i] : ((nx[i] & (1023u | kJStop)) | (s2 << 10));
                    }
                    *(uint4*)(lds + kJumpOff + 16 * l) = make_uint4(jv[0] | (jv[1] << 16), jv[2] | (jv[3] << 16),
                                                                    jv[4] | (jv[5] << 16), jv[6] | (jv[7] << 16));
                }
            }
            STAMP(0);
            COUNT(8, 1);
            // ---- 2. walk: up to 4 instructions a jump; lane k keeps the k-th node
            // when a jump starts there (one exit, one ballot a step)
            uint32_t cv = ((p - P) << 1) | (st == ST_A ? 0u : 1u);
            uint32_t nv = 0, jw = 0, mine = 0, hd = 0;
            uint64_t go;
            do {
                jw = jump[cv];
                const uint32_t s = (jw >> 10) & 7u;
                const bool me = l == nv;
                mine = me ? cv : mine;
                hd = me ? s : hd;
                nv += s;
                cv = jw & 1023u;
                go = __ballot(!(jw & kJStop) && nv <= kWave - 4);
            } while (go);
            const uint32_t nwalk = uni(nv);
            n = nwalk;
            cur = uni(cv);
            rare = (uni(jw) & kJStop) && (cur >> 1) < kPiece;
            {
                // the nodes between jump starts: one step from the lane before, three rounds
                uint32_t res = (l < n && hd != 0) ? 1u : 0u;
#pragma unroll
                for (int i = 0; i < 3; i++) {
                    const uint32_t pm = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mine, 0x138, 0xF, 0xF, true);
                    const uint32_t pr = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)res, 0x138, 0xF, 0xF, true);
                    const bool take = l < n && !res && pr;
                    const uint32_t e = lds[kStepOff + (pm & 511u)];
                    const uint32_t nn = ((((pm & 511u) >> 1) + (e & 63u)) << 1) | (e >> 6);
                    mine = take ? nn : mine;
                    res = take ? 1u : res;
                }
            }
            STAMP(1);
            COUNT(9, nwalk);

            if (n) {
                // ---- 3. decode with exact states; positions; checks ------------------
                const bool act = l < n;
                const uint32_t r = act ? (mine >> 1) : 0u;
                const uint32_t a = r & ~3u;
                const uint32_t w = __builtin_amdgcn_alignbyte(*(const uint32_t*)(lds + kStageOff + a + 4),
                                                              *(const uint32_t*)(lds + kStageOff + a), r & 3u);
                const uint32_t t = w & 0xFF, b1 = (w >> 8) & 0xFF, b2 = (w >> 16) & 0xFF, b3 = w >> 24;
                const bool lo = t < 16, m2 = t >= 64, m3 = t >= 32 && t < 64, m4 = t >= 16 && t < 32;
                const bool run = lo && (mine & 1u) == 0;
                const bool ext = (m3 && (t & 31) == 0) || (m4 && (t & 7) == 0);
                const uint32_t ww = ext ? (b2 | (b3 << 8)) : (b1 | (b2 << 8));
                const uint32_t ilen = (m2 || lo) ? 2u : (ext ? 4u : 3u);
                const uint32_t T = ((m2 || lo) ? t : ww) & 3u;
                const uint32_t nst = run ? ST_B : (T ? ST_C : ST_A);
                // the exact state of lane k is lane k-1's next state (wave_shr:1)
                const uint32_t prv = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)nst, 0x138, 0xF, 0xF, true);
                const uint32_t s = l == 0 ? st : prv;
                const uint32_t L = !act ? 0u
                                 : run ? 0u
                                 : m2 ? (t >> 5) + 1u
                                 : m3 ? (ext ? 31u + b1 : (t & 31u)) + 2u
                                 : m4 ? (ext ? 7u + b1 : (t & 7u)) + 2u
                                 : (s == ST_B ? 3u : 2u);
                const uint32_t d = m2 ? 1u + ((t >> 2) & 7u) + (b1 << 3)
                                 : m3 ? 1u + (ww >> 2)
                                 : m4 ? ((t & 8u) << 11) + (ww >> 2) + 0x4000u
                                 : (s == ST_B ? 0x801u : 1u) + (t >> 2) + (b1 << 2);
                const uint32_t lit = !act ? 0u : run ? (t ? t + 3u : 18u + b1) : T;
                const uint32_t lrel = r + (run ? (t ? 1u : 2u) : ilen);   // literal start, piece-relative
                const uint32_t tot = L + lit;
                const uint32_t incl = wave_incl_scan(tot);
                const uint32_t ok0 = op + incl - tot;            // this instruction's output position
                const bool far = L != 0 && d > kFarT;
                uint32_t span = lane_read(incl, n - 1);
                // a window with far copies keeps its output within kFarSpan (ring
                // slots and HBM visibility, see the far copies below)
                const uint64_t fm0 = __ballot(act && far);
                bool slow1 = false;
                if (fm0 && span > kFarSpan) {
                    const uint64_t over = __ballot(act && incl > kFarSpan);
                    const uint32_t cut = (uint32_t)__builtin_ctzll(over);
                    if (cut == 0) {
                        slow1 = true;                    // a far match over kFarSpan: alone, slow
                        n = 1;
                    } else {
                        n = cut;
                    }
                    // resume at node n (its exact state is lane n - 1's next state)
                    if (n < nwalk) {
                        cur = uni(lane_read(mine, n));
                        rare = false;
                    }
                    span = lane_read(incl, n - 1);
                }
                const bool act2 = l < n;
                // capacity (NEED_OP) and look-behind (TEST_LB), lane-parallel
                const bool bad = act2 && (op + incl > cap || (L != 0 && d > ok0));
                if (__ballot(bad) != 0 || op + span > cap) {
                    ok = false;
                    break;
                }
                const uint32_t stn = lane_read(nst, n - 1);     // the state after the window
                if (slow1) {
                    exec_slow(lds, O, S, P, op, lane_read(L, 0), lane_read(d, 0), lane_read(lit, 0),
                              P + lane_read(lrel, 0));
                    op += span;
                    p = P + (cur >> 1);
                    st = stn;
                    continue;
                }
                // the next piece's words, unless a rare instruction comes first
                if (!rare) {
                    const uint32_t nP = (P + (cur >> 1)) & ~3u;
                    if (l < kStage / 8) {
                        const uint32_t a0 = (S.sh + nP + 8 * l) & ~3u;
                        pf0 = __builtin_amdgcn_raw_buffer_load_b32(S.rs, a0, 0, 0);
                        pf1 = __builtin_amdgcn_raw_buffer_load_b32(S.rs, a0 + 4, 0, 0);
                        pf2 = __builtin_amdgcn_raw_buffer_load_b32(S.rs, a0 + 8, 0, 0);
                    }
                    pfP = nP;
                }
                const uint32_t O0 = op, O1 = op + span;
                const bool farl = act2 && far;
                const uint64_t fm = __ballot(farl);
                flush_to(lds, O, O0 & ~(kChunk - 1));
                STAMP(2);
                // ---- 4. far copies: 4 bytes a lane, one load round trip per 1 KiB
                if (fm) {
                    // Sources are more than kFarT back: below O1 - kFarT <= O0 - kChunk
                    // < O.stored, so in HBM; the ring slots of [O0, O1) hold output
                    // older than O1 - kRing < O.stored, which no near source of this
                    // window reads (>= O0 - kFarT - kGroup).
                    __builtin_amdgcn_s_waitcnt(0x0F70);            // vmcnt(0): the stores landed
                    uint64_t rest = fm;
                    uint32_t k = (uint32_t)__builtin_ctzll(rest);
                    uint32_t fo = lane_read(ok0, k), fl = lane_read(L, k), fd = lane_read(d, k), c = 0;
                    bool more = true;
                    while (more) {
                        COUNT(12, 1);
                        // four passes of 256 bytes, 4 a lane, one round trip
                        uint32_t w0[4], w1[4], at[4], cnt[4], sh[4];
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            cnt[i] = 0;
                            at[i] = sh[i] = w0[i] = w1[i] = 0;
                            if (more) {
                                const uint32_t o = c + 4 * l;
                                const uint32_t left = o < fl ? fl - o : 0u;
                                cnt[i] = left < 4 ? left : 4u;
                                at[i] = fo + o;
                                const uint32_t sp = cnt[i] ? fo + o - fd : 0u;
                                sh[i] = sp & 3u;
                                w0[i] = out_dword(O, sp);
                                w1[i] = out_dword(O, sp + 4);
                                c += 4 * kWave;
                                if (c >= fl) {
                                    rest &= rest - 1;
                                    more = rest != 0;
                                    if (more) {
                                        k = (uint32_t)__builtin_ctzll(rest);
                                        fo = lane_read(ok0, k);
                                        fl = lane_read(L, k);
                                        fd = lane_read(d, k);
                                        c = 0;
                                    }
                                }
                            }
                        }
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            const uint32_t wv = __builtin_amdgcn_alignbyte(w1[i], w0[i], sh[i]);
#pragma unroll
                            for (uint32_t x = 0; x < 4; x++)
                                lds[x < cnt[i] ? ((at[i] + x) & kRingMask) : trash] = (uint8_t)(wv >> (8 * x));
                        }
                    }
                }
                STAMP(3);
                // ---- 5. rows, four at a time ----------------------------------------
                // descriptors (the jump table is free now): code 2k+1 = match of
                // lane k, 2k+2 = its literals, at kJumpOff + 8 * code
                {
                    const bool pers = L > d && d < 256;
                    const uint32_t M = pers ? (uint32_t)(65536.0f * __builtin_amdgcn_rcpf((float)d)) + 1u : 0u;
                    const uint32_t hm = far ? (d | kFar) : pers ? (d | (M << 8) | kPerS) : d;
                    *(uint2*)(lds + kJumpOff + 16 * l + 8) = make_uint2(ok0, hm);
                    *(uint2*)(lds + kJumpOff + 16 * l + 16) = make_uint2(kStageOff + lrel - (ok0 + L), 0u);
                    if (l == 0)                          // code 0: bytes before the window's first segment
                        *(uint2*)(lds + kJumpOff) = make_uint2(0u, kFar);
                }
                const uint32_t e1 = (act2 && L) ? ok0 : 0xFFFFFFFFu;
                const uint32_t e2 = (act2 && lit) ? ok0 + L : 0xFFFFFFFFu;
                uint32_t carry = 0;
#ifdef POM_SEG_NOROWS
                for (uint32_t R = O1; R < O1; R += kGroup) {   // (timing counterfactual: no rows)
#else
                for (uint32_t R = O0 & ~(kWave - 1); R < O1; R += kGroup) {
#endif
                    COUNT(10, 1);
                    if (R + kGroup - O.stored > kRing)
                        flush_to(lds, O, R & ~(kChunk - 1));
                    // segment codes: a running maximum over the group's marked starts
                    const uint32_t a1 = e1 - R, a2 = e2 - R;
                    uint32_t m[kRows];
#pragma unroll
                    for (int j = 0; j < kRows; j++)
                        m[j] = 0;
                    if (__ballot(a1 < kGroup || a2 < kGroup)) {
                        COUNT(14, 1);
                        if (kRows == 4)
                            *(uint32_t*)(lds + kMarkOff + 4 * l) = 0;
                        else if (kRows == 2)
                            *(uint16_t*)(lds + kMarkOff + 2 * l) = 0;
                        else
                            lds[kMarkOff + l] = 0;
                        lds[a1 < kGroup ? kMarkOff + a1 : trash] = (uint8_t)(2 * l + 1);
                        lds[a2 < kGroup ? kMarkOff + a2 : trash] = (uint8_t)(2 * l + 2);
#pragma unroll
                        for (int j = 0; j < kRows; j++)
                            m[j] = lds[kMarkOff + kWave * j + l];
#pragma unroll
                        for (int j = 0; j < kRows; j++)
                            m[j] = wave_incl_max(m[j]);
                    }
                    uint32_t g[kRows], c[kRows + 1];
                    c[0] = carry;
#pragma unroll
                    for (int j = 0; j < kRows; j++) {
                        g[j] = umax(m[j], c[j]);
                        c[j + 1] = umax(c[j], uni(lane_read(m[j], kWave - 1)));
                    }
                    carry = c[kRows];
                    uint2 dsc[kRows];
#pragma unroll
                    for (int j = 0; j < kRows; j++)
                        dsc[j] = *(const uint2*)(lds + kJumpOff + 8 * g[j]);
                    // sources: a staged literal, or the ring byte d back -- for a
                    // period d, the congruent byte of the period before the group
                    // or the segment start (x = pp - xb < kGroup)
                    uint32_t addr[kRows], wr[kRows], sp[kRows];
                    bool pd[kRows];
#pragma unroll
                    for (int j = 0; j < kRows; j++) {
                        const uint32_t pp = R + kWave * j + l;
                        const bool islit = (g[j] & 1u) == 0;
                        const uint32_t hi = dsc[j].y;
                        const bool ps = (hi & kPerS) != 0;
                        const uint32_t dd = hi & (ps ? 0xFFu : 0xFFFFu);
                        const uint32_t Mg = (hi >> 8) & 0x1FFFFu;
                        // (a segment that started before the group: R; a literal's
                        // xb does not matter)
                        const uint32_t xb = umax(R, dsc[j].x);
                        const uint32_t x = pp - xb;
                        const uint32_t rm = ps ? x - __umul24(dd, __umul24(x, Mg) >> 16) : x;
                        sp[j] = xb - dd + rm;
                        const bool act3 = pp < O1 && !(hi & kFar);   // (code 0 is kFar)
                        const bool rdy = islit || sp[j] < R;
                        addr[j] = islit ? dsc[j].x + pp : (sp[j] & kRingMask);
                        wr[j] = (act3 && rdy) ? (pp & kRingMask) : trash;
                        addr[j] = (act3 && rdy) ? addr[j] : trash;
                        pd[j] = act3 && !rdy;
                    }
                    uint8_t v[kRows];
#pragma unroll
                    for (int j = 0; j < kRows; j++)
                        v[j] = lds[addr[j]];
#pragma unroll
                    for (int j = 0; j < kRows; j++)
                        lds[wr[j]] = v[j];
                    uint64_t pm[kRows];
                    uint64_t pany = 0;
#pragma unroll
                    for (int j = 0; j < kRows; j++)
                        pany |= (pm[j] = __ballot(pd[j]));
#ifdef POM_SEG_NOSUB
                    pany = 0;                            // (timing counterfactual: output not exact)
#endif
                    if (pany) {
                        // sources inside the group: each sub-pass moves the bytes
                        // whose source byte is final
                        for (;;) {
                            COUNT(11, 1);
                            uint32_t ad2[kRows], wr2[kRows];
                            bool go2[kRows];
#pragma unroll
                            for (int j = 0; j < kRows; j++) {
                                if (!pm[j]) {
                                    go2[j] = false;
                                    ad2[j] = wr2[j] = trash;
                                    continue;
                                }
                                const uint32_t o = sp[j] - R;
                                uint64_t sel = pm[0];
#pragma unroll
                                for (int jj = 1; jj < kRows; jj++)
                                    sel = o >= kWave * jj ? pm[jj] : sel;
                                go2[j] = pd[j] && !((sel >> (o & 63u)) & 1ull);
                                ad2[j] = go2[j] ? (sp[j] & kRingMask) : trash;
                                wr2[j] = go2[j] ? ((R + kWave * j + l) & kRingMask) : trash;
                            }
                            uint8_t v2[kRows];
#pragma unroll
                            for (int j = 0; j < kRows; j++)
                                v2[j] = lds[ad2[j]];
#pragma unroll
                            for (int j = 0; j < kRows; j++)
                                lds[wr2[j]] = v2[j];
                            pany = 0;
#pragma unroll
                            for (int j = 0; j < kRows; j++) {
                                pd[j] = pd[j] && !go2[j];
                                pany |= (pm[j] = __ballot(pd[j]));
                            }
                            if (!pany)
                                break;
                        }
                    }
                }
                op = O1;
                p = P + (cur >> 1);
                st = stn;
                STAMP(4);
            }
        }
        if (rare) {
            // ---- a rare instruction (or the first one), decoded from HBM ----------
            const bool staged = st != ST_F;              // (the piece at P is in LDS)
            const Ins x = decode_slow(S, p, st);
            const uint32_t kind = uni(x.kind);
            if (kind == 1) {                             // EOF exactly at the input end
                flush_tail(lds, O, op);
                break;
            }
            if (kind != 0) {
                ok = false;
                break;
            }
            const uint32_t L = uni(x.L), d = uni(x.d), lit = uni(x.lit), lsrc = uni(x.lsrc);
            if (op + L + lit > cap || (L != 0 && d > op) || op + L + lit < op) {
                ok = false;
                break;
            }
            exec_slow(lds, O, S, staged ? P : 0xFFFFF000u, op, L, d, lit, lsrc);
            op += L + lit;
            p = uni(x.next);
            st = uni(x.nst);
            STAMP(5);
            COUNT(13, 1);
        }
    }
    close_block(b, ok, op, out_len, status, fallback, fallback_ids);
    if (STAMPS && l == 0)
        for (int i = 0; i < 16; i++)
            dbg[(size_t)b * 16 + i] = acc[i];
#undef STAMP
#undef COUNT
}

}  // namespace

extern "C" int lzo_mi355x_launch_decompress_seg(const uint8_t* src, const uint64_t* src_off,
                                                const uint32_t* src_len, uint8_t* dst,
                                                const uint64_t* dst_off, const uint32_t* dst_cap,
                                                uint32_t* out_len, int32_t* status,
                                                uint32_t* fallback, uint32_t* fallback_ids,
                                                uint32_t nblocks, hipStream_t stream)
{
    if (nblocks == 0)
        return 0;
    hipLaunchKernelGGL(lzo1x_decode_seg_kernel<false>, dim3(nblocks), dim3(kWave), 0, stream, src, src_off,
                       src_len, dst, dst_off, dst_cap, out_len, status, fallback, fallback_ids, nblocks, nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Diagnostic: the same decoder with per-phase cycle stamps (see the kernel).
extern "C" int lzo_mi355x_debug_decompress_seg_stamps(const uint8_t* src, const uint64_t* src_off,
                                                      const uint32_t* src_len, uint8_t* dst,
                                                      const uint64_t* dst_off, const uint32_t* dst_cap,
                                                      uint32_t* out_len, int32_t* status,
                                                      uint32_t* fallback, uint32_t* fallback_ids,
                                                      uint32_t nblocks, uint64_t* stamps,
                                                      hipStream_t stream)
{
    if (nblocks == 0)
        return 0;
    hipLaunchKernelGGL(lzo1x_decode_seg_kernel<true>, dim3(nblocks), dim3(kWave), 0, stream, src, src_off,
                       src_len, dst, dst_off, dst_cap, out_len, status, fallback, fallback_ids, nblocks, stamps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
