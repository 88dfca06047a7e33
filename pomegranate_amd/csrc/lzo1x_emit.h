// lzo1x_emit.h -- LZO1X-1 token emission shared by the two encoders
// (lzo1x_kernels.hip: any block size; lzo1x_encode_fast.hip: blocks up to
// 64 KiB).  One wave writes the token stream into an LDS staging ring and
// flushes it to HBM 64 bytes per instruction.  Byte layout follows
// lib/minilzo.c:3023-3145 (literal runs, match tokens) and :3175-3203 (tail,
// EOF marker); SURVEY.md Appendix A.1.
#ifndef POM_LZO1X_EMIT_H
#define POM_LZO1X_EMIT_H 1

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

namespace emit {

constexpr int kWave = 64;

__device__ __forceinline__ uint32_t lane()
{
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
// Compiler-only ordering point: one wave's DS instructions execute in order.
__device__ __forceinline__ void order() { __atomic_signal_fence(__ATOMIC_SEQ_CST); }

constexpr uint32_t kSlots = 1u << 14;            // D_BITS 14, lib/minilzo.c:2627

__device__ __forceinline__ uint32_t slot_primary(uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3)
{
    uint32_t v = (((b3 << 6) ^ b2) << 5) ^ b1;     // DX3(p,5,5,6), lib/minilzo.c:2697-2704
    v = (v << 5) ^ b0;
    return ((v * 33u) >> 5) & (kSlots - 1);       // D_INDEX1, :2629
}

__device__ __forceinline__ uint32_t slot_secondary(uint32_t h)
{
    return (h & 0x7FFu) ^ 0x201Fu;                // D_INDEX2, :2630
}

// Output state of one block.  stage is an LDS ring of smask + 1 bytes; the
// last two bytes stay staged because a following short literal run ORs its
// length into out[op-2] (lib/minilzo.c:3027-3030, 3181-3182).
struct Enc {
    const uint8_t* in;
    uint32_t n;
    uint8_t* out;
    uint32_t cap;
    uint8_t* stage;
    uint32_t smask;     // ring size - 1
    uint32_t sflush;    // flush once this many bytes are staged
    uint32_t op, flushed;
};

__device__ __forceinline__ void flush(Enc& e, uint32_t upto)
{
    order();
    const uint32_t l = lane();
    for (uint32_t k = e.flushed; k < upto; k += kWave) {
        const uint32_t j = k + l;
        if (j < upto && j < e.cap)
            e.out[j] = e.stage[j & e.smask];
    }
    e.flushed = upto;
    order();
}

__device__ __forceinline__ void maybe_flush(Enc& e)
{
    if (e.op - e.flushed >= e.sflush + 2)
        flush(e, e.op - 2);
}

__device__ __forceinline__ void byte(Enc& e, uint32_t v)
{
    if (lane() == 0)
        e.stage[e.op & e.smask] = (uint8_t)v;
    order();
    e.op++;
}

__device__ __forceinline__ void patch(Enc& e, uint32_t v)
{
    if (lane() == 0)
        e.stage[(e.op - 2) & e.smask] |= (uint8_t)v;
    order();
}

__device__ __forceinline__ void zeros(Enc& e, uint32_t count)
{
    const uint32_t l = lane();
    while (count > 0) {
        const uint32_t c = count < (uint32_t)kWave ? count : (uint32_t)kWave;
        if (l < c)
            e.stage[(e.op + l) & e.smask] = 0;
        order();
        e.op += c;
        count -= c;
        maybe_flush(e);
    }
}

// ext(x): x/255 zero bytes then the remainder (lib/minilzo.c:3034-3046)
__device__ __forceinline__ void ext(Enc& e, uint32_t x)
{
    const uint32_t z = (x - 1) / 255;
    zeros(e, z);
    byte(e, x - 255 * z);
}

__device__ __forceinline__ void lits(Enc& e, uint32_t from, uint32_t count)
{
    const uint32_t l = lane();
    while (count > 0) {
        const uint32_t c = count < (uint32_t)kWave ? count : (uint32_t)kWave;
        if (l < c)
            e.stage[(e.op + l) & e.smask] = e.in[from + l];
        order();
        e.op += c;
        from += c;
        count -= c;
        maybe_flush(e);
    }
}

// Literal-run header (lib/minilzo.c:3023-3048, tail :3179-3199)
__device__ __forceinline__ void lit_header(Enc& e, uint32_t r)
{
    if (r <= 3)
        patch(e, r);
    else if (r <= 18)
        byte(e, r - 3);
    else {
        byte(e, 0);
        ext(e, r - 18);
    }
}

// Match token (lib/minilzo.c:3064-3145)
__device__ __forceinline__ void match(Enc& e, uint32_t len, uint32_t off)
{
    if (len <= 8) {
        if (off <= 0x800) {
            const uint32_t o = off - 1;
            byte(e, ((len - 1) << 5) | ((o & 7) << 2));
            byte(e, o >> 3);
            return;
        }
        if (off <= 0x4000) {
            const uint32_t o = off - 1;
            byte(e, 0x20 | (len - 2));
            byte(e, (o & 63) << 2);
            byte(e, o >> 6);
            return;
        }
        const uint32_t o = off - 0x4000;
        byte(e, 0x10 | ((o & 0x4000) >> 11) | (len - 2));
        byte(e, (o & 63) << 2);
        byte(e, o >> 6);
        return;
    }
    uint32_t o;
    if (off <= 0x4000) {
        o = off - 1;
        if (len <= 33)
            byte(e, 0x20 | (len - 2));
        else {
            byte(e, 0x20);
            ext(e, len - 33);
        }
    } else {
        o = off - 0x4000;
        const uint32_t hi = (o & 0x4000) >> 11;
        if (len <= 9)
            byte(e, 0x10 | hi | (len - 2));
        else {
            byte(e, 0x10 | hi);
            ext(e, len - 9);
        }
    }
    byte(e, (o & 63) << 2);
    byte(e, o >> 6);
}

// Tail literals after the last match and the EOF marker (lib/minilzo.c:3175-3203).
__device__ __forceinline__ void tail_and_eof(Enc& e, uint32_t ii)
{
    const uint32_t t = e.n - ii;
    if (t > 0) {
        if (e.op == 0 && t <= 238)
            byte(e, 17 + t);
        else
            lit_header(e, t);
        lits(e, ii, t);
    }
    byte(e, 0x11);
    byte(e, 0);
    byte(e, 0);
    flush(e, e.op);
}

}  // namespace emit

}  // namespace

#endif
