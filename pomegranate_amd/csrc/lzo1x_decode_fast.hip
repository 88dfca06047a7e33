// lzo1x_decode_fast.hip -- the throughput LZO1X decoder for MI355X (gfx950).
//
// One workgroup of two waves per block, working on pieces of kPiece bytes of
// compressed input as a pipeline:
//
//  * PARSER wave (wave 1) finds the instructions of piece q+1.. while the
//    executor runs piece q, and is also the block's only HBM writer.
//    Parse (lane = kSeg-byte input segment): the LZO1X grammar
//    (lib/minilzo.c:3308-3699) is a state machine
//    over instruction starts (pos, state), state A (top), B (after a literal
//    run) or C (after 1-3 trailing literals).  Every lane decodes
//    speculatively from kLook bytes before its segment (restarting one byte
//    later whenever the guess runs into an impossible instruction) and keeps
//    the instruction starts its final attempt visits inside its segment as
//    per-state bitmaps in registers, plus a bitmap of the starts that yield
//    two ops (a match and its trailing literals).  Each lane then walks the
//    TRUE path from its assumed entry (its predecessor's exit) until it lands
//    on one of its own starts: from there the paths agree, and the bitmaps
//    give the op count of the rest of the segment (popcounts), so no separate
//    counting walk is needed.  A scalar scan chains the true entries, walking
//    exactly only where a guess was wrong.  One more walk per lane writes the
//    ops (length, source) of the true path to one of kSlots per-block op slots
//    in global scratch.
//    Writer duty, between parse steps: copy final output from the LDS ring to
//    HBM in 1-KiB dwordx4 chunks; publish `issued` (ring slots reusable) at
//    once and `landed` (readable from HBM) when the executor needs it.
//
//  * EXECUTOR wave (wave 0) issues no stores, so its loads never queue behind
//    stores (gfx9 vmcnt retires a wave's loads and stores in one in-order
//    queue).  Per 64 ops of a published piece: a DPP prefix sum gives output
//    offsets; literal spans and far match sources are copied into an LDS
//    source buffer with one batched load round trip; source forwarding and
//    batches whose match sources all precede the batch.  Every batch is
//    produced 1 KiB per step into the LDS output ring: a lane is a 16-byte
//    chunk of one op (op starts tagged per chunk, a ballot maps every chunk to
//    its op), read with misaligned ds_read_b128:
//      - contiguous sources (literals, matches that do not overlap
//        themselves): one read;
//      - a match of period p >= 16 whose chunk wraps the period: two reads
//        (the wrapped part read p bytes lower) merged by a byte mask;
//      - a match of period 1..15: its pattern, expanded by v_perm with a
//        selector table indexed by (period, phase).
//
// Anything the fast path does not handle exactly (malformed input, lookbehind
// or capacity errors, op-list overflow, EOF not at the end, misaligned
// destination...) marks the block for the exact decoder (lzo1x_kernels.hip),
// which produces the reference's output and LZO_E_* code bit for bit.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "lzo_mi355x_kernels.h"

namespace {

constexpr int kWave = 64;
#ifndef POM_SEG
#define POM_SEG 32
#endif
#ifndef POM_LOOK
#define POM_LOOK 24
#endif
constexpr uint32_t kSeg = POM_SEG;               // input bytes per lane per piece
static_assert(kSeg <= 32, "segment starts are 32-bit bitmaps");
constexpr uint32_t kLook = POM_LOOK;             // speculative lead-in before a segment
static_assert(kLook <= kSeg, "lead-in stays inside the previous segment");
constexpr uint32_t kPiece = kWave * kSeg;        // 2 KiB of compressed input
constexpr uint32_t kStageBytes = kPiece + 64;    // + the longest non-extended instruction
// Ops per piece: an instruction that yields two ops (a match and its 1-3
// trailing literals) is at least 3 bytes, so a piece holds at most
// ceil(kPiece / 3) * 2 ops.
constexpr uint32_t kOpMax = (kPiece + 2) / 3 * 2 + 64;
static_assert(kOpMax < (1u << 16), "piece info: 16-bit op count");
#ifndef POM_SLOTS
#define POM_SLOTS 4
#endif
constexpr uint32_t kSlots = POM_SLOTS;           // parsed pieces the parser may run ahead
static_assert((kSlots & (kSlots - 1)) == 0, "slots: power of two");
#ifndef POM_WRITER_SLEEP
#define POM_WRITER_SLEEP 127                     // idle writer sleeps ~8K cycles between polls
#endif
#ifndef POM_FWD_ROUNDS
#define POM_FWD_ROUNDS 3                         // source-forwarding rounds per window
#endif
#ifndef POM_WAVES_PER_EU
#define POM_WAVES_PER_EU 8                       // 16 blocks (executor + parser wave) per CU
#endif
#ifndef POM_RING
#define POM_RING 4096
#endif
#ifndef POM_PRIO
#define POM_PRIO 1                               // final-round blocks: parser at priority 3, executor 3..0 by bytes left
#endif
#ifndef POM_PRIO_STEP
#define POM_PRIO_STEP 10240                      // executor priority drops every this many bytes left
#endif
#ifndef POM_PARSER_PRIO
#define POM_PARSER_PRIO 1                        // final-round parser wave priority (3 while it was also the writer)
#endif
#ifndef POM_LAZY_PUB
#define POM_LAZY_PUB 1                           // hand output to the writer per completed 1-KiB chunk
#endif
#ifndef POM_EXEC_SLEEP
#define POM_EXEC_SLEEP 16                        // executor waits sleep ~1K cycles between polls
#endif
#ifndef POM_DUTY_EVERY
#define POM_DUTY_EVERY 4                         // parser pass-1 iterations between writer duties
#endif
#ifndef POM_EXEC_STORES
#define POM_EXEC_STORES 1                        // the executor stores its own output (the parser only parses)
#endif
#ifndef POM_STORE_LAG
#define POM_STORE_LAG 2048                       // executor stores trail its production by this much
#endif
constexpr uint32_t kRing = POM_RING;             // recent output kept in LDS
constexpr uint32_t kRingMask = kRing - 1;
constexpr uint32_t kMirror = 32;                 // ring[0, 16) mirrored after its end (+ write spill)
#ifndef POM_SRCBUF
#define POM_SRCBUF 1024
#endif
constexpr uint32_t kSrcBytes = POM_SRCBUF;       // per-window copy of literal spans and far sources
constexpr uint32_t kSrcDw = kSrcBytes / 4;
static_assert(kSrcDw <= 4 * kWave, "source copy: at most 4 dwords per lane");
constexpr uint32_t kLitFlag = 0x80000000u;
constexpr uint32_t kLinHbm = 0x4000;             // linear source addresses from here: input in HBM
constexpr uint32_t kMaxOpLen = 1u << 25;         // 64 ops per window cannot wrap 32 bits
constexpr int32_t kFallback = 0x7FFF0001;        // status: exact decoder pending
constexpr uint32_t kInfoEof = 1u << 16;          // piece info: the piece ends with EOF
constexpr uint32_t kInfoErr = 1u << 17;          // piece info: the block needs the exact decoder
// A step covers at most 64 chunks of 16 bytes: an op read by a step whose
// first byte is xs lies at most kStepSpan bytes after xs.
constexpr uint32_t kStepSpan = 16 * kWave + 16;
// (diagnostics: why, in bits 20..23 of the piece info / the CN_REASON stamp)
enum { RS_NONE, RS_OFF_END, RS_BAD, RS_OPS, RS_DEAD, RS_EWAIT, RS_OVERRUN, RS_LOOKBEHIND,
       RS_SPACE, RS_LANDED, RS_HEAD, RS_WRITER, RS_POOL };

// parse states (instruction starts)
constexpr uint32_t ST_A = 0;   // top: t < 16 is a literal run
constexpr uint32_t ST_B = 1;   // after a literal run: t < 16 is a 3-byte M1 (dist > 0x800)
constexpr uint32_t ST_C = 2;   // after trailing literals: t < 16 is a 2-byte M1
constexpr uint32_t ST_F = 3;   // first byte of the stream (lib/minilzo.c:3357)
constexpr uint32_t kPosEnd = 0xFFFFFFF0u;        // exit marker: EOF reached / dead path
// walk outcome
constexpr uint32_t FL_OK = 0;                    // reached the segment end
constexpr uint32_t FL_EOF = 1;                   // EOF at the end of the input
constexpr uint32_t FL_DEAD = 2;                  // malformed / past the input end without EOF
constexpr uint32_t FL_UNK = 3;                   // speculative walk gave up (slow instruction)

struct __attribute__((aligned(16))) FastLds {
    // executor
    uint32_t ring[(kRing + kMirror) / 4];
    uint32_t src[kSrcDw];     // this window's literal spans and far match sources
    uint4 wop[kWave];         // window op: {o, source base (| kLitFlag: linear), first 16-B chunk, L}
    uint2 wper[kWave];        // window op: {period, floor((2^32-1)/period)}
    uint32_t flags[kWave + 4];  // per-step chunk tags (src_issue: per-dword byte flags); [kWave]: spare
                              // (+4: the fields after it stay 16-byte aligned)
    // v_perm selectors of the period-p pattern expansion (p < 16): byte i of
    // psel[0][p] selects pattern byte i mod p from dwords 1:0 (12 = zero when
    // it lies in 2:3), psel[1][p] the same from dwords 3:2.  A chunk of phase
    // r reads its 16 selectors at offset r (lib/minilzo.c:3622-3646 is the
    // byte-serial copy this replaces).
    uint32_t psel[2][16][8];
    // parser
    uint32_t stage[kStageBytes / 4];
    // hand-off words (LDS, workgroup scope)
    uint32_t produced;        // executor -> writer: output bytes final in the ring
    uint32_t issued;          // writer -> executor: stores issued (ring slots reusable)
    uint32_t landed;          // writer -> executor: output bytes stored to HBM and landed
    uint32_t need;            // executor -> writer: landed position it waits for
    uint32_t state;           // executor -> parser: 0 running, 1 finished, 2 refused
    uint32_t parsed;          // parser -> executor: pieces whose ops are in their slot
    uint32_t consumed;        // executor -> parser: pieces whose slot is free again
    uint32_t pinfo[kSlots];   // per slot: op count | kInfoEof | kInfoErr
    uint32_t opset;           // this workgroup's op-slot set (from the pool)
    uint32_t done;            // waves done with the block (the second one closes it)
    uint32_t why;             // executor's refusal reason
};

constexpr uint32_t kRingOff = 0;                                  // offsetof(FastLds, ring)
constexpr uint32_t kSrcOff = kRing + kMirror;                     // offsetof(FastLds, src)
static_assert(offsetof(FastLds, ring) == kRingOff, "layout");
static_assert(offsetof(FastLds, src) == kSrcOff, "layout");
constexpr uint32_t kLdsMask = 0x3FFF;                              // LDS-linear address space
static_assert(sizeof(FastLds) <= kLdsMask + 1 && kLdsMask + 1 == kLinHbm,
              "linear LDS addresses are masked to 16 KiB");
static_assert(offsetof(FastLds, psel) % 16 == 0 && offsetof(FastLds, stage) % 16 == 0,
              "16-byte LDS reads of the selectors and the staging stay aligned");
// 16 blocks per CU share its 160 KiB of LDS
static_assert(sizeof(FastLds) * 2 * POM_WAVES_PER_EU <= 160 * 1024, "LDS budget");


__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ uint32_t lane_read(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint64_t wave_ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ void wave_order() { __atomic_signal_fence(__ATOMIC_SEQ_CST); }
// Lane masks straight from a v_cmp (a ballot of a compound bool costs a
// v_cndmask and a v_cmp more): active lanes with a < b, a >= b, (int)a >= 0.
__device__ __forceinline__ uint64_t mask_lt(uint32_t a, uint32_t b) { return __builtin_amdgcn_uicmp(a, b, 36); }
__device__ __forceinline__ uint64_t mask_ge(uint32_t a, uint32_t b) { return __builtin_amdgcn_uicmp(a, b, 35); }
__device__ __forceinline__ uint64_t mask_nonneg(uint32_t a) { return __builtin_amdgcn_sicmp((int32_t)a, 0, 39); }

// Inclusive prefix sum over the wave: DPP row shifts inside each 16-lane row,
// then the row totals via readlane (no LDS round trip).
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

// (diagnostics only) maximum over the wave
__device__ __forceinline__ uint32_t wave_max_dbg(uint32_t v)
{
    uint32_t m = 0;
    for (uint32_t i = 0; i < (uint32_t)kWave; i++) {
        const uint32_t x = __builtin_amdgcn_readlane(v, i);
        m = x > m ? x : m;
    }
    return m;
}

__device__ __forceinline__ uint32_t shift_up1(uint32_t v, uint32_t fill)
{
    const uint32_t u = (uint32_t)__shfl_up((int)v, 1, kWave);
    return lane_id() == 0 ? fill : u;
}

__device__ __forceinline__ uint32_t lds_load(const uint32_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store(uint32_t* p, uint32_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Drain of the last round of blocks.  Arbitration by age lets the oldest
// waves of a CU run ahead; the blocks then finish one by one and the last few
// waves cannot fill their SIMDs.  In the final round (blockIdx >= prio_from)
// the executor's priority follows the output bytes it has left: 3 while 3 steps
// (POM_PRIO_STEP) or more remain, then 2, 1 and 0 below one step, so blocks
// that are behind win issue over those ahead and a CU's blocks finish
// together.  The parser wave (also the block's HBM writer) stays at 3 so that
// it keeps ahead of its executor.  Earlier rounds keep the default priority:
// with blocks queued behind them, finishing early is what frees a slot.
__device__ __forceinline__ void prio_by_bytes_left(uint32_t left)
{
    constexpr uint32_t st = POM_PRIO_STEP;
    const uint32_t q = __builtin_amdgcn_readfirstlane(left >= 3u * st ? 3u : left >= 2u * st ? 2u
                                                      : left >= st ? 1u : 0u);
    switch (q) {
    case 3: __builtin_amdgcn_s_setprio(3); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    default: __builtin_amdgcn_s_setprio(0); break;
    }
}

struct Blk {
    const uint8_t* in;      // compressed block
    uint32_t z;             // its length
    uint8_t* out;
    uint32_t cap;
    uint32_t P;             // current piece start (input offset)
    uint32_t staged;        // bytes of input staged at stage[0] (from P)
};

__device__ __forceinline__ uint32_t stage_byte(const FastLds& s, uint32_t i)
{
    return (s.stage[i >> 2] >> (8u * (i & 3u))) & 0xFFu;
}

// Input byte for the parser (0 at or beyond z: oracle convention).
__device__ __forceinline__ uint32_t rdin(const FastLds& s, const Blk& k, uint32_t pos)
{
    if (pos >= k.z)
        return 0;
    const uint32_t r = pos - k.P;
    if (r < k.staged)
        return stage_byte(s, r);
    return *((__attribute__((address_space(1))) const uint8_t*)(k.in + pos));
}

// One instruction from (pos, st).  Produces up to two ops (A: literal run or
// match; B: trailing literals) and the next point.  `bad` reports reads past
// the end of the input, literal runs past the end, or an EOF marker that is
// not the final instruction; `eof` the EOF marker (lib/minilzo.c:3580).
struct Step {
    uint32_t pos, st;
    uint32_t aL, aS;        // op A: length, source (literal: kLitFlag | in pos; match: dist)
    uint32_t bL, bS;        // op B (bL == 0: none)
    bool eof, bad;
};

__device__ __forceinline__ uint32_t read_ext(const FastLds& s, const Blk& k, uint32_t& pos,
                                             uint32_t base, bool& bad)
{
    uint32_t v = 0;
    while (pos < k.z && rdin(s, k, pos) == 0) {
        v += 255;
        pos++;
    }
    if (pos >= k.z) {
        bad = true;
        return 0;
    }
    v += base + rdin(s, k, pos);
    pos++;
    return v;
}

// (k by value: a noinline callee reached from divergent code must not read
// its arguments from the caller's scratch)
__device__ __noinline__ Step decode_one(const FastLds& s, const Blk k, uint32_t pos, uint32_t st)
{
    Step r;
    r.aL = r.bL = 0;
    r.aS = r.bS = 0;
    r.eof = r.bad = false;
    uint32_t t = rdin(s, k, pos);
    if (pos >= k.z)
        r.bad = true;
    if (st == ST_F) {
        if (t > 17) {
            const uint32_t n = t - 17;
            r.aL = n;
            r.aS = kLitFlag | (pos + 1);
            r.pos = pos + 1 + n;
            r.st = n < 4 ? ST_C : ST_B;
            if (r.pos > k.z)
                r.bad = true;
            return r;
        }
        st = ST_A;
    }
    uint32_t L, d;
    if (t < 16 && st == ST_A) {                       // literal run, :3367-3414
        pos++;
        if (t == 0)
            t = read_ext(s, k, pos, 15, r.bad);
        const uint32_t n = t + 3;
        r.aL = n;
        r.aS = kLitFlag | pos;
        r.pos = pos + n;
        r.st = ST_B;
        if (r.pos > k.z || r.pos < pos)
            r.bad = true;
        return r;
    }
    if (t < 16) {                                     // M1 forms, :3416-3443 / :3600-3612
        d = (st == ST_B ? 0x801u : 1u) + (t >> 2) + (rdin(s, k, pos + 1) << 2);
        L = st == ST_B ? 3u : 2u;
        pos += 2;
    } else if (t >= 64) {                             // M2
        d = 1 + ((t >> 2) & 7) + (rdin(s, k, pos + 1) << 3);
        L = (t >> 5) + 1;
        pos += 2;
    } else if (t >= 32) {                             // M3
        L = t & 31;
        pos++;
        if (L == 0)
            L = read_ext(s, k, pos, 31, r.bad);
        L += 2;
        d = 1 + ((rdin(s, k, pos) | (rdin(s, k, pos + 1) << 8)) >> 2);
        pos += 2;
    } else {                                          // M4 / EOF
        uint32_t dd = (t & 8) << 11;
        L = t & 7;
        pos++;
        if (L == 0)
            L = read_ext(s, k, pos, 7, r.bad);
        L += 2;
        dd += (rdin(s, k, pos) | (rdin(s, k, pos + 1) << 8)) >> 2;
        pos += 2;
        if (dd == 0) {
            r.eof = true;
            r.pos = pos;
            r.st = ST_A;
            if (pos != k.z)
                r.bad = true;                         // INPUT_NOT_CONSUMED / OVERRUN
            return r;
        }
        d = dd + 0x4000;
    }
    if (pos > k.z)
        r.bad = true;
    r.aL = L;
    r.aS = d;
    const uint32_t tl = rdin(s, k, pos - 2) & 3;      // match_done, :3650-3653
    if (tl) {
        r.bL = tl;
        r.bS = kLitFlag | pos;
        pos += tl;
        r.st = ST_C;
        if (pos > k.z)
            r.bad = true;
    } else
        r.st = ST_A;
    r.pos = pos;
    return r;
}

// Branch-free form of decode_one for the common case: the instruction lies in
// the staged input and any length extension is a single non-zero byte.  One
// LDS round trip (two aligned dwords -> 4 bytes at pos), then selects; lanes
// decoding different instruction kinds do not diverge.  Falls back to
// decode_one otherwise (long extensions, input beyond the staging window).
// SPEC: speculative use -- never take the slow path; report it as `slow`
// (the caller restarts or re-walks exactly) instead.
template <bool SPEC = false>
__device__ __forceinline__ Step decode_step(const FastLds& s, const Blk& k, uint32_t pos, uint32_t st,
                                            bool* slow = nullptr)
{
    const uint32_t rel = pos - k.P;
    const bool inwin = rel + 8 <= kStageBytes && pos < k.z;
    // Every field of a non-extended instruction lies in its first 4 bytes
    // (t, then at most 3 more; bytes past z read 0 from the stage): two LDS
    // dwords, one alignbyte, then bit-field extracts -- no 64-bit shifts.
    // (The dwords are read from a clamped offset; ignored when !inwin.)
    const uint32_t wi = inwin ? rel >> 2 : 0u;
    const uint32_t lo = __builtin_amdgcn_alignbyte(s.stage[wi + 1], s.stage[wi], rel & 3u);
    const uint32_t t = lo & 0xFFu, b1 = __builtin_amdgcn_ubfe(lo, 8, 8);
    const bool flit = st == ST_F && t > 17;                        // :3357-3365
    const uint32_t se = st == ST_F ? ST_A : st;
    const bool lit = !flit && se == ST_A && t < 16;                // :3367-3414
    const bool m1 = !flit && !lit && t < 16;
    const bool m2 = !flit && t >= 64;
    const bool m3 = !flit && t >= 32 && t < 64;
    const bool m4 = !flit && t >= 16 && t < 32;
    const bool ext = (lit && t == 0) || (m3 && (t & 31) == 0) || (m4 && (t & 7) == 0);
    const bool needs_slow = !inwin || (ext && b1 == 0);            // 255-chunk extension
    const uint32_t e = ext ? 1u : 0u;
    const uint32_t o16 = __builtin_amdgcn_ubfe(lo, 8u + 8u * e, 16);   // bytes 1+e, 2+e
    const uint32_t dd4 = ((t & 8u) << 11) + (o16 >> 2);
    const uint32_t used = (m1 || m2) ? 2u : 3u + e;                // match instruction bytes
    const uint32_t tl = __builtin_amdgcn_ubfe(lo, 8u * (used - 2u), 2);   // match_done, :3650
    const uint32_t nlit = flit ? t - 17 : (ext ? 15u + b1 : t) + 3u;
    const uint32_t L = m1 ? (se == ST_B ? 3u : 2u)
                     : m2 ? (t >> 5) + 1u
                     : m3 ? (ext ? 31u + b1 : (t & 31u)) + 2u
                          : (ext ? 7u + b1 : (t & 7u)) + 2u;
    const uint32_t d = m1 ? (se == ST_B ? 0x801u : 1u) + (t >> 2) + (b1 << 2)
                     : m2 ? 1u + ((t >> 2) & 7u) + (b1 << 3)
                     : m3 ? 1u + (o16 >> 2) : dd4 + 0x4000u;
    const bool eof = m4 && dd4 == 0;                               // :3580
    const bool islit = flit || lit;
    const uint32_t hdr = flit ? 1u : 1u + e;                       // literal-run header bytes
    Step r;
    r.eof = eof;
    r.aL = eof ? 0u : islit ? nlit : L;
    r.aS = islit ? kLitFlag | (pos + hdr) : d;
    r.bL = (islit || eof) ? 0u : tl;
    r.bS = kLitFlag | (pos + used);
    r.pos = islit ? pos + hdr + nlit : pos + used + (eof ? 0u : tl);
    r.st = islit ? (flit && nlit < 4 ? ST_C : ST_B) : (tl && !eof ? ST_C : ST_A);
    r.bad = eof ? r.pos != k.z : r.pos > k.z;
    if (__builtin_expect(needs_slow, 0)) {
        if (SPEC) {
            r.pos = pos;
            r.st = st;
            r.aL = r.bL = 0;
            r.eof = false;
            r.bad = true;
            *slow = true;
        } else
            r = decode_one(s, k, pos, st);
    }
    return r;
}

// Wave-uniform form of decode_step for the parser's exact walks (the scalar
// scan below walks one segment's true path with every lane at the same
// point): the two stage dwords are made scalar with readfirstlane, so the
// decode runs on the scalar unit -- a few SALU per field instead of a VALU
// instruction for all 64 lanes (~55 per instruction decoded).  Same fields as
// decode_step; the rare instructions take decode_one (per lane, all alike).
#ifndef POM_UWALK
#define POM_UWALK 1
#endif
__device__ __forceinline__ Step decode_step_u(const FastLds& s, const Blk& k, uint32_t pos, uint32_t st)
{
    const uint32_t rel = pos - k.P;
    const bool inwin = rel + 8 <= kStageBytes && pos < k.z;
    const uint32_t wi = inwin ? rel >> 2 : 0u;
    const uint32_t w0 = __builtin_amdgcn_readfirstlane(s.stage[wi]);
    const uint32_t w1 = __builtin_amdgcn_readfirstlane(s.stage[wi + 1]);
    const uint32_t lo = (uint32_t)((((uint64_t)w1 << 32) | w0) >> (8u * (rel & 3u)));
    const uint32_t t = lo & 0xFFu, b1 = (lo >> 8) & 0xFFu;
    const bool flit = st == ST_F && t > 17;                        // :3357-3365
    const uint32_t se = st == ST_F ? ST_A : st;
    const bool lit = !flit && se == ST_A && t < 16;                // :3367-3414
    const bool m1 = !flit && !lit && t < 16;
    const bool m2 = !flit && t >= 64;
    const bool m3 = !flit && t >= 32 && t < 64;
    const bool m4 = !flit && t >= 16 && t < 32;
    const bool ext = (lit && t == 0) || (m3 && (t & 31) == 0) || (m4 && (t & 7) == 0);
    const bool needs_slow = !inwin || (ext && b1 == 0);            // 255-chunk extension
    const uint32_t e = ext ? 1u : 0u;
    const uint32_t o16 = (lo >> (8u + 8u * e)) & 0xFFFFu;          // bytes 1+e, 2+e
    const uint32_t dd4 = ((t & 8u) << 11) + (o16 >> 2);
    const uint32_t used = (m1 || m2) ? 2u : 3u + e;                // match instruction bytes
    const uint32_t tl = (lo >> (8u * (used - 2u))) & 3u;           // match_done, :3650
    const uint32_t nlit = flit ? t - 17 : (ext ? 15u + b1 : t) + 3u;
    const uint32_t L = m1 ? (se == ST_B ? 3u : 2u)
                     : m2 ? (t >> 5) + 1u
                     : m3 ? (ext ? 31u + b1 : (t & 31u)) + 2u
                          : (ext ? 7u + b1 : (t & 7u)) + 2u;
    const bool eof = m4 && dd4 == 0;                               // :3580
    const bool islit = flit || lit;
    const uint32_t hdr = flit ? 1u : 1u + e;                       // literal-run header bytes
    Step r;
    r.eof = eof;
    r.aL = eof ? 0u : islit ? nlit : L;
    r.aS = 0;                                                      // (the walks count ops only)
    r.bL = (islit || eof) ? 0u : tl;
    r.bS = 0;
    r.pos = islit ? pos + hdr + nlit : pos + used + (eof ? 0u : tl);
    r.st = islit ? (flit && nlit < 4 ? ST_C : ST_B) : (tl && !eof ? ST_C : ST_A);
    r.bad = eof ? r.pos != k.z : r.pos > k.z;
    if (__builtin_expect(needs_slow, 0)) {
        // (every lane decodes the same instruction: keep the fields scalar)
        const Step q = decode_one(s, k, pos, st);
        r.pos = __builtin_amdgcn_readfirstlane(q.pos);
        r.st = __builtin_amdgcn_readfirstlane(q.st);
        r.aL = __builtin_amdgcn_readfirstlane(q.aL);
        r.bL = __builtin_amdgcn_readfirstlane(q.bL);
        r.eof = __builtin_amdgcn_readfirstlane(q.eof ? 1u : 0u) != 0;
        r.bad = __builtin_amdgcn_readfirstlane(q.bad ? 1u : 0u) != 0;
    }
    return r;
}

// Output / input byte helpers -------------------------------------------------
__device__ __forceinline__ uint32_t ring_byte(const FastLds& s, uint32_t y)
{
    const uint32_t i = y & kRingMask;
    return (s.ring[i >> 2] >> (8u * (i & 3u))) & 0xFFu;
}

__device__ __forceinline__ uint32_t funnel(uint32_t lo, uint32_t hi, uint32_t sh)
{
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8u * sh));
}

// Misaligned LDS accesses for the 16-byte steps.  gfx950 runs LDS in
// unaligned mode: ds_read_b128 / ds_write_b128 / b64 / b32 / b16 at any byte
// address are exact (scripts/probe/lds_misaligned_probe.hip; ~1.5x the
// latency of an aligned access).  The compiler assumes natural alignment for
// its own accesses, so these are written out.  The reads wait for their data
// themselves; LDS accesses of one wave complete in order, so the compiler's
// own lgkmcnt waits stay correct (they only become more conservative).
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t lds_off(const void* p)
{
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void lds_read16x4(uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                                             uint4& va, uint4& vb, uint4& vc, uint4& vd)
{
    v4u32 x, y, z, w;
    asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %5\n\t"
                 "ds_read_b128 %2, %6\n\tds_read_b128 %3, %7\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(x), "=&v"(y), "=&v"(z), "=&v"(w) : "v"(a), "v"(b), "v"(c), "v"(d) : "memory");
    va = make_uint4(x.x, x.y, x.z, x.w);
    vb = make_uint4(y.x, y.y, y.z, y.w);
    vc = make_uint4(z.x, z.y, z.z, z.w);
    vd = make_uint4(w.x, w.y, w.z, w.w);
}
__device__ __forceinline__ uint4 lds_read16(uint32_t a)
{
    v4u32 x;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(x) : "v"(a) : "memory");
    return make_uint4(x.x, x.y, x.z, x.w);
}
__device__ __forceinline__ void lds_read16x2(uint32_t a, uint32_t b, uint4& va, uint4& vb)
{
    v4u32 x, y;
    asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(x), "=&v"(y) : "v"(a), "v"(b) : "memory");
    va = make_uint4(x.x, x.y, x.z, x.w);
    vb = make_uint4(y.x, y.y, y.z, y.w);
}
__device__ __forceinline__ void lds_read16x3(uint32_t a, uint32_t b, uint32_t c, uint4& va, uint4& vb,
                                             uint4& vc)
{
    v4u32 x, y, z;
    asm volatile("ds_read_b128 %0, %3\n\tds_read_b128 %1, %4\n\tds_read_b128 %2, %5\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(x), "=&v"(y), "=&v"(z) : "v"(a), "v"(b), "v"(c) : "memory");
    va = make_uint4(x.x, x.y, x.z, x.w);
    vb = make_uint4(y.x, y.y, y.z, y.w);
    vc = make_uint4(z.x, z.y, z.z, z.w);
}
__device__ __forceinline__ void lds_write16(uint32_t a, uint4 v)
{
    const v4u32 t = {v.x, v.y, v.z, v.w};
    asm volatile("ds_write_b128 %0, %1" : : "v"(a), "v"(t) : "memory");
}
__device__ __forceinline__ void lds_write8(uint32_t a, uint32_t lo, uint32_t hi)
{
    const v2u32 t = {lo, hi};
    asm volatile("ds_write_b64 %0, %1" : : "v"(a), "v"(t) : "memory");
}
__device__ __forceinline__ void lds_write4(uint32_t a, uint32_t v)
{
    asm volatile("ds_write_b32 %0, %1" : : "v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_write2(uint32_t a, uint32_t v)
{
    asm volatile("ds_write_b16 %0, %1" : : "v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_write1(uint32_t a, uint32_t v)
{
    asm volatile("ds_write_b8 %0, %1" : : "v"(a), "v"(v) : "memory");
}


// The first len (<= 16) bytes of v at LDS address a: one b128 for a whole
// chunk, else b64/b32/b16/b8 pieces.
__device__ __forceinline__ __attribute__((unused)) void lds_write_part(uint32_t a, uint4 v, uint32_t len)
{
#ifdef POM_BYTE_WRITES
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (uint32_t i = 0; i < 16; i++)
        if (i < len)
            lds_write1(a + i, w[i >> 2] >> (8 * (i & 3)));
    return;
#endif
    if (len == 16u) {
        lds_write16(a, v);
        return;
    }
    uint32_t w0 = v.x, w1 = v.y, ad = a;
    if (len & 8u) {
        lds_write8(ad, v.x, v.y);
        w0 = v.z;
        w1 = v.w;
        ad += 8;
    }
    if (len & 4u) {
        lds_write4(ad, w0);
        w0 = w1;
        ad += 4;
    }
    if (len & 2u) {
        lds_write2(ad, w0);
        w0 >>= 16;
        ad += 2;
    }
    if (len & 1u)
        lds_write1(ad, w0);
}

typedef __attribute__((address_space(1))) const uint32_t gdword;

// 4 bytes at an arbitrary global address via two aligned dword loads (an
// aligned dword that overlaps valid bytes never leaves their page).  NT: L2
// served (the vector L1 is not coherent with the writer wave's stores).
// Address-space-1 pointers keep these global_load (vmcnt only), not flat_load
// (which also waits on lgkmcnt and so on every outstanding LDS access).
#ifndef POM_OUT_NT
#define POM_OUT_NT 0                             // writer: non-temporal output stores
#endif
#ifndef POM_SRC_SC1
#define POM_SRC_SC1 1                            // source-buffer loads: agent-scope (L2-allocating) instead of non-temporal
#endif
#ifndef POM_FAR_SC1
#define POM_FAR_SC1 1                            // far reads: agent-scope (L2-allocating) loads instead of non-temporal
#endif
#ifndef POM_WRAP_MIRROR
#define POM_WRAP_MIRROR 1                        // a ring-wrapping chunk: one write through the mirror, then a 16-byte copy
#endif
#ifndef POM_FAR_UNCOND
#define POM_FAR_UNCOND 1                         // far reads: all five loads unconditional (clamped addresses)
#endif
template <bool NT>
__device__ __forceinline__ uint32_t global_dword(const uint8_t* p)
{
    const uintptr_t a = (uintptr_t)p;
    gdword* q = (gdword*)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    uint32_t w0, w1 = 0;
    if (NT) {
        w0 = __builtin_nontemporal_load(q);
        if (sh)
            w1 = __builtin_nontemporal_load(q + 1);
    } else {
        w0 = q[0];
        if (sh)
            w1 = q[1];
    }
    return sh ? funnel(w0, w1, sh) : w0;
}

// Bytes [lo, hi) (hi <= 16) of the 16 at global address p, read through L2
// with aligned dword loads that each hold at least one of those bytes (so no
// load leaves their pages); the other bytes read as 0.
__device__ __forceinline__ uint4 global_read16(const uint8_t* p, uint32_t lo, uint32_t hi)
{
    const uintptr_t a = (uintptr_t)p;
    gdword* q = (gdword*)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    uint32_t w[5];
#if POM_FAR_UNCOND
    // every load issued (no exec branch per dword): a dword outside
    // [i0, i1] reads dword i0 or i1 again and is then dropped
    const uint32_t i0 = (lo + sh) >> 2, i1 = (hi + sh - 1) >> 2;
#pragma unroll
    for (uint32_t i = 0; i < 5; i++) {
        const uint32_t j = i < i0 ? i0 : i > i1 ? i1 : i;
        const uint32_t v = __hip_atomic_load((uint32_t*)(q + j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        w[i] = i == j ? v : 0u;
    }
#else
#pragma unroll
    for (uint32_t i = 0; i < 5; i++) {
        // aligned dword i holds bytes 4i - sh .. 4i + 3 - sh of the span
        const bool use = 4 * i < hi + sh && 4 * i + 4 > lo + sh;
        w[i] = use ? (POM_FAR_SC1 ? __hip_atomic_load((uint32_t*)(q + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                  : __builtin_nontemporal_load(q + i)) : 0u;
    }
#endif
    uint4 v;
    v.x = __builtin_amdgcn_alignbyte(w[1], w[0], sh);
    v.y = __builtin_amdgcn_alignbyte(w[2], w[1], sh);
    v.z = __builtin_amdgcn_alignbyte(w[3], w[2], sh);
    v.w = __builtin_amdgcn_alignbyte(w[4], w[3], sh);
    return v;
}

// ---------------------------------------------------------------------------
// Parser walks.  A lane's final speculative attempt leaves, per state, a
// bitmap of the instruction starts it visited in its segment [c0, c0 + kSeg)
// and a bitmap of those starts that yield two ops.  A walk of the true path
// that lands on one of them follows the speculative path from there: its op
// count is the popcount of the starts at or after that point (plus the
// two-op starts), and its exit is the speculative exit.
// ---------------------------------------------------------------------------
struct Marks {
    uint32_t m[4];          // instruction starts, per state (A, B, C, F)
    uint32_t two;           // starts that yield two ops
    uint32_t xpos, xst;     // the speculative exit
};

struct WalkRes {
    uint32_t pos, st, cnt, fl;
};

__device__ __forceinline__ uint32_t mark_of(const Marks& M, uint32_t st)
{
    return st == ST_A ? M.m[0] : st == ST_B ? M.m[1] : st == ST_C ? M.m[2] : M.m[3];
}

template <bool SPEC>
__device__ __forceinline__ WalkRes walk_true(const FastLds& S, const Blk& k, uint32_t c0, uint32_t c1,
                                             const Marks& M, uint32_t pos, uint32_t st)
{
    WalkRes w;
    w.cnt = 0;
    w.fl = FL_OK;
    while (pos < c1) {
        if (pos >= k.z) {
            w.fl = FL_DEAD;
            pos = kPosEnd;
            break;
        }
        if (pos >= c0) {
            const uint32_t bit = 1u << (pos - c0);
            if (mark_of(M, st) & bit) {            // joined the speculative path
                const uint32_t from = ~(bit - 1u);
                const uint32_t starts = M.m[0] | M.m[1] | M.m[2] | M.m[3];
                w.cnt += (uint32_t)__builtin_popcount(starts & from) + (uint32_t)__builtin_popcount(M.two & from);
                pos = M.xpos;
                st = M.xst;
                if (pos == kPosEnd)
                    w.fl = FL_DEAD;                // it runs off the input end
                break;
            }
        }
        bool slow = false;
        const Step r = (!SPEC && POM_UWALK) ? decode_step_u(S, k, pos, st) : decode_step<SPEC>(S, k, pos, st, &slow);
        if (SPEC && slow) {
            w.fl = FL_UNK;
            break;
        }
        if (r.eof) {
            w.fl = r.bad ? FL_DEAD : FL_EOF;
            pos = kPosEnd;
            break;
        }
        if (r.bad) {
            w.fl = FL_DEAD;
            pos = kPosEnd;
            break;
        }
        w.cnt += (r.aL ? 1u : 0u) + (r.bL ? 1u : 0u);
        pos = r.pos;
        st = r.st;
    }
    w.pos = pos;
    w.st = st;
    return w;
}

// Diagnostic build only (STAMPS): per-phase s_memtime cycle sums and event
// counts go to stamps[b * kStampSlots + i]; no output value depends on them.
// Each wave writes only the slots it owns (parser: parser_slot).
// scripts/diag_decode.py knows this order.
enum { PH_STAGE, PH_PASS1, PH_PWALK, PH_MERGE, PH_COUNT, PH_WRITE, PH_PSLOT, PH_PDUTY,
       PH_EWAIT, PH_WLOAD, PH_WSCAN, PH_FARI, PH_FWD, PH_FARC, PH_BATCH,
       PH_SPACE, PH_FLAGS, PH_GATHER, PH_PUB,
       CN_FIRST, CN_WALKS = CN_FIRST, CN_IT_PASS1, CN_IT_PWALK, CN_IT_WALK, CN_IT_COUNT,
       CN_IT_WRITE, CN_PIECES,
       CN_WINDOWS, CN_SRCWIN, CN_SRCMISS, CN_BATCHES, CN_STEPS, CN_FWD_ROUNDS,
       CN_WBATCHES, CN_NW_GOP, CN_NW_PER, CN_REASON, PH_N };
constexpr int kStampSlots = 40;
static_assert(PH_N <= kStampSlots, "stamp slots per block");
__device__ __forceinline__ bool parser_slot(int i)
{
    return i <= PH_PDUTY || (i >= CN_WALKS && i <= CN_PIECES);
}

#define STAMP(ph)                                                   \
    do {                                                            \
        if (STAMPS) {                                               \
            const uint64_t now_ = __builtin_amdgcn_s_memtime();     \
            acc[ph] += now_ - tmark;                                \
            tmark = now_;                                           \
        }                                                           \
    } while (0)

// ---------------------------------------------------------------------------
// Writer duty (parser wave, between parse steps): final ring bytes go to HBM
// in 1-KiB chunks, one dwordx4 store per lane.  Two positions are published:
//   issued  -- stores issued (their data left the ring): those ring slots
//              may be overwritten;
//   landed  -- stores known to be in HBM: that output may be read back.
// `landed` trails by one batch of chunks: the wait for a batch is taken when
// the next one is issued (by then it has long landed), or at once when the
// executor asks for more (S.need) -- so the executor never waits on a store
// it does not read.
// Returns 2 once the executor refused the block, 1 once everything it
// produced has landed after it finished, 0 otherwise.
// ---------------------------------------------------------------------------
constexpr uint32_t kChunk = 16 * kWave;          // 1 KiB per store instruction

struct WState {
    uint32_t issued;        // output bytes whose stores were issued
    uint32_t landed;        // output bytes published as landed
};

__device__ __forceinline__ uint32_t writer_duty(FastLds& S, uint8_t* out, uint32_t l, WState& w)
{
    if (POM_EXEC_STORES)
        return 0;                                      // (the executor stores its own output)
    const uint32_t state = lds_load(&S.state);
    const uint32_t prod = lds_load(&S.produced);
    if (state == 2)
        return 2;                                      // refused: the exact decoder redoes it
    const uint32_t upto = state == 1 ? prod : (prod & ~(kChunk - 1));
    const bool fresh = upto > w.issued;
    if (w.landed < w.issued && (fresh || state == 1 || lds_load(&S.need) > w.landed)) {
        __builtin_amdgcn_s_waitcnt(0x0F70);            // vmcnt(0): the last batch landed
        w.landed = w.issued;
        lds_store(&S.landed, w.landed);
    }
    if (!fresh)
        return (state == 1 && w.landed == prod) ? 1u : 0u;
    for (int c = 0; c < 4 && w.issued < upto; c++) {
        const uint32_t end = upto - w.issued > kChunk ? w.issued + kChunk : upto;
        const uint32_t x = w.issued + 16 * l;
        if (x + 16 <= end) {
            const uint32_t i = x & kRingMask;
            const uint4 v = *(const uint4*)&S.ring[i >> 2];
            if (POM_OUT_NT)
                __builtin_nontemporal_store((v4u32){v.x, v.y, v.z, v.w}, (v4u32*)(out + x));
            else
                *(uint4*)(out + x) = v;
        } else if (x < end) {
            for (uint32_t q = 0; x + q < end; q++)
                out[x + q] = (uint8_t)ring_byte(S, x + q);
        }
        w.issued = end;
    }
    lds_store(&S.issued, w.issued);                    // (after the ring reads completed)
    return 0;
}

// Executor-side stores (POM_EXEC_STORES): the executor stores ring bytes
// [at, end) of its own output, one dwordx4 per lane for whole 16-byte pieces
// (bytes past `end` are not written).  Its LDS reads of the ring come before
// any later ring write of the wave (LDS accesses of a wave complete in order),
// so a slot may be overwritten by the next step as soon as its store is issued.
__device__ __forceinline__ void exec_store_chunk(const FastLds& S, uint8_t* out, uint32_t l, uint32_t at)
{
    // (a whole 1-KiB piece: no partial lanes, no branches in the step loop)
    const uint32_t x = at + 16 * l;
    const uint4 v = *(const uint4*)&S.ring[(x & kRingMask) >> 2];
    *(uint4*)(out + x) = v;
}
__device__ __forceinline__ void exec_store(const FastLds& S, uint8_t* out, uint32_t l, uint32_t at, uint32_t end)
{
    const uint32_t x = at + 16 * l;
    if (x + 16 <= end) {
        const uint4 v = *(const uint4*)&S.ring[(x & kRingMask) >> 2];
        *(uint4*)(out + x) = v;
    } else if (x < end) {
        for (uint32_t q = 0; x + q < end; q++)
            out[x + q] = (uint8_t)ring_byte(S, x + q);
    }
}

// ---------------------------------------------------------------------------
// Parser wave: pieces in stream order with exact entries (the true exit of
// the previous piece), ops to slot q mod kSlots; writer duty in between.
// ---------------------------------------------------------------------------
template <bool STAMPS>
__device__ __forceinline__ void parser_wave(FastLds& S, Blk k, uint2* __restrict__ gops, uint32_t l,
                                            uint64_t* acc)
{
    uint64_t tmark = STAMPS ? __builtin_amdgcn_s_memtime() : 0;
    WState w;
    w.issued = 0;
    w.landed = 0;
    uint32_t entry_pos = 0, entry_st = ST_F;   // true entry of the current piece
    for (uint32_t q = 0;; q++) {
        // Skip pieces in which no instruction starts (inside a long literal run).
        if (entry_pos >= k.P + kPiece)
            k.P = entry_pos - (entry_pos % kPiece);
        // a free slot: the executor is done with piece q - kSlots
        for (uint32_t spin = 0; q - lds_load(&S.consumed) >= kSlots; spin++) {
            if (writer_duty(S, k.out, l, w) == 2 || spin > (1u << 22) ||
                (POM_EXEC_STORES && lds_load(&S.state) == 2))
                return;                        // the executor refused (or is stuck)
            __builtin_amdgcn_s_sleep(POM_WRITER_SLEEP);
        }
        STAMP(PH_PSLOT);
        if (STAMPS)
            acc[CN_PIECES] += 1;
        uint2* const slot = gops + (q & (kSlots - 1)) * kOpMax;
        bool err = k.P >= k.z;                 // ran off the end without EOF
        uint32_t reason = err ? (uint32_t)RS_OFF_END : (uint32_t)RS_NONE;
        bool eof = false;
        uint32_t total_ops = 0;
        uint32_t next_pos = 0, next_st = 0;
        if (!err) {
            // ---- stage the piece's input --------------------------------------
            const uint32_t avail = k.z - k.P;
            k.staged = avail < kStageBytes ? avail : kStageBytes;
            const uint8_t* base = k.in + k.P;
            for (uint32_t i = l * 4; i < kStageBytes; i += kWave * 4) {
                uint32_t v = 0;
                if (i + 4 <= k.staged)
                    v = global_dword<false>(base + i);
                else
                    for (uint32_t j = i; j < k.staged; j++)
                        v |= (uint32_t)base[j] << (8 * (j - i));
                S.stage[i >> 2] = v;
            }
            wave_order();
            STAMP(PH_STAGE);
            const uint32_t c0 = k.P + l * kSeg;        // this lane's segment
            const uint32_t c1 = c0 + kSeg;

            // ---- pass 1: speculative walk; the final attempt's starts -----------
            const bool p1 = c1 > entry_pos;            // else no instruction starts here
            uint32_t pos = c0 >= k.P + kLook ? c0 - kLook : k.P;
            if (pos < entry_pos)
                pos = entry_pos;
            uint32_t st = pos == entry_pos ? entry_st : ST_A;
            Marks M;
            M.m[0] = M.m[1] = M.m[2] = M.m[3] = 0;
            M.two = 0;
            for (uint32_t it = 1;; it++) {
                const bool act = p1 && pos < c1 && pos < k.z;
                if (!wave_ballot(act))
                    break;
                if (act) {
                    bool slow = false;
                    const Step r = decode_step<true>(S, k, pos, st, &slow);
                    const bool mine = pos >= c0;
                    const uint32_t bit = mine ? 1u << (pos - c0) : 0u;
                    if (r.bad || r.eof) {              // impossible guess: restart later
                        pos++;
                        st = ST_A;
                        if (mine) {                    // only the final attempt counts
                            M.m[0] = M.m[1] = M.m[2] = M.m[3] = 0;
                            M.two = 0;
                        }
                    } else {
                        M.m[0] |= st == ST_A ? bit : 0u;
                        M.m[1] |= st == ST_B ? bit : 0u;
                        M.m[2] |= st == ST_C ? bit : 0u;
                        M.m[3] |= st == ST_F ? bit : 0u;
                        M.two |= r.bL ? bit : 0u;
                        pos = r.pos;
                        st = r.st;
                    }
                }
                if (STAMPS)
                    acc[CN_IT_PASS1] += 1;
                if (it % POM_DUTY_EVERY == 0) {
                    STAMP(PH_PASS1);
                    if (writer_duty(S, k.out, l, w) == 2)
                        return;
                    STAMP(PH_PDUTY);
                }
            }
            M.xpos = !p1 ? entry_pos : pos >= k.z ? kPosEnd : pos;
            M.xst = !p1 ? entry_st : st;
            wave_order();
            STAMP(PH_PASS1);

            // ---- true entries: one parallel walk from the assumed entries, then
            // a scalar scan that reuses it and walks only where the guess was wrong.
            const uint32_t apos = shift_up1(M.xpos, entry_pos), ast = shift_up1(M.xst, entry_st);
            const WalkRes f = walk_true<true>(S, k, c0, c1, M, apos, ast);
            STAMP(PH_PWALK);
            if (writer_duty(S, k.out, l, w) == 2)
                return;
            STAMP(PH_PDUTY);
            // Where lane i's true entry E equals its assumed one and its walk
            // finished, lanes i, i+1, ... stay right as long as each walk ended
            // at the next lane's assumed entry (f_l == x_l, FL_OK) and that
            // lane's own walk finished; the scan jumps to the first lane q
            // where that fails, E_q = f_{q-1}.
            uint32_t epos = kPosEnd, est = ST_A, ecnt = 0;
            uint64_t run = 0;                          // lanes whose parallel walk is true
            bool dead = false;
#ifdef POM_DEBUG_DEAD
            bool dbg_stage_bad = false;
#endif
            {
                const uint64_t brk = wave_ballot(f.fl != FL_OK || f.pos != M.xpos || f.st != M.xst) << 1;
                const uint64_t unk = wave_ballot(f.fl == FL_UNK);
                uint32_t E = entry_pos, Est = entry_st;
                uint32_t i = 0;
#ifdef POM_DEBUG_DEAD
                uint32_t dbg_i = 99, dbg_E = 0, dbg_Est = 0;
                (void)dbg_i; (void)dbg_E; (void)dbg_Est;
#endif
                while (i < (uint32_t)kWave) {
                    const uint32_t ci1 = k.P + (i + 1) * kSeg;
                    if (E >= ci1) {                    // no true start in segment i
                        const uint32_t j = E - k.P < kPiece ? (E - k.P) / kSeg : (uint32_t)kWave;
                        i = j > i + 1 ? j : i + 1;
                        continue;
                    }
                    if (E == lane_read(apos, i) && Est == lane_read(ast, i) && !((unk >> i) & 1)) {
                        const uint64_t cand = i + 1 < (uint32_t)kWave ? (brk | unk) & (~0ull << (i + 1)) : 0ull;
                        const uint32_t qq = cand ? (uint32_t)__builtin_ctzll(cand) : (uint32_t)kWave;
                        run |= (qq == 64 ? ~0ull : ((1ull << qq) - 1)) & (~0ull << i);
                        E = lane_read(f.pos, qq - 1);
                        Est = lane_read(f.st, qq - 1);
                        const uint32_t fl = lane_read(f.fl, qq - 1);
                        if (fl == FL_EOF) {
                            eof = true;
                            break;
                        }
                        if (fl == FL_DEAD) {
                            dead = true;
#ifdef POM_DEBUG_DEAD
                            dbg_i = 100 + qq - 1;
#endif
                            break;
                        }
                        i = qq;
                        continue;
                    }
                    // lane i on its own, from its true entry E
                    Marks Mi;
                    Mi.m[0] = lane_read(M.m[0], i);
                    Mi.m[1] = lane_read(M.m[1], i);
                    Mi.m[2] = lane_read(M.m[2], i);
                    Mi.m[3] = lane_read(M.m[3], i);
                    Mi.two = lane_read(M.two, i);
                    Mi.xpos = lane_read(M.xpos, i);
                    Mi.xst = lane_read(M.xst, i);
#ifdef POM_DEBUG_DEAD
                    dbg_E = E;
                    dbg_Est = Est;
#endif
                    const WalkRes g = walk_true<false>(S, k, ci1 - kSeg, ci1, Mi, E, Est);
                    if (STAMPS)
                        acc[CN_WALKS] += 1;
                    if (l == i) {
                        epos = E;
                        est = Est;
                        ecnt = g.cnt;
                    }
                    E = g.pos;
                    Est = g.st;
                    STAMP(PH_MERGE);
                    if (writer_duty(S, k.out, l, w) == 2)
                        return;
                    STAMP(PH_PDUTY);
                    if (g.fl == FL_EOF) {
                        eof = true;
                        break;
                    }
                    if (g.fl == FL_DEAD) {
                        dead = true;
#ifdef POM_DEBUG_DEAD
                        dbg_i = i;
#endif
                        break;
                    }
                    i++;
                }
                next_pos = E;                          // (uniform: the piece's true exit)
                next_st = Est;
#ifdef POM_DEBUG_DEAD
                if (dead || (!eof && E == kPosEnd)) {
                    // (diagnostic) does the LDS stage still hold the input?
                    bool diff = false;
                    for (uint32_t i = l * 4; i < kStageBytes; i += kWave * 4) {
                        uint32_t v = 0;
                        if (i + 4 <= k.staged)
                            v = global_dword<false>(k.in + k.P + i);
                        else
                            for (uint32_t j = i; j < k.staged; j++)
                                v |= (uint32_t)k.in[k.P + j] << (8 * (j - i));
                        diff |= S.stage[i >> 2] != v;
                    }
                    dbg_stage_bad = wave_ballot(diff) != 0;
                }
#endif
                if ((run >> l) & 1) {
                    epos = apos;
                    est = ast;
                    ecnt = f.cnt;
                }
            }
            STAMP(PH_MERGE);
            const uint32_t incl = wave_incl_scan(ecnt);
            total_ops = lane_read(incl, kWave - 1);
            if (dead) {
                err = true;
                reason = RS_DEAD;
#ifdef POM_DEBUG_DEAD
                if (dbg_stage_bad)
                    reason = 12;                       // (diagnostic) the stage was overwritten
#endif
            } else if (total_ops > kOpMax) {
                err = true;
                reason = RS_OPS;
            }
            // ---- write the ops (length, source) of the true path to the slot ------
            if (!err) {
                uint32_t wi = incl - ecnt;
                const uint32_t wend = incl;
                uint32_t p = epos, s = est;
                bool lane_err = false;
                uint32_t itw = 0;
                while (p < c1 && wi < wend) {
                    itw++;
                    const Step r = decode_step(S, k, p, s);
                    if (r.eof || r.bad) {
                        lane_err = true;               // (the scan saw ops here)
                        break;
                    }
                    if (r.aL > kMaxOpLen || r.bL > kMaxOpLen || wi + (r.aL ? 1u : 0u) + (r.bL ? 1u : 0u) > wend) {
                        lane_err = true;
                        break;
                    }
                    if (r.aL)
                        slot[wi++] = make_uint2(r.aL, r.aS);
                    if (r.bL)
                        slot[wi++] = make_uint2(r.bL, r.bS);
                    p = r.pos;
                    s = r.st;
                }
                lane_err = lane_err || wi != wend;
                if (STAMPS)
                    acc[CN_IT_WRITE] += wave_max_dbg(itw);
                if (wave_ballot(lane_err)) {
                    err = true;
                    reason = RS_BAD;
                }
            }
            if (!err && !eof && next_pos == kPosEnd) {
                err = true;                            // dead without EOF
                reason = RS_DEAD;
            }
            STAMP(PH_WRITE);
        }
        // publish piece q once its op records landed
        __builtin_amdgcn_s_waitcnt(0x0F70);            // vmcnt(0)
        lds_store(&S.pinfo[q & (kSlots - 1)],
                  total_ops | (eof ? kInfoEof : 0u) | (err ? kInfoErr : 0u) | (reason << 20));
        lds_store(&S.parsed, q + 1);
        STAMP(PH_WRITE);
        if (err || eof)
            break;
        entry_pos = next_pos;                          // next piece: the true exit
        entry_st = next_st;
        k.P += kPiece;
        if (writer_duty(S, k.out, l, w) == 2)
            return;
        STAMP(PH_PDUTY);
    }
    // parse finished: writer only (with executor-side stores: nothing left)
    for (uint32_t spin = 0; !POM_EXEC_STORES && spin < (1u << 22); spin++) {
        if (writer_duty(S, k.out, l, w) != 0)
            break;
        __builtin_amdgcn_s_sleep(POM_WRITER_SLEEP);
    }
    STAMP(PH_PSLOT);
}

// ---------------------------------------------------------------------------
// Source buffer (executor).  Literal runs and far matches (whose source may
// have left the ring by the time their step runs) get their source span
// copied into S.src once per window -- one batched global round trip -- and
// then read LDS like everything else.  Literal spans come first (they are
// short), then far sources, each class a prefix in window order while the
// buffer lasts.  Ops that do not fit read HBM in their steps: literals
// through linear addresses from kLinHbm (input position + kLinHbm).
//
// Where output bytes are (carry = output before this window): the ring holds
// every position >= carry - kRing, and the executor waited for `landed` >=
// carry - kRing, so every position below `landed` is in HBM.  Sources lie
// below carry (db + span <= carry is required).
// Far ops are never forwarded (their sources lie below the window), so the
// copy is issued before forwarding -- which then hands buffer sources on to
// the ops that forward to them -- and only committed to LDS after it, so the
// loads' latency hides under the forwarding rounds.
// ---------------------------------------------------------------------------
// Executor: waits until the writer published landed >= need (asking for it
// through S.need).
__device__ __forceinline__ uint32_t wait_landed(FastLds& S, uint32_t need, uint32_t seen,
                                                bool& refuse)
{
    if (seen >= need)
        return seen;
    seen = lds_load(&S.landed);
    if (seen >= need)
        return seen;
    lds_store(&S.need, need);
    for (uint32_t spin = 0; seen < need; spin++) {
        if (spin > (1u << 20)) {               // writer stuck: let the exact path redo it
            refuse = true;
            break;
        }
        __builtin_amdgcn_s_sleep(POM_EXEC_SLEEP);
        seen = lds_load(&S.landed);
    }
    return seen;
}

struct SrcCopy {
    uint32_t v[4];          // this lane's buffer dwords 4l .. 4l+3 (first aligned dword)
    uint32_t v1[4];         // (the next aligned dword, for unaligned input)
    uint32_t sh;            // funnel shift of dword i at bits 2i..2i+1
    uint32_t used;          // buffer dwords filled (0: nothing copied)
    bool miss;              // (diagnostics) some candidate did not fit
};

__device__ __forceinline__ SrcCopy src_issue(FastLds& S, const Blk& k, uint32_t l, uint32_t nwin,
                                             uint32_t carry, uint32_t landed, uint32_t o,
                                             uint32_t L, uint32_t dp,
                                             bool lit, uint32_t ipos, uint32_t& db)
{
    SrcCopy fc;
    fc.used = 0;
    fc.miss = false;
    const uint32_t span = dp ? dp : L;
    const bool litc = l < nwin && lit && L != 0;
    // some byte may be read from below the ring: a step starting at xs reads
    // the ring down to xs - kRing, and the step of the op's last chunk starts
    // after o + (dp ? L : 0) - kStepSpan
    const bool far = l < nwin && !lit && db + span <= carry &&
                     db + kRing < o + (dp ? L : 0u) + kStepSpan;
    if (!wave_ballot(litc || far))
        return fc;
    const uint32_t sdw = litc ? ipos >> 2 : db >> 2;           // first source dword
    const uint32_t nd_lit = litc ? ((ipos + L + 3u) >> 2) - sdw : 0u;
    const uint32_t nd_far = far ? ((db + span + 3u) >> 2) - sdw : 0u;
    const uint32_t cl = wave_incl_scan(nd_lit);
    const uint32_t lit_total = lane_read(cl, kWave - 1);
    const uint32_t cf = wave_incl_scan(nd_far) + lit_total;
    const uint32_t nd = nd_lit + nd_far;
    const uint32_t cum = litc ? cl : cf;
    const bool acc = (litc || far) && cum <= kSrcDw;          // the buffer takes a prefix of each
    const uint64_t accl = wave_ballot(acc && litc);
    const uint64_t accf = wave_ballot(acc && far);
    fc.miss = wave_ballot((litc || far) && !acc) != 0;
    if (!(accl | accf))
        return fc;
    const uint32_t used_l = accl ? lane_read(cl, 63u - (uint32_t)__builtin_clzll(accl)) : 0u;
    const uint32_t used_f = accf ? lane_read(cf, 63u - (uint32_t)__builtin_clzll(accf)) : lit_total;
    const uint32_t used = accf ? used_f : used_l;
    fc.used = used;
    // Buffer dword t -> its op, as in the gather steps: flag each op's first
    // buffer dword (S.flags, one byte per dword), scan the flag counts; the
    // r-th op in buffer order has (source dword - buffer dword) at delta[r],
    // bit 31 set for an input source (the window's op records are not written
    // yet, so their space is free).
    uint32_t* const delta = (uint32_t*)S.wop;
    S.flags[l] = 0;
    wave_order();
    const uint32_t nl = (uint32_t)__builtin_popcountll(accl);
    const uint32_t rank = litc
        ? __builtin_amdgcn_mbcnt_hi((uint32_t)(accl >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)accl, 0u))
        : nl + __builtin_amdgcn_mbcnt_hi((uint32_t)(accf >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)accf, 0u));
    if (acc) {
        ((uint8_t*)S.flags)[cum - nd] = 1;
        delta[rank] = ((sdw - (cum - nd)) & 0x7FFFFFFFu) | (litc ? 0x80000000u : 0u);
    }
    wave_order();
    const uint32_t f = S.flags[l];
    const uint32_t nst = (uint32_t)__builtin_popcount(f);
    const uint32_t jb = wave_incl_scan(nst) - nst - 1u;      // ops starting before 4l, minus 1
    // every load first, then the funnels: one batched round trip
    const uintptr_t in_last = ((uintptr_t)k.in + k.z - 1) & ~(uintptr_t)3;   // last dword with input
    uint32_t w0[4], w1[4], sh[4];
    bool hbm[4];
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) {
        const uint32_t t = l * 4 + i;                        // buffer dword
        const uint32_t j = (jb + (uint32_t)__builtin_popcount(f & ((2u << (8 * i)) - 1u))) & 63u;
        const uint32_t dj = delta[j];
        const uint32_t a = ((t + dj) & 0x3FFFFFFFu) * 4u;   // source byte offset, dword aligned
        const bool need = t < used;
        const bool in_src = (dj & 0x80000000u) != 0;
        // input: any byte address (two aligned dwords, the second only while it
        // holds input); output: 16-byte aligned, below `landed` in HBM
        const uintptr_t pa = (uintptr_t)(in_src ? k.in + a : k.out + a);
        const uintptr_t qa = pa & ~(uintptr_t)3;
        sh[i] = (uint32_t)(pa & 3);
        hbm[i] = need && (in_src || a + 4u <= landed);
        const uintptr_t qb = in_src && qa + 4 <= in_last ? qa + 4 : qa;
        w0[i] = S.ring[(a & kRingMask) >> 2];
        w1[i] = 0;
        if (hbm[i]) {
#if POM_SRC_SC1
            w0[i] = __hip_atomic_load((uint32_t*)qa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            w1[i] = __hip_atomic_load((uint32_t*)qb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
            w0[i] = __builtin_nontemporal_load((gdword*)qa);
            w1[i] = __builtin_nontemporal_load((gdword*)qb);
#endif
        }
    }
    // (funnels in src_commit: the loads' latency hides under forwarding)
    fc.sh = 0;
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) {
        fc.v[i] = w0[i];
        fc.v1[i] = w1[i];
        fc.sh |= (hbm[i] ? sh[i] : 0u) << (2 * i);
    }
    if (acc)
        db = kLitFlag | (kSrcOff + 4u * (cum - nd) + ((litc ? ipos : db) & 3u));
    return fc;
}

__device__ __forceinline__ void src_commit(FastLds& S, uint32_t l, const SrcCopy& fc)
{
    if (!fc.used)
        return;
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) {
        const uint32_t sh = (fc.sh >> (2 * i)) & 3u;
        if (l * 4 + i < fc.used)
            S.src[l * 4 + i] = sh ? funnel(fc.v[i], fc.v1[i], sh) : fc.v[i];
    }
}

// ---------------------------------------------------------------------------
// Op-slot pool.  The scratch holds `nsets` op-slot sets, as many as there are
// workgroups resident at once, not one per block.  A workgroup takes a set
// when it starts and returns it when both its waves are done.  The sets are
// split over kPoolParts partitions (block b uses partition b mod parts) so
// that the workgroups starting together do not all hit one atomic counter;
// within partition p (count_p sets p, p + parts, ...):
//   take:   i = take_p++; i < count_p is set p + i * parts, fresh; a later i
//           waits for partition p's (i - count_p)-th return, published in ring
//           entry (i - count_p) mod count_p as {sequence number + 1, set};
//   return: j = ret_p++; that ring entry for j = {j + 1, set}.
// A workgroup waits only while every set of its partition is held by a
// running workgroup (resident, so it finishes): no deadlock, whatever the
// occupancy or dispatch order.  (The wait is still bounded: after ~1 s the
// block goes to the exact decoder, which needs no op slots.)
// ---------------------------------------------------------------------------
constexpr uint32_t kPoolParts = 32;
constexpr uint32_t kPoolStride = 64;             // u32 words per partition (256 B: two 128-B lines)

static_assert(kPoolParts * kPoolStride * 4 == LZO_MI355X_FAST_POOL_BYTES, "pool counters");

struct OpPool {
    uint32_t* ctr;                               // [parts][kPoolStride]: take at 0, return at 32
    unsigned long long* ring;                    // entry p + k * parts: partition p's k-th slot
    uint32_t nsets;
};

__device__ __forceinline__ uint32_t pool_parts(uint32_t nsets)
{
    return nsets < kPoolParts ? nsets : kPoolParts;
}

constexpr uint32_t kNoSet = 0xFFFFFFFFu;

__device__ uint32_t opset_take(const OpPool& P, uint32_t b)
{
    const uint32_t parts = pool_parts(P.nsets), p = b % parts;
    const uint32_t count = (P.nsets - p + parts - 1) / parts;
    const uint32_t i = atomicAdd(&P.ctr[p * kPoolStride], 1u);
    if (i < count)
        return p + i * parts;
    const uint32_t j = i - count;
    const unsigned long long want = (unsigned long long)(j + 1) << 32;
    unsigned long long* const e = &P.ring[p + (j % count) * parts];
    for (uint32_t spin = 0; spin < (1u << 22); spin++) {
        // relaxed: only the set number passes (an acquire would invalidate the L2)
        const unsigned long long v = __hip_atomic_load(e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((v & ~0xFFFFFFFFull) == want)
            return (uint32_t)v;
        __builtin_amdgcn_s_sleep(8);
    }
    return kNoSet;
}

__device__ void opset_return(const OpPool& P, uint32_t set)
{
    const uint32_t parts = pool_parts(P.nsets), p = set % parts;
    const uint32_t count = (P.nsets - p + parts - 1) / parts;
    const uint32_t j = atomicAdd(&P.ctr[p * kPoolStride + 32], 1u);
    // relaxed: the op slots carry nothing to the next user, and every access
    // to them has completed (the parser waits for its stores before publishing
    // a piece; the executor has used what it read).  A release here would write
    // back the XCD's whole L2 (the block's fresh output) once per block.
    __hip_atomic_store(&P.ring[p + (j % count) * parts], ((unsigned long long)(j + 1) << 32) | set,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Lane 0 of each wave when it is done with block b.  The second wave out
// publishes the block -- by then the executor has decided (state 1: finished,
// 2: refused) and the writer has landed what it could -- and returns the op
// set.  A writer that gave up (it polls for a bounded time) leaves bytes
// unstored: that block goes to the exact decoder like any refusal.
__device__ void block_close(FastLds& S, uint32_t b, uint32_t* __restrict__ out_len,
                            int32_t* __restrict__ status, uint32_t* __restrict__ fallback,
                            uint32_t* __restrict__ fallback_ids, const OpPool& P)
{
    if (__hip_atomic_fetch_add(&S.done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
        return;                                    // the other wave closes the block
    const uint32_t st = lds_load(&S.state);
    const uint32_t prod = lds_load(&S.produced);
    if (st == 1 && lds_load(&S.landed) == prod) {
        out_len[b] = prod;
        status[b] = 0;
    } else {
        status[b] = kFallback;
        out_len[b] = 0xFA110000u | (st == 2 ? lds_load(&S.why) : (uint32_t)RS_WRITER);  // (diagnostics)
        const uint32_t at = atomicAdd(&fallback[0], 1u);
        fallback_ids[at] = b;
    }
    if (S.opset != kNoSet)
        opset_return(P, S.opset);
}

template <bool STAMPS>
__global__ __launch_bounds__(2 * kWave, POM_WAVES_PER_EU) void lzo1x_decode_fast_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ src_len, uint8_t* __restrict__ dst,
    const uint64_t* __restrict__ dst_off, const uint32_t* __restrict__ dst_cap,
    uint32_t* __restrict__ out_len, int32_t* __restrict__ status,
    uint32_t* __restrict__ fallback, uint32_t* __restrict__ fallback_ids,
    uint2* __restrict__ ops, uint32_t nblocks,
    uint32_t prio_from, uint64_t* __restrict__ stamps, uint32_t* __restrict__ pool,
    unsigned long long* __restrict__ ring, uint32_t nsets, const uint32_t* __restrict__ order)
{
    __shared__ FastLds S;
    const uint32_t bi = blockIdx.x;                  // start order
    if (bi >= nblocks)
        return;
    const uint32_t b = order ? order[bi] : bi;       // (largest first: lzo_mi355x_launch_order_by_size)
    const bool last_round = bi >= prio_from;
    const uint32_t l = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x == 0) {
        S.produced = 0;
        S.issued = 0;
        S.landed = 0;
        S.need = 0;
        S.state = 0;
        S.parsed = 0;
        S.consumed = 0;
        S.done = 0;
        S.opset = opset_take(OpPool{pool, ring, nsets}, bi);
    }
    if (threadIdx.x < kWave)
        S.flags[threadIdx.x] = 0;             // chunk tags start at 0x80000001
    for (uint32_t d = threadIdx.x; d < 2 * 16 * 8; d += 2 * kWave) {
        const uint32_t h = d >> 7, p = (d >> 3) & 15, i0 = (d & 7) * 4;
        uint32_t v = 0;
        for (uint32_t i = 0; i < 4; i++) {
            const uint32_t idx = p ? (i0 + i) % p : 0u;
            const uint32_t sel = h ? (idx >= 8 ? idx - 8 : 12u) : (idx < 8 ? idx : 12u);
            v |= sel << (8 * i);
        }
        S.psel[h][p][d & 7] = v;
    }
    __syncthreads();

    uint64_t acc[PH_N] = {};
    Blk k;
    k.in = src + src_off[b];
    k.z = src_len[b];
    k.out = dst + dst_off[b];
    k.cap = dst_cap[b];
    k.P = 0;
    k.staged = 0;
    const uint32_t opset = __builtin_amdgcn_readfirstlane(S.opset);
    uint2* const gops = ops + (size_t)(opset == kNoSet ? 0u : opset) * (kSlots * kOpMax);

    // The exact decoder takes: destinations not 16-byte aligned, empty or huge
    // blocks (lengths up to 255 * z must not wrap 32 bits).
    bool refuse = ((uintptr_t)k.out & 15) != 0 || k.z >= (1u << 24) || k.z == 0 || opset == kNoSet;
    uint32_t reason = opset == kNoSet ? (uint32_t)RS_POOL : refuse ? (uint32_t)RS_HEAD : (uint32_t)RS_NONE;
    if (wave == 1) {
        if (POM_PRIO && last_round)
            __builtin_amdgcn_s_setprio(POM_PARSER_PRIO);
        if (!refuse)
            parser_wave<STAMPS>(S, k, gops, l, acc);
        if (STAMPS && l == 0)
            for (int i = 0; i < PH_N; i++)
                if (parser_slot(i))
                    stamps[(size_t)b * kStampSlots + i] = acc[i];
        if (l == 0)
            block_close(S, b, out_len, status, fallback, fallback_ids, OpPool{pool, ring, nsets});
        return;
    }

    uint64_t tmark = STAMPS ? __builtin_amdgcn_s_memtime() : 0;
    // (LDS addresses as offsets from one readfirstlane'd base: the compiler
    // otherwise re-derives each generic-to-LDS cast, with its null check, in
    // every step)
    const uint32_t base = __builtin_amdgcn_readfirstlane(lds_off(&S));
    const uint32_t psel0 = base + (uint32_t)offsetof(FastLds, psel);
    const uint32_t psel1 = psel0 + (uint32_t)sizeof(S.psel[0]);
    uint32_t carry = 0;                        // output produced so far
    uint32_t issued_seen = 0, landed_seen = 0; // last `issued` / `landed` read
    // (POM_EXEC_STORES) output bytes whose stores this wave issued; landed_seen
    // is then the stored count at its last vmcnt(0)
    uint32_t stored = 0;
    uint32_t tag = 0;                          // step counter for the chunk tags
    uint32_t published = 0;                    // last `produced` handed to the writer
    uint32_t q = 0, w0 = 0, total_ops = 0;     // piece, window start, piece's op count
    bool have_piece = false, eofq = false;
    uint64_t pf = 0;                           // prefetched op record of the next window
    bool have_pf = false;

    while (!refuse) {
        if (!have_piece) {
            // ---- the parser's piece q -------------------------------------------
            for (uint32_t spin = 0; lds_load(&S.parsed) <= q; spin++) {
                if (spin > (1u << 20)) {       // parser stuck: let the exact path redo it
                    refuse = true;
                    reason = RS_EWAIT;
                    break;
                }
                __builtin_amdgcn_s_sleep(POM_EXEC_SLEEP);
            }
            if (refuse)
                break;
            const uint32_t info = lds_load(&S.pinfo[q & (kSlots - 1)]);
            STAMP(PH_EWAIT);
            if (info & kInfoErr) {
                refuse = true;
                reason = (info >> 20) & 15u;
                break;
            }
            eofq = (info & kInfoEof) != 0;
            total_ops = info & 0xFFFFu;
#ifdef POM_EXEC_SKIP
            total_ops = 0;                     // (measurement only: the parser alone)
#endif
            have_piece = true;
            w0 = 0;
            have_pf = false;
        }
        if (w0 >= total_ops) {                 // piece done: its slot is free again
            lds_store(&S.consumed, q + 1);
            if (eofq)
                break;                         // EOF consumed
            q++;
            have_piece = false;
            continue;
        }
        const uint2* const slot = gops + (q & (kSlots - 1)) * kOpMax;
        {
            const uint32_t nwin = total_ops - w0 < (uint32_t)kWave ? total_ops - w0 : (uint32_t)kWave;
            uint32_t L = 0, Sv = 0;
            {
                // agent scope: served by L2, never by a stale L1 line of the slot's last use
                uint64_t r = pf;
                if (!have_pf && l < nwin)
                    r = __hip_atomic_load((const uint64_t*)(slot + w0 + l), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
                if (l < nwin) {
                    L = (uint32_t)r;
                    Sv = (uint32_t)(r >> 32);
                }
            }
            // what the source copy does not find in the ring (below carry -
            // kRing) it reads from HBM: that output must have landed
            if (!POM_EXEC_STORES && carry > kRing)
                landed_seen = wait_landed(S, carry - kRing, landed_seen, refuse);
            if (refuse) {
                reason = RS_LANDED;
                break;
            }
            // prefetch the next window's op records of this piece (with
            // executor-side stores: after the landed check below, whose
            // vmcnt(0) would otherwise wait for it)
            have_pf = w0 + kWave < total_ops;
            auto prefetch_records = [&]() {
                if (have_pf && w0 + kWave + l < total_ops)
                    pf = __hip_atomic_load((const uint64_t*)(slot + w0 + kWave + l), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
            };
            if (!POM_EXEC_STORES)
                prefetch_records();
            STAMP(PH_WLOAD);
            if (STAMPS)
                acc[CN_WINDOWS] += 1;
            const uint32_t inc = wave_incl_scan(L);
            const uint32_t o = carry + inc - L;
            const uint32_t wtotal = lane_read(inc, kWave - 1);
            if (carry + wtotal < carry || carry + wtotal > k.cap) {
                refuse = true;                         // OUTPUT_OVERRUN (or wrap)
                reason = RS_OVERRUN;
                break;
            }
            const bool lit = (Sv & kLitFlag) != 0;
            const bool lb = l < nwin && !lit && Sv > o;     // LOOKBEHIND_OVERRUN
            if (wave_ballot(lb)) {
                refuse = true;
                reason = RS_LOOKBEHIND;
                break;
            }
            // ---- op descriptors: byte x of op j reads
            //   src[b + ((x - o) mod p)]   (p == 0: src[b + x - o])
            // at linear address b (kLitFlag set: the LDS source buffer, or from
            // kLinHbm the input in HBM) or in the output (ring / HBM).  A match
            // starts as b = o - d, p = d if it overlaps itself (d < L).
            const uint32_t ipos = Sv & ~kLitFlag;
            uint32_t db = lit ? kLitFlag | (kLinHbm + ipos) : o - Sv;
            uint32_t dp = (!lit && Sv < L) ? Sv : 0u;
            if (POM_EXEC_STORES) {
                // sources older than the ring are read back from HBM: the
                // stores of those bytes (issued before their slots were
                // reused, so stored >= carry - kRing) must have completed
                if (carry > kRing && landed_seen < carry - kRing &&
                    wave_ballot(l < nwin && !lit && db < carry - kRing)) {
                    __builtin_amdgcn_s_waitcnt(0x0F70);                      // vmcnt(0)
                    landed_seen = stored;
                }
                prefetch_records();
            }
            STAMP(PH_WSCAN);
            const SrcCopy fc = src_issue(S, k, l, nwin, carry, landed_seen, o, L, dp, lit, ipos, db);
            STAMP(PH_FARI);
            if (STAMPS && fc.used)
                acc[CN_SRCWIN] += 1;
            if (STAMPS && fc.miss)
                acc[CN_SRCMISS] += 1;
            // Source forwarding: a match whose source span lies inside one
            // earlier op of this window reads that op's source instead, so it
            // no longer waits for it.  Three parallel rounds reach the
            // sequential fixed point on ITB streams (600 -> 205 batches per
            // 64 KiB block).
            const uint32_t o_first = lane_read(o, 0);
            // periods' inverses for the mod by mulhi (forwarding moves sources,
            // never periods: the steps use them too)
            uint32_t inv = 0;
            if (wave_ballot(dp != 0))
                inv = dp ? 0xFFFFFFFFu / dp : 0u;
            for (int round = 0; round < POM_FWD_ROUNDS; round++) {
                const uint32_t span = dp ? dp : L;
                const bool need = l < nwin && !(db & kLitFlag) && db + span > o_first;
                if (!wave_ballot(need))
                    break;
                if (STAMPS)
                    acc[CN_FWD_ROUNDS] += 1;
                uint32_t k2 = 0;                       // last op with o <= db
#pragma unroll
                for (uint32_t w = 32; w >= 1; w >>= 1) {
                    const uint32_t c = k2 + w;
                    const uint32_t oc = (uint32_t)__shfl((int)o, (int)(c & 63u), kWave);
                    if (c < nwin && oc <= db)
                        k2 = c;
                }
                const uint32_t ko = (uint32_t)__shfl((int)o, (int)k2, kWave);
                const uint32_t kL = (uint32_t)__shfl((int)L, (int)k2, kWave);
                const uint32_t kb = (uint32_t)__shfl((int)db, (int)k2, kWave);
                const uint32_t kp = (uint32_t)__shfl((int)dp, (int)k2, kWave);
                const uint32_t kinv = (uint32_t)__shfl((int)inv, (int)k2, kWave);
                uint32_t r = db - ko;
                const uint32_t rr = r - kp * (uint32_t)__umulhi(r, kinv);   // (kp == 0: kinv == 0, rr == r)
                r = min(rr, rr - kp);                  // r mod kp
                const bool ok = need && k2 < l && ko <= db && db + span <= ko + kL && (!kp || r + span <= kp);
                if (ok)
                    db = kb + r;                       // (kb carries k's linear flag)
            }
            STAMP(PH_FWD);
            src_commit(S, l, fc);
            // end of each output-sourced op's source span: a batch may not read
            // its own output
            const bool outsrc = l < nwin && !(db & kLitFlag);
            const uint32_t span = dp ? dp : L;
            const uint32_t send = outsrc ? db + span : 0u;
            // Chunks: op j covers the window's 16-byte chunks cs .. cs +
            // ceil(L/16) - 1, each up to 16 bytes of that op alone.
            const uint32_t nch = l < nwin ? (L + 15u) >> 4 : 0u;
            const uint32_t cinc = wave_incl_scan(nch);
            const uint32_t cs = cinc - nch;
            const uint32_t wchunks = lane_read(cinc, kWave - 1);
            S.wop[l] = make_uint4(o, db, cs, L);
            S.wper[l] = make_uint2(dp, inv);
            wave_order();
            STAMP(PH_FARC);
            uint32_t s = 0;
            while (s < nwin) {
                const uint32_t os = lane_read(o, s);
                // lanes l > s reading output at or after os (send is 0 unless outsrc)
                const uint64_t bm = mask_lt(os, send) & (~1ull << s);
                const uint32_t e = bm ? (uint32_t)__builtin_ctzll(bm) : nwin;
                const uint32_t c_beg = lane_read(cs, s);
                const uint32_t c_end = e < nwin ? lane_read(cs, e) : wchunks;
                const bool starter = l >= s && l < e;
                STAMP(PH_BATCH);
                if (STAMPS)
                    acc[CN_BATCHES] += 1;
                // ---- batch [s, e): chunks [c_beg, c_end), 64 per step (1 KiB) ----
                uint32_t jcarry = s;                   // ops of the batch started before C
                for (uint32_t C = c_beg; C < c_end; C += kWave) {
                    // chunk -> op: each op starting in this step tags its first
                    // chunk's slot; lane l's op is the last one started at or
                    // before chunk C + l (a ballot and mbcnt, no scan).
                    tag++;
                    const uint32_t tagv = tag | 0x80000000u;   // src_issue's byte flags never set bit 31
                    S.flags[starter && cs >= C && cs < C + kWave ? cs - C : (uint32_t)kWave] = tagv;
                    wave_order();
                    const bool st0 = S.flags[l] == tagv;
                    const uint64_t Mb = wave_ballot(st0);
                    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(Mb >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)Mb, 0u));
                    const uint32_t j = (jcarry + below + (st0 ? 0u : ~0u)) & 63u;
                    jcarry += (uint32_t)__builtin_popcountll(Mb);
                    const uint4 op = S.wop[j];
                    const uint2 pr = S.wper[j];
                    const uint32_t c = C + l;
                    const bool live = c < c_end;
                    const uint32_t k16 = (c - op.z) * 16u;
                    const uint32_t x = op.x + k16;
                    const uint32_t rem = op.w - k16;
                    const uint32_t len = live ? (rem < 16u ? rem : 16u) : 0u;
                    const uint32_t nl = c_end - C < (uint32_t)kWave ? c_end - C : (uint32_t)kWave;
                    const uint32_t xs = lane_read(x, 0);
                    const uint32_t step_end = POM_EXEC_STORES ? 0u : lane_read(x + len, nl - 1);
                    STAMP(PH_FLAGS);
                    // ring space: the stores of what the slots of [xs, step_end)
                    // held must have been issued.  Executor-side stores: this
                    // wave issues them itself, whole 1-KiB pieces of final
                    // output (below xs), trailing its production by
                    // POM_STORE_LAG so that a read back from HBM rarely waits
                    // for a store still in flight.
                    if (POM_EXEC_STORES) {
                        const uint32_t want = xs > POM_STORE_LAG ? xs - POM_STORE_LAG : 0u;
                        // (xs + kStepSpan bounds step_end without its readlane)
                        while (stored + kChunk <= want || stored + kRing < (POM_EXEC_STORES ? xs + kStepSpan : step_end)) {
                            exec_store_chunk(S, k.out, l, stored);
                            stored += kChunk;
                        }
                    }
                    for (uint32_t spin = 0; !POM_EXEC_STORES && step_end > issued_seen + kRing; spin++) {
                        if (spin > (1u << 20)) {       // writer stuck: let the exact path redo it
                            refuse = true;
                            reason = RS_SPACE;
                            break;
                        }
                        if (spin) {
                            if (spin == 1) {           // hand over what is final
                                lds_store(&S.produced, xs);
                                published = xs;
                            }
                            __builtin_amdgcn_s_sleep(POM_EXEC_SLEEP);
                        }
                        issued_seen = __builtin_amdgcn_readfirstlane(lds_load(&S.issued));
                    }
                    if (refuse)
                        break;
                    STAMP(PH_SPACE);
                    if (STAMPS)
                        acc[CN_STEPS] += 1;
                    // ---- source bytes of the chunk ---------------------------
                    // byte i reads src[b + ((k16 + i) mod p)] (p == 0: b + k16 + i)
                    const uint32_t p = pr.x;
                    const bool lin = (op.y & kLitFlag) != 0;
                    const uint32_t bb = op.y & ~kLitFlag;
                    // (p == 0: the inverse is 0, so r0 stays k16 without a branch)
                    uint32_t r0 = k16 - p * (uint32_t)__umulhi(k16, pr.y);
                    r0 = min(r0, r0 - p);
                    const bool small = p != 0 && p < 16u;       // pattern expansion
                    const uint32_t n1 = p - r0;                 // (p >= 16) bytes before the wrap
                    const bool two = p >= 16u && n1 < len;      // the chunk wraps the period
                    const uint32_t aA = small ? bb : bb + r0;
                    const uint32_t aB = bb + r0 - p;            // wrapped part, read p lower
                    const uint64_t mlive = mask_lt(c, c_end);
                    const uint64_t mtwo = mask_ge(p, 16u) & mask_lt(n1, len);
                    const uint64_t smask = mlive & mask_lt(p - 1u, 15u);
                    const uint32_t ps = small ? p * 32u + r0 : 0u;   // selectors of the expansion
                    // LDS: the ring (its mirror takes reads across the end) or
                    // the linear source buffer; HBM: literals beyond the buffer,
                    // output below the ring (a + kRing < xs: those slots were
                    // overwritten before this step)
                    // (as signed distances, without branches: lin -> a - kLinHbm >= 0,
                    // else xs - kRing - 1 - a >= 0)
                    const uint32_t hbase = lin ? kLinHbm : 0u, hlim = lin ? 0u : xs - kRing - 1u;
                    const uint32_t kA = lin ? aA - hbase : hlim - aA, kB = lin ? aB - hbase : hlim - bb;
                    const bool hA = live && (int32_t)kA >= 0;
                    const bool hB = live && two && (int32_t)kB >= 0;
                    const uint64_t mhbm = mlive & (mask_nonneg(kA) | (mtwo & mask_nonneg(kB)));
                    const uint32_t amask = lin ? kLdsMask : kRingMask;
                    // only the reads some lane of the step needs (uniform branches;
                    // vB / sl / sh are read only on the paths that load them)
                    uint4 vA, vB, sl, sh;
                    const bool any_two = mtwo != 0;
                    const uint32_t ra = base + (live ? aA & amask : 0u);
                    if (!smask) {
                        if (!any_two)
                            vA = lds_read16(ra);
                        else
                            lds_read16x2(ra, base + (two ? aB & amask : 0u), vA, vB);
                    } else if (!any_two) {
                        lds_read16x3(ra, psel0 + ps, psel1 + ps, vA, sl, sh);
                    } else {
                        lds_read16x4(ra, base + (two ? aB & amask : 0u), psel0 + ps, psel1 + ps, vA, vB, sl,
                                     sh);
                    }
                    if (mhbm) {
                        if ((mhbm & mask_nonneg(op.y)) && xs + 16u > kRing) {  // (!lin: bit 31 clear)
                            if (!POM_EXEC_STORES)
                                landed_seen = wait_landed(S, xs + 16u - kRing, landed_seen, refuse);
                            else if (landed_seen < xs + 16u - kRing) {
                                // (stored >= step_end - kRing covers every byte read here:
                                // sources below xs - kRing, 16 bytes from there)
                                while (stored < xs + 16u - kRing) {
                                    exec_store_chunk(S, k.out, l, stored);
                                    stored += kChunk;
                                }
                                __builtin_amdgcn_s_waitcnt(0x0F70);          // vmcnt(0)
                                landed_seen = stored;
                            }
                        }
                        const uint8_t* gb = lin ? k.in - kLinHbm : k.out;
                        if (hA)
                            vA = global_read16(gb + aA, 0u, small ? p : two ? n1 : len);
                        if (hB)                        // bytes n1.. of the span: from b on
                            vB = global_read16(gb + bb - n1, n1, len);
                    }
                    if (refuse)
                        break;
                    uint4 v = vA;
                    if (any_two) {
                        // bytes i < n1 from vA, the rest from vB
                        const uint32_t n = two ? n1 : 16u;
                        // bytes below n (1 <= n <= 16) as two 64-bit masks, no
                        // branches: (2 << (8k - 1)) - 1 is k bytes for k = 1..8
                        const uint32_t nl = n < 8u ? n : 8u, nh = n > 8u ? n - 8u : 1u;
                        const uint64_t mlo = (2ull << (8u * nl - 1u)) - 1ull;
                        const uint64_t mhi = n > 8u ? (2ull << (8u * nh - 1u)) - 1ull : 0ull;
                        const uint32_t m0 = (uint32_t)mlo, m1 = (uint32_t)(mlo >> 32);
                        const uint32_t m2 = (uint32_t)mhi, m3 = (uint32_t)(mhi >> 32);
                        v.x = (vA.x & m0) | (vB.x & ~m0);
                        v.y = (vA.y & m1) | (vB.y & ~m1);
                        v.z = (vA.z & m2) | (vB.z & ~m2);
                        v.w = (vA.w & m3) | (vB.w & ~m3);
                    }
                    if (smask) {
                        if (small) {
                            v.x = __builtin_amdgcn_perm(vA.y, vA.x, sl.x) | __builtin_amdgcn_perm(vA.w, vA.z, sh.x);
                            v.y = __builtin_amdgcn_perm(vA.y, vA.x, sl.y) | __builtin_amdgcn_perm(vA.w, vA.z, sh.y);
                            v.z = __builtin_amdgcn_perm(vA.y, vA.x, sl.z) | __builtin_amdgcn_perm(vA.w, vA.z, sh.z);
                            v.w = __builtin_amdgcn_perm(vA.y, vA.x, sl.w) | __builtin_amdgcn_perm(vA.w, vA.z, sh.w);
                        }
                    }
                    // ---- destination: the ring at x -----------------------------
                    const uint32_t xd = x & kRingMask;
#if POM_WRAP_MIRROR
                    // a chunk that wraps the ring end runs on into the mirror
                    // of ring[0, 16); the ring's head is then copied back from
                    // the mirror (after every lane's mirror write: bytes other
                    // lanes put in ring[0, 16) this step are in the mirror too)
                    if (live) {
                        lds_write_part(base + xd, v, len);
                        if (xd < 16u)                  // keep the mirror of ring[0, 16)
                            lds_write_part(base + kRing + xd, v, len);
                    }
                    if (mask_lt(kRing, xd + len) && l == 0)     // (len is 0 off the step)
                        lds_write16(base, lds_read16(base + kRing));
#else
                    const bool wcross = live && xd + len > kRing;
                    if (live && !wcross) {
                        lds_write_part(base + xd, v, len);
                        if (xd < 16u)                  // keep the mirror of ring[0, 16)
                            lds_write_part(base + kRing + xd, v, len);
                    }
                    if (mask_lt(kRing, xd + len)) {     // (wcross; len is 0 off the step)
                        if (wcross) {                  // destination wraps the ring end
                            const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
                            uint8_t* ldsw = (uint8_t*)&S;
#pragma unroll
                            for (uint32_t i = 0; i < 16; i++)
                                if (i < len) {
                                    const uint32_t y = (x + i) & kRingMask;
                                    const uint8_t bv = (uint8_t)(wv[i >> 2] >> (8 * (i & 3)));
                                    ldsw[y] = bv;
                                    if (y < 16u)
                                        ldsw[kRing + y] = bv;
                                }
                        }
                    }
#endif
                    wave_order();
                    STAMP(PH_GATHER);
                    // bytes below step_end are final: hand them over once a
                    // 1-KiB store chunk is complete (the writer stores whole chunks)
                    if (!POM_EXEC_STORES && (!POM_LAZY_PUB || (step_end ^ published) >= kChunk)) {
                        lds_store(&S.produced, step_end);
                        published = step_end;
                    }
                    STAMP(PH_PUB);
                }
                if (refuse)
                    break;
                s = e;
            }
            if (refuse)
                break;
            carry += wtotal;
            if (POM_PRIO && last_round)
                prio_by_bytes_left(k.cap > carry ? k.cap - carry : 0u);
            wave_order();
        }
        w0 += kWave;
    }

    if (STAMPS)
        acc[CN_REASON] = reason | (q << 4) | ((uint64_t)w0 << 32);
    if (STAMPS && l == 0)
        for (int i = 0; i < PH_N; i++)
            if (!parser_slot(i))
                stamps[(size_t)b * kStampSlots + i] = acc[i];
    if (POM_EXEC_STORES && !refuse) {
        // the rest of the output, then wait for every store to land
        for (; stored < carry; stored += kChunk)
            exec_store(S, k.out, l, stored, carry - stored < kChunk ? carry : stored + kChunk);
        __builtin_amdgcn_s_waitcnt(0x0F70);                  // vmcnt(0)
        stored = carry;
    }
    if (l == 0) {
        if (refuse) {
            lds_store(&S.why, reason);
            lds_store(&S.state, 2u);
        } else {
            if (POM_EXEC_STORES)
                lds_store(&S.landed, carry);                 // (block_close checks landed == produced)
            lds_store(&S.produced, carry);
            lds_store(&S.state, 1u);
        }
        block_close(S, b, out_len, status, fallback, fallback_ids, OpPool{pool, ring, nsets});
    }
}
#undef STAMP

}  // namespace

// Op-slot sets: as many as workgroups are resident at once, 16 per CU (LDS
// and 8 waves per SIMD).
extern "C" uint32_t lzo_mi355x_fast_resident_blocks(void)
{
    static int cus[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64)
        return 256u * (2 * POM_WAVES_PER_EU);
    if (!cus[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            return 256u * (2 * POM_WAVES_PER_EU);
        cus[dev] = n;
    }
    return (uint32_t)cus[dev] * (2 * POM_WAVES_PER_EU);
}

// Bytes of one op-slot set (lzo_host.c sizes the scratch).
extern "C" size_t lzo_mi355x_fast_ops_bytes_per_block(void)
{
    return (size_t)kSlots * kOpMax * sizeof(uint2);
}

// First block of the final round: the last `resident` blocks.
static uint32_t prio_from(uint32_t nblocks, uint32_t resident)
{
    return nblocks > resident ? nblocks - resident : 0u;
}

extern "C" int lzo_mi355x_launch_decompress_fast(const uint8_t* src, const uint64_t* src_off,
                                                 const uint32_t* src_len, uint8_t* dst,
                                                 const uint64_t* dst_off, const uint32_t* dst_cap,
                                                 uint32_t* out_len, int32_t* status,
                                                 uint32_t* fallback, uint32_t* fallback_ids,
                                                 uint32_t* pool, void* ring, void* ops,
                                                 uint32_t nsets, uint32_t nblocks,
                                                 uint32_t* order, hipStream_t stream)
{
    if (nblocks == 0)
        return 0;
    if (nsets == 0)
        return -1;
    if (order && lzo_mi355x_launch_order_by_size(dst_cap, nblocks, order, stream) != 0)
        return -1;
    hipLaunchKernelGGL(lzo1x_decode_fast_kernel<false>, dim3(nblocks), dim3(2 * kWave), 0,
                       stream, src, src_off, src_len, dst, dst_off, dst_cap, out_len, status,
                       fallback, fallback_ids, (uint2*)ops, nblocks,
                       prio_from(nblocks, lzo_mi355x_fast_resident_blocks()), nullptr, pool,
                       (unsigned long long*)ring, nsets, (const uint32_t*)order);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

namespace {
// Counting sort of the block indices by key, largest 4 KiB class first (one
// workgroup: class counts in LDS, their prefix sums, then each index to its
// class's next slot; the order within a class is whatever the atomics give).
constexpr uint32_t kOrderClasses = 256;
__device__ __forceinline__ uint32_t order_class(uint32_t key)
{
    const uint32_t k = key >> 12;
    return kOrderClasses - 1u - (k < kOrderClasses - 1u ? k : kOrderClasses - 1u);
}
__global__ __launch_bounds__(1024) void lzo1x_order_kernel(const uint32_t* __restrict__ key, uint32_t n,
                                                           uint32_t* __restrict__ order)
{
    __shared__ uint32_t cnt[kOrderClasses];
    const uint32_t t = threadIdx.x;
    if (t < kOrderClasses)
        cnt[t] = 0;
    __syncthreads();
    for (uint32_t i = t; i < n; i += blockDim.x)
        atomicAdd(&cnt[order_class(key[i])], 1u);
    __syncthreads();
    if (t == 0) {
        uint32_t sum = 0;
        for (uint32_t c = 0; c < kOrderClasses; c++) {
            const uint32_t v = cnt[c];
            cnt[c] = sum;
            sum += v;
        }
    }
    __syncthreads();
    for (uint32_t i = t; i < n; i += blockDim.x)
        order[atomicAdd(&cnt[order_class(key[i])], 1u)] = i;
}
}  // namespace

extern "C" int lzo_mi355x_launch_order_by_size(const uint32_t* key, uint32_t n, uint32_t* order,
                                               hipStream_t stream)
{
    if (n == 0)
        return 0;
    hipLaunchKernelGGL(lzo1x_order_kernel, dim3(1), dim3(1024), 0, stream, key, n, order);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Diagnostic: the same decoder with per-phase cycle stamps (kStampSlots x u64 per block).
extern "C" int lzo_mi355x_debug_decompress_fast_stamps(
    const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len, uint8_t* dst,
    const uint64_t* dst_off, const uint32_t* dst_cap, uint32_t* out_len, int32_t* status,
    uint32_t* fallback, uint32_t* fallback_ids, uint32_t* pool, void* ring, void* ops,
    uint32_t nsets, uint32_t nblocks, uint64_t* stamps, hipStream_t stream)
{
    if (nblocks == 0)
        return 0;
    if (nsets == 0)
        return -1;
    hipLaunchKernelGGL(lzo1x_decode_fast_kernel<true>, dim3(nblocks), dim3(2 * kWave), 0,
                       stream, src, src_off, src_len, dst, dst_off, dst_cap, out_len, status,
                       fallback, fallback_ids, (uint2*)ops, nblocks,
                       prio_from(nblocks, lzo_mi355x_fast_resident_blocks()), stamps, pool,
                       (unsigned long long*)ring, nsets, nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
