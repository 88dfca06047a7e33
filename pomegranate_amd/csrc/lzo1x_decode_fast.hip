// lzo1x_decode_fast.hip -- the throughput LZO1X decoder for MI355X (gfx950).
//
// One 64-lane wave per block.  The compressed block is processed in pieces of
// kPiece input bytes; each piece goes through:
//
//  1. PARSE (lane = kSeg-byte input segment).  The LZO1X grammar
//     (lib/minilzo.c:3308-3699) is a state machine
//     over instruction starts (pos, state), state A (top), B (after a literal
//     run) or C (after 1-3 trailing literals).  Every lane decodes
//     speculatively from kLook bytes before its segment (state A, restarting
//     one byte later whenever the guess runs into an impossible instruction)
//     and marks the points it visits inside its segment.  Each lane then walks
//     the TRUE path from its entry (its predecessor's exit) until it lands on
//     one of its own marks (merged) or leaves the segment; the entry/exit
//     chain is iterated until no entry changes (lane 0's entry is exact, so
//     this converges; on real data speculation re-synchronises within a few
//     instructions and one round suffices).  Two more walks count and write
//     the ops (literal runs and matches) of the true path into an LDS op list
//     in stream order.
//
//  2. EXECUTE (lane = op, then lane = 4-byte output unit).  64 ops at a time:
//     a DPP prefix sum gives output offsets; the ops are cut into batches
//     whose match sources all precede the batch (no dependency inside a
//     batch), and each batch's output is produced 256 bytes per step: op
//     starts are flagged per byte in LDS, a DPP scan of the per-unit flag
//     counts gives every byte its op, and each lane gathers its 4 bytes
//     (input staging / global input for literals; the LDS output ring or,
//     beyond the ring, the already-stored HBM output for matches) and writes
//     the dword to the ring and to HBM.
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
#define POM_SEG 16
#endif
#ifndef POM_LOOK
#define POM_LOOK 24
#endif
constexpr uint32_t kSeg = POM_SEG;               // input bytes per lane per piece
constexpr uint32_t kLook = POM_LOOK;             // speculative lead-in before a segment
constexpr uint32_t kPiece = kWave * kSeg;        // 1 KiB of compressed input
constexpr uint32_t kStageBytes = kPiece + 512;
constexpr uint32_t kOpMax = 32 * kSeg;           // ops per piece
#ifndef POM_WRITER_SLEEP
#define POM_WRITER_SLEEP 127                     // idle writer sleeps ~8K cycles between polls
#endif
#ifndef POM_FWD_ROUNDS
#define POM_FWD_ROUNDS 3                         // source-forwarding rounds per window
#endif
#ifndef POM_WAVES_PER_EU
#define POM_WAVES_PER_EU 8                       // 16 blocks (decoder + writer wave) per CU
#endif
#ifndef POM_RING
#define POM_RING 4096
#endif
constexpr uint32_t kRing = POM_RING;             // recent output kept in LDS
constexpr uint32_t kRingSlack = kRing / 4;       // decoder keeps this much ring unflushed-free
constexpr uint32_t kRingMask = kRing - 1;
#ifndef POM_FAR
#define POM_FAR 1024
#endif
constexpr uint32_t kFarBytes = POM_FAR;          // per-window copy of far match sources
constexpr uint32_t kFarDw = kFarBytes / 4;
static_assert(kFarDw <= 4 * kWave, "far copy: at most 4 dwords per lane");
constexpr uint32_t kLitFlag = 0x80000000u;
constexpr uint32_t kMaxOpLen = 1u << 25;         // 64 ops per window cannot wrap 32 bits
constexpr int32_t kFallback = 0x7FFF0001;        // status: exact decoder pending

// parse states (instruction starts)
constexpr uint32_t ST_A = 0;   // top: t < 16 is a literal run
constexpr uint32_t ST_B = 1;   // after a literal run: t < 16 is a 3-byte M1 (dist > 0x800)
constexpr uint32_t ST_C = 2;   // after trailing literals: t < 16 is a 2-byte M1
constexpr uint32_t ST_F = 3;   // first byte of the stream (lib/minilzo.c:3357)
constexpr uint32_t kPosEnd = 0xFFFFFFF0u;        // exit marker: EOF reached / dead path
constexpr uint32_t kPosUnknown = 0xFFFFFFE0u;    // speculative walk gave up

struct __attribute__((aligned(16))) FastLds {
    uint32_t ring[kRing / 4];
    uint32_t far[kFarDw];     // sources of this window's far matches (beyond the ring)
    uint32_t stage[kStageBytes / 4];

    uint4 wop[kWave];         // window op: {o, source base (| kLitFlag: LDS-linear), first chunk, L (| kLitFlag: needs HBM)}
    uint2 wper[kWave];        // window op: {period, floor((2^32-1)/period)}
    uint32_t flags[kWave];    // per-step chunk tags (far_issue: per-dword byte flags)
    uint32_t sink;            // target of masked-off byte writes
    union {
        uint8_t marks[kPiece];        // parse: speculative path marks (pass 1, merge)
        uint16_t opref[kOpMax];       // then: the piece's ops as instruction references
    };
    // decoder -> writer hand-off (LDS words, workgroup scope)
    uint32_t produced;      // output bytes final in the ring
    uint32_t flushed;       // output bytes stored to HBM and landed
    uint32_t state;         // 0 running, 1 finished, 2 refused
};

constexpr uint32_t kRingOff = 0;                                  // offsetof(FastLds, ring)
constexpr uint32_t kFarOff = kRing;                               // offsetof(FastLds, far)
constexpr uint32_t kStageOff = kRing + kFarBytes;                 // offsetof(FastLds, stage)
static_assert(offsetof(FastLds, ring) == kRingOff, "layout");
static_assert(offsetof(FastLds, far) == kFarOff, "layout");
static_assert(offsetof(FastLds, stage) == kStageOff, "layout");
constexpr uint32_t kSinkOff = kStageOff + kStageBytes + (kWave * (16 + 8 + 4));   // offsetof(FastLds, sink)
static_assert(offsetof(FastLds, sink) == kSinkOff, "layout");
constexpr uint32_t kLdsMask = 0x3FFF;                              // LDS-linear address space
static_assert(sizeof(FastLds) <= kLdsMask + 1, "linear LDS addresses are masked to 16 KiB");
// 16 blocks per CU share its 160 KiB of LDS
static_assert(sizeof(FastLds) * 2 * POM_WAVES_PER_EU <= 160 * 1024, "LDS budget");

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ uint32_t lane_read(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint64_t wave_ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ void wave_order() { __atomic_signal_fence(__ATOMIC_SEQ_CST); }

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

__device__ __noinline__ Step decode_one(const FastLds& s, const Blk& k, uint32_t pos, uint32_t st)
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
// LDS round trip (three aligned dwords -> 8 bytes at pos), then selects; lanes
// decoding different instruction kinds do not diverge.  Falls back to
// decode_one otherwise (long extensions, input beyond the staging window).
// SPEC: speculative use -- never take the slow path; report it as `slow`
// (the caller restarts or re-walks exactly) instead.
template <bool SPEC = false>
__device__ __forceinline__ Step decode_step(const FastLds& s, const Blk& k, uint32_t pos, uint32_t st,
                                            bool* slow = nullptr)
{
    const uint32_t rel = pos - k.P;
    const bool inwin = rel + 12 <= kStageBytes && pos < k.z;
    // The 8 bytes at pos (read unconditionally from a clamped window offset;
    // ignored when !inwin).
    const uint32_t wi = inwin ? rel >> 2 : 0u;
    const uint32_t w0 = s.stage[wi], w1 = s.stage[wi + 1], w2 = s.stage[wi + 2];
    const uint32_t sh = 8u * (rel & 3u);
    const uint32_t lo = (uint32_t)((((uint64_t)w1 << 32) | w0) >> sh);
    const uint32_t hi = (uint32_t)((((uint64_t)w2 << 32) | w1) >> sh);
    const uint64_t b8 = ((uint64_t)hi << 32) | lo;                 // bytes pos..pos+7
#define BYTE(i) ((uint32_t)(b8 >> (8u * (i))) & 0xFFu)
    const uint32_t t = lo & 0xFFu, b1 = BYTE(1);
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
    const uint32_t o16 = BYTE(1 + e) | (BYTE(2 + e) << 8);
    const uint32_t dd4 = ((t & 8u) << 11) + (o16 >> 2);
    const uint32_t used = (m1 || m2) ? 2u : 3u + e;                // match instruction bytes
    const uint32_t tl = BYTE(used - 2) & 3u;                       // match_done, :3650
#undef BYTE
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



// 4 bytes at an arbitrary global address via two aligned dword loads (an
// aligned dword that overlaps valid bytes never leaves their page).  NT: L2
// served (the vector L1 is not coherent with this wave's earlier stores).
typedef __attribute__((address_space(1))) const uint32_t gdword;

// 4 bytes at an arbitrary global address via two aligned dword loads (an
// aligned dword that overlaps valid bytes never leaves their page).  NT: L2
// served (the vector L1 is not coherent with the writer wave's stores).
// Address-space-1 pointers keep these global_load (vmcnt only), not flat_load
// (which also waits on lgkmcnt and so on every outstanding LDS access).
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

__device__ __forceinline__ uint32_t global_byte_nt(const uint8_t* p)
{
    const uintptr_t a = (uintptr_t)p;
    const uint32_t w = __builtin_nontemporal_load((gdword*)(a & ~(uintptr_t)3));
    return (w >> (8u * (uint32_t)(a & 3))) & 0xFFu;
}


// Diagnostic build only (STAMPS): per-phase s_memtime cycle sums (slots
// 0..CN_FIRST-1) and event counts (CN_*) go to stamps[b * kStampSlots + i];
// no output value depends on them.  scripts/diag_decode.py knows this order.
enum { PH_STAGE, PH_PASS1, PH_PWALK, PH_MERGE, PH_COUNT, PH_WRITE,
       PH_WLOAD, PH_WSCAN, PH_FARI, PH_FWD, PH_FARC, PH_BATCH,
       PH_SPACE, PH_FLAGS, PH_GATHER, PH_PUB,
       CN_FIRST, CN_WALKS = CN_FIRST, CN_WINDOWS, CN_FARWIN, CN_BATCHES, CN_STEPS,
       CN_IT_PASS1, CN_IT_PWALK, CN_IT_WALK, CN_IT_COUNT, CN_IT_WRITE, CN_FWD_ROUNDS, PH_N };
constexpr int kStampSlots = 32;
static_assert(PH_N <= kStampSlots, "stamp slots per block");

// Uniform walk of the true path from (pos, st) through lane i's segment
// [c0, c1) until it lands on one of lane i's final-generation marks (then
// lane i's speculative exit is the answer) or leaves the segment.
// SPEC: per-lane speculative walk that gives up (pos = kPosUnknown) where the
// exact slow decoder would be needed; the scalar scan then walks exactly.
template <bool SPEC>
__device__ __forceinline__ uint32_t walk_uniform(const FastLds& S, const Blk& k, uint32_t c0,
                                                 uint32_t c1, uint32_t gen, uint32_t xpos,
                                                 uint32_t xst, uint32_t& pos, uint32_t& st)
{
    uint32_t steps = 0;                      // (diagnostics)
    while (pos < c1) {
        steps++;
        if (pos >= k.z) {
            pos = kPosEnd;
            st = 0;
            return steps;
        }
        if (pos >= c0 && S.marks[pos - k.P] == ((st + 1) | (gen << 2))) {
            pos = xpos;
            st = xst;
            return steps;
        }
        bool slow = false;
        const Step r = decode_step<SPEC>(S, k, pos, st, &slow);
        if (SPEC && slow) {
            pos = kPosUnknown;
            st = 0;
            return steps;
        }
        if (r.bad || r.eof) {
            pos = kPosEnd;
            st = 0;
            return steps;
        }
        pos = r.pos;
        st = r.st;
    }
    return steps;
}

// ---------------------------------------------------------------------------
// Writer wave: copies final output from the LDS ring to HBM with 16-byte
// stores, keeping a few chunks in flight; publishes `flushed` once stores have
// landed.  It issues no loads, so its stores never hold up the decoder wave's
// loads (gfx9 vmcnt retires loads and stores in one in-order queue per wave).
// ---------------------------------------------------------------------------
__device__ void writer_wave(FastLds& S, uint8_t* out, uint32_t l)
{
    constexpr uint32_t kChunk = 16 * kWave;        // 1 KiB per store instruction
    uint32_t issued = 0;
    uint32_t pend[2] = {0, 0};                     // ends of chunks in flight, oldest first
    uint32_t npend = 0;
    for (uint32_t spin = 0; spin < (1u << 22); spin++) {
        const uint32_t state = lds_load(&S.state);
        const uint32_t prod = lds_load(&S.produced);
        if (state == 2)
            return;                                // refused: exact decoder redoes the block
        const uint32_t upto = state == 1 ? prod : (prod & ~15u);
        if (upto > issued && (upto - issued >= kChunk || state == 1)) {
            const uint32_t end = upto - issued > kChunk ? issued + kChunk : upto;
            const uint32_t x = issued + 16 * l;
            if (x + 16 <= end) {
                const uint32_t i = x & kRingMask;
                const uint4 v = *(const uint4*)&S.ring[i >> 2];
                *(uint4*)(out + x) = v;
            } else if (x < end) {
                for (uint32_t q = 0; x + q < end; q++)
                    out[x + q] = (uint8_t)ring_byte(S, x + q);
            }
            issued = end;
            if (npend == 2) {
                __builtin_amdgcn_s_waitcnt(0x0F71);        // vmcnt(1): oldest chunk landed
                lds_store(&S.flushed, pend[0]);
                pend[0] = pend[1];
                npend = 1;
            }
            pend[npend++] = end;
            continue;
        }
        if (npend) {                               // nothing new: drain and publish
            __builtin_amdgcn_s_waitcnt(0x0F70);            // vmcnt(0)
            lds_store(&S.flushed, issued);
            npend = 0;
            continue;
        }
        if (state == 1)
            return;
        // Poll rarely: the scalar unit is shared by every wave of the CU, and a
        // tight poll loop costs the decoder waves their SALU issue slots.  (The
        // ring's 3 KiB of headroom covers ~8K cycles of decoder output; waking
        // the writer with s_wakeup per ready chunk measured slower than
        // letting it drain several chunks per poll.)
        __builtin_amdgcn_s_sleep(POM_WRITER_SLEEP);
    }
}

// ---------------------------------------------------------------------------
// Far sources.  A match whose source may have left the ring by the time its
// step runs would read HBM byte by byte in every step it touches (61% of the
// steps of an ITB block).  Instead its whole source span is copied once per
// window into S.far -- one batched global round trip -- and the op becomes an
// LDS-linear source like a literal.  Called after forwarding, with the window
// ops' output offset o, length L, period dp and source b (in/out).
//
// Where the bytes are at this point (carry = output before this window): the
// last step of the previous window ended at most 255 bytes past carry, so the
// ring still holds every position >= carry + 255 - kRing, and its space check
// left flushed >= carry - kRing + kRingSlack, so every position below that is
// in HBM.  Sources lie below carry (db + span <= carry is required).
// ---------------------------------------------------------------------------
// Far ops are never forwarded (their sources lie below the window), so the
// copy is issued before forwarding -- which then hands far-buffer sources on
// to the ops that forward to them -- and only committed to LDS after it, so
// the loads' latency hides under the forwarding rounds.
struct FarCopy {
    uint32_t v[4];          // this lane's buffer dwords 4l .. 4l+3
    uint32_t used;          // buffer dwords filled (0: no far op in the window)
};

__device__ __forceinline__ FarCopy far_issue(FastLds& S, const Blk& k, uint32_t l,
                                             uint32_t nwin, uint32_t carry, uint32_t o,
                                             uint32_t L, uint32_t dp, uint32_t& db)
{
    FarCopy fc;
    fc.used = 0;
    const uint32_t span = dp ? dp : L;
    // some byte may read below the ring: sp + kRing < step_end + 4 with
    // step_end <= x + 259 and sp - db <= x - o (p == 0) or < p
    const bool far = l < nwin && !(db & kLitFlag) && db + span <= carry &&
                     db + kRing < o + (dp ? L : 0u) + 260u;
    if (!wave_ballot(far))
        return fc;
    const uint32_t nd = far ? ((db + span + 3u) >> 2) - (db >> 2) : 0u;
    const uint32_t cum = wave_incl_scan(nd);
    const bool acc = far && cum <= kFarDw;                  // the buffer takes a prefix of them
    const uint32_t acc_nd = acc ? nd : 0u;
    const uint64_t accm = wave_ballot(acc);
    const uint32_t used = accm ? lane_read(cum, 63u - (uint32_t)__builtin_clzll(accm)) : 0u;
    fc.used = used;
    if (!used)
        return fc;
    const uint32_t gl_end = carry + kRingSlack - kRing;     // below: in HBM (may wrap: none)
    const bool gl_any = carry + kRingSlack > kRing;
    // Buffer dword t -> its op, as in the gather steps: flag each op's first
    // buffer dword (S.flags, one byte per dword), scan the flag counts; the
    // k-th op's (source dword - buffer dword) sits in a table at k (the
    // window's op records are not written yet, so their space is free).
    uint32_t* const delta = (uint32_t*)S.wop;
    S.flags[l] = 0;
    wave_order();
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(accm >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)accm, 0u));
    if (acc_nd) {
        ((uint8_t*)S.flags)[cum - acc_nd] = 1;
        delta[rank] = (db >> 2) - (cum - acc_nd);
    }
    wave_order();
    const uint32_t f = S.flags[l];
    const uint32_t nst = (uint32_t)__builtin_popcount(f);
    const uint32_t jb = wave_incl_scan(nst) - nst - 1u;      // ops starting before 4l, minus 1
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) {
        const uint32_t t = l * 4 + i;                        // buffer dword
        const uint32_t j = (jb + (uint32_t)__builtin_popcount(f & ((2u << (8 * i)) - 1u))) & 63u;
        const uint32_t a = (t + delta[j]) * 4u;              // output byte offset, aligned
        const bool need = t < used;
        const bool hbm = need && gl_any && a + 4u <= gl_end;
        fc.v[i] = S.ring[(a & kRingMask) >> 2];
        if (hbm)
            fc.v[i] = __builtin_nontemporal_load((gdword*)(k.out + a));
    }
    if (acc_nd)
        db = kLitFlag | (kFarOff + 4u * (cum - acc_nd) + (db & 3u));
    return fc;
}

__device__ __forceinline__ void far_commit(FastLds& S, uint32_t l, const FarCopy& fc)
{
    if (!fc.used)
        return;
#pragma unroll
    for (uint32_t i = 0; i < 4; i++)
        if (l * 4 + i < fc.used)
            S.far[l * 4 + i] = fc.v[i];
}

// ---------------------------------------------------------------------------
template <bool STAMPS>
__global__ __launch_bounds__(2 * kWave, POM_WAVES_PER_EU) void lzo1x_decode_fast_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ src_len, uint8_t* __restrict__ dst,
    const uint64_t* __restrict__ dst_off, const uint32_t* __restrict__ dst_cap,
    uint32_t* __restrict__ out_len, int32_t* __restrict__ status,
    uint32_t* __restrict__ fallback, uint32_t nblocks, uint64_t* __restrict__ stamps)
{
    __shared__ FastLds S;
    const uint32_t b = blockIdx.x;
    if (b >= nblocks)
        return;
    const uint32_t l = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x == 0) {
        S.produced = 0;
        S.flushed = 0;
        S.state = 0;
    }
    if (threadIdx.x < kWave)
        S.flags[threadIdx.x] = 0;             // chunk tags start at 0x80000001
    __syncthreads();
    uint8_t* const out = dst + dst_off[b];
    if (wave == 1) {
        // The decoder refuses misaligned destinations before publishing anything.
        writer_wave(S, out, l);
        return;
    }

    uint64_t acc[PH_N] = {};
    uint64_t tmark = STAMPS ? __builtin_amdgcn_s_memtime() : 0;
#define STAMP(ph)                                                   \
    do {                                                            \
        if (STAMPS) {                                               \
            const uint64_t now_ = __builtin_amdgcn_s_memtime();     \
            acc[ph] += now_ - tmark;                                \
            tmark = now_;                                           \
        }                                                           \
    } while (0)

    Blk k;
    k.in = src + src_off[b];
    k.z = src_len[b];
    k.out = out;
    k.cap = dst_cap[b];
    k.P = 0;
    k.staged = 0;

    // The exact decoder takes: destinations not 16-byte aligned, empty or huge
    // blocks (lengths up to 255 * z must not wrap 32 bits).
    bool refuse = ((uintptr_t)k.out & 15) != 0 || k.z >= (1u << 24) || k.z == 0;
    uint32_t entry_pos = 0, entry_st = ST_F;   // true entry of the current piece
    uint32_t carry = 0;                        // output produced so far
    uint32_t flushed_seen = 0;                 // last `flushed` read
    uint32_t tag = 0;                          // step counter for the chunk tags
    bool done = false;                         // EOF consumed

    while (!refuse && !done) {
        // Skip pieces in which no instruction starts (inside a long literal run).
        if (entry_pos >= k.P + kPiece)
            k.P = entry_pos - (entry_pos % kPiece);
        if (k.P >= k.z) {                      // ran off the end without EOF
            refuse = true;
            break;
        }
        // ---- stage the piece's input --------------------------------------
        {
            const uint32_t avail = k.z - k.P;
            k.staged = avail < kStageBytes ? avail : kStageBytes;
            const uint8_t* base = k.in + k.P;
            for (uint32_t i = l * 4; i < kStageBytes; i += kWave * 4) {
                uint32_t w = 0;
                if (i + 4 <= k.staged)
                    w = global_dword<false>(base + i);
                else
                    for (uint32_t j = i; j < k.staged; j++)
                        w |= (uint32_t)base[j] << (8 * (j - i));
                S.stage[i >> 2] = w;
            }
            for (uint32_t i = l * 4; i < kPiece; i += kWave * 4)
                *(uint32_t*)&S.marks[i] = 0;
        }
        wave_order();
        STAMP(PH_STAGE);
        const uint32_t c0 = k.P + l * kSeg;            // this lane's segment
        const uint32_t c1 = c0 + kSeg;

        // ---- pass 1: speculative walk, mark visited points -------------------
        // A mark is (state + 1) | (gen << 2); gen counts this lane's restarts,
        // and only marks of the final generation lie on the path that really
        // reaches xpos (a restart breaks the chain).
        uint32_t xpos, xst, xgen = 0;
        uint32_t it_local = 0;                         // (diagnostics)
        if (c1 <= entry_pos) {                         // no instruction starts here
            xpos = entry_pos;
            xst = entry_st;
        } else {
            uint32_t pos = c0 >= k.P + kLook ? c0 - kLook : k.P;
            if (pos < entry_pos)
                pos = entry_pos;
            uint32_t st = pos == entry_pos ? entry_st : ST_A;
            uint32_t gen = 0;
            while (pos < c1 && pos < k.z) {
                if (STAMPS)
                    it_local++;
                if (pos >= c0)
                    S.marks[pos - k.P] = (uint8_t)((st + 1) | (gen << 2));
                bool slow = false;
                const Step r = decode_step<true>(S, k, pos, st, &slow);
                if (r.bad || r.eof) {                  // impossible guess: restart later
                    pos++;
                    st = ST_A;
                    gen = gen < 63 ? gen + 1 : 63;
                    continue;
                }
                pos = r.pos;
                st = r.st;
            }
            xpos = pos >= k.z ? kPosEnd : pos;
            xst = st;
            xgen = gen < 63 ? gen : 0xFFu;             // saturated: never merge
        }
        wave_order();
        STAMP(PH_PASS1);

        // ---- true entries: one parallel walk from the assumed entries, then a
        // scalar scan that reuses it and walks only where the guess was wrong.
        const uint32_t apos = shift_up1(xpos, entry_pos), ast = shift_up1(xst, entry_st);
        uint32_t fpos = apos, fst = ast;
        if (STAMPS)
            acc[CN_IT_PASS1] += wave_max_dbg(it_local);
        {
            const uint32_t ws = walk_uniform<true>(S, k, c0, c1, xgen, xpos, xst, fpos, fst);   // per lane (divergent)
            if (STAMPS)
                acc[CN_IT_PWALK] += wave_max_dbg(ws);
        }
        STAMP(PH_PWALK);
        // The scan visits only the lanes that need it.  Where lane i's true
        // entry E equals its assumed one, lanes i, i+1, ... stay right as long
        // as each walk landed on the next lane's assumed entry (f_l == x_l)
        // and none gave up, so the scan jumps to the first lane q where that
        // fails: mm (lane q-1's walk missed lane q's assumed entry) or uk
        // (lane q's own walk gave up), with E_q = f_{q-1}.
        uint32_t epos = apos, est = ast;
        {
            const uint64_t mm = wave_ballot(fpos != xpos || fst != xst) << 1;
            const uint64_t uk = wave_ballot(fpos == kPosUnknown);
            uint32_t E = entry_pos, Est = entry_st;
            uint32_t i = 0;
            while (i < (uint32_t)kWave) {
                if (E == lane_read(apos, i) && Est == lane_read(ast, i)) {
                    const uint64_t from_i = ~0ull << i;
                    const uint64_t cand = (mm & (from_i << 1)) | (uk & from_i);
                    if (!cand) {                       // right through lane 63
                        E = lane_read(fpos, kWave - 1);
                        Est = lane_read(fst, kWave - 1);
                        break;
                    }
                    const uint32_t q = (uint32_t)__builtin_ctzll(cand);
                    if (q > i) {
                        E = lane_read(fpos, q - 1);
                        Est = lane_read(fst, q - 1);
                        i = q;
                    }
                }
                // lane i on its own, from its true entry E
                if (l == i) {
                    epos = E;
                    est = Est;
                }
                const uint32_t ci1 = k.P + (i + 1) * kSeg;
                if (E < ci1) {                         // else: segment i has no true start
                    if (E == lane_read(apos, i) && Est == lane_read(ast, i) &&
                        lane_read(fpos, i) != kPosUnknown) {
                        E = lane_read(fpos, i);
                        Est = lane_read(fst, i);
                    } else {
                        const uint32_t ws = walk_uniform<false>(S, k, ci1 - kSeg, ci1, lane_read(xgen, i),
                                                                lane_read(xpos, i), lane_read(xst, i), E, Est);
                        if (STAMPS) {
                            acc[CN_WALKS] += 1;
                            acc[CN_IT_WALK] += ws;
                        }
                    }
                }
                i++;
            }
            fpos = E;                                  // (uniform: the piece's true exit)
            fst = Est;
        }
        const uint32_t next_pos = fpos, next_st = fst;
        STAMP(PH_MERGE);

        // ---- pass 3: count ops of the true path ------------------------------
        uint32_t nops = 0;
        bool lane_eof = false, lane_err = false;
        {
            uint32_t pos = epos, st = est;
            uint32_t itc = 0;
            while (pos < c1) {
                itc++;
                const Step r = decode_step(S, k, pos, st);
                if (r.bad) {
                    lane_err = true;
                    break;
                }
                if (r.eof) {                           // EOF carries no op
                    lane_eof = true;
                    break;
                }
                if (r.aL > kMaxOpLen || r.bL > kMaxOpLen) {
                    lane_err = true;
                    break;
                }
                nops += (r.aL ? 1u : 0u) + (r.bL ? 1u : 0u);
                pos = r.pos;
                st = r.st;
            }
            if (STAMPS)
                acc[CN_IT_COUNT] += wave_max_dbg(itc);
        }
        if (wave_ballot(lane_err)) {
            refuse = true;
            break;
        }
        const uint32_t incl = wave_incl_scan(nops);
        const uint32_t total_ops = lane_read(incl, kWave - 1);
        STAMP(PH_COUNT);
        if (total_ops > kOpMax) {
            refuse = true;
            break;
        }
        // ---- pass 4: write the ops --------------------------------------------
        {
            uint32_t w = incl - nops;
            uint32_t pos = epos, st = est;
            uint32_t itw = 0;
            while (pos < c1) {
                itw++;
                const Step r = decode_step(S, k, pos, st);
                if (r.eof)
                    break;
                // An op is stored as a reference to its instruction
                // (piece offset | state << 10 | part << 12, part 1 = trailing
                // literals; instructions start inside the 1-KiB piece) and is
                // re-decoded when its window executes: 2 bytes of LDS, not 8.
                const uint32_t ref = (pos - k.P) | (st << 10);
                if (r.aL)
                    S.opref[w++] = (uint16_t)ref;
                if (r.bL)
                    S.opref[w++] = (uint16_t)(ref | (1u << 12));
                pos = r.pos;
                st = r.st;
            }
            if (STAMPS)
                acc[CN_IT_WRITE] += wave_max_dbg(itw);
        }
        wave_order();
        STAMP(PH_WRITE);
        if (wave_ballot(lane_eof))
            done = true;
        else {
            entry_pos = next_pos;                      // next piece: the true exit
            entry_st = next_st;
            if (entry_pos == kPosEnd) {                // dead without EOF
                refuse = true;
                break;
            }
        }

        // ---- execute the piece's ops, 64 at a time ----------------------------
        for (uint32_t w0 = 0; w0 < total_ops && !refuse; w0 += kWave) {
            const uint32_t nwin = total_ops - w0 < (uint32_t)kWave ? total_ops - w0 : (uint32_t)kWave;
            uint32_t L = 0, Sv = 0;
            if (l < nwin) {
                const uint32_t ref = S.opref[w0 + l];
                const Step r = decode_step(S, k, k.P + (ref & 0x3FFu), (ref >> 10) & 3u);
                const bool part = (ref >> 12) != 0;
                L = part ? r.bL : r.aL;
                Sv = part ? r.bS : r.aS;
            }
            STAMP(PH_WLOAD);
            if (STAMPS)
                acc[CN_WINDOWS] += 1;
            const uint32_t inc = wave_incl_scan(L);
            const uint32_t o = carry + inc - L;
            const uint32_t wtotal = lane_read(inc, kWave - 1);
            if (carry + wtotal < carry || carry + wtotal > k.cap) {
                refuse = true;                         // OUTPUT_OVERRUN (or wrap)
                break;
            }
            const bool lit = (Sv & kLitFlag) != 0;
            const bool lb = l < nwin && !lit && Sv > o;     // LOOKBEHIND_OVERRUN
            if (wave_ballot(lb)) {
                refuse = true;
                break;
            }
            // ---- op descriptors: byte x of op j reads
            //   src[b + ((x - o) mod p)]   (p == 0: src[b + x - o])
            // in LDS at linear address b (kLitFlag set: the input staging or
            // the far buffer; past the staging, the input in HBM) or in the
            // output (ring / HBM).  A match starts as b = o - d, p = d if it
            // overlaps itself (d < L).
            uint32_t db = lit ? Sv + (kStageOff - k.P) : o - Sv;
            uint32_t dp = (!lit && Sv < L) ? Sv : 0u;
            // Source forwarding: a match whose source span lies inside one
            // earlier op of this window reads that op's source instead, so it
            // no longer waits for it.  Three parallel rounds reach the
            // sequential fixed point on ITB streams (600 -> 205 batches per
            // 64 KiB block).
            STAMP(PH_WSCAN);
            FarCopy fc;
            fc.used = 0;
            if (kFarDw)
                fc = far_issue(S, k, l, nwin, carry, o, L, dp, db);
            STAMP(PH_FARI);
            if (STAMPS && fc.used)
                acc[CN_FARWIN] += 1;
            const uint32_t o_first = lane_read(o, 0);
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
                bool ok = need && k2 < l && ko <= db && db + span <= ko + kL;
                uint32_t r = db - ko;
                if (ok && kp) {
                    r %= kp;
                    ok = r + span <= kp;
                }
                if (ok)
                    db = kb + r;                       // (kb carries k's input flag)
            }
            // end of each output-sourced op's source span: a batch may not read
            // its own output
            STAMP(PH_FWD);
            if (kFarDw)
                far_commit(S, l, fc);
            const bool outsrc = l < nwin && !(db & kLitFlag);
            const uint32_t span = dp ? dp : L;
            const uint32_t send = outsrc ? db + span : 0u;
            uint32_t inv = 0;                          // mod by mulhi; only overlapping matches
            if (wave_ballot(dp != 0))
                inv = dp ? 0xFFFFFFFFu / dp : 0u;
            // An op needs HBM reads if its literal source runs past the staging,
            // or its output source may leave the ring before its last step
            // (sp + kRing < step start + 260 for some byte; far ops the buffer
            // did not take).
            const uint32_t lin_end = kStageOff + k.staged;
            const bool gop = l < nwin && (outsrc ? db + kRing < o + (dp ? L : 0u) + 260u
                                                 : (db & ~kLitFlag) + span > lin_end);
            // Chunks: op j covers output chunks cs .. cs + ceil(L/4) - 1 of the
            // window, each up to 4 bytes of that op alone.
            const uint32_t nch = l < nwin ? (L + 3u) >> 2 : 0u;
            const uint32_t cinc = wave_incl_scan(nch);
            const uint32_t cs = cinc - nch;
            const uint32_t wchunks = lane_read(cinc, kWave - 1);
            S.wop[l] = make_uint4(o, db, cs, L | (gop ? kLitFlag : 0u));
            S.wper[l] = make_uint2(dp, inv);
            wave_order();
            STAMP(PH_FARC);
            uint32_t s = 0;
            while (s < nwin) {
                const uint32_t os = lane_read(o, s);
                const bool brk = l > s && outsrc && send > os;
                const uint64_t bm = wave_ballot(brk);
                const uint32_t e = bm ? (uint32_t)__builtin_ctzll(bm) : nwin;
                const uint32_t c_beg = lane_read(cs, s);
                const uint32_t c_end = e < nwin ? lane_read(cs, e) : wchunks;
                const bool gbatch = wave_ballot(l >= s && l < e && gop) != 0;
                const bool starter = l >= s && l < e;
                STAMP(PH_BATCH);
                if (STAMPS)
                    acc[CN_BATCHES] += 1;
                // ---- batch [s, e): chunks [c_beg, c_end), 64 per step --------
                uint32_t jcarry = s;                   // ops of the batch started before C
                for (uint32_t C = c_beg; C < c_end; C += kWave) {
                    // chunk -> op: each op starting in this step tags its first
                    // chunk's slot; lane l's op is the last one started at or
                    // before chunk C + l (a ballot and mbcnt, no scan).
                    tag++;
                    const uint32_t tagv = tag | 0x80000000u;   // far_issue's byte flags never set bit 31
                    if (starter && cs >= C && cs < C + kWave)
                        S.flags[cs - C] = tagv;
                    wave_order();
                    const bool st0 = S.flags[l] == tagv;
                    const uint64_t M = wave_ballot(st0);
                    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(M >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0u));
                    const uint32_t j = (jcarry + below + (st0 ? 0u : ~0u)) & 63u;
                    jcarry += (uint32_t)__builtin_popcountll(M);
                    const uint4 op = S.wop[j];
                    const uint2 pr = S.wper[j];
                    const uint32_t c = C + l;
                    const bool live = c < c_end;
                    const uint32_t k4 = (c - op.z) * 4u;
                    const uint32_t x = op.x + k4;
                    const uint32_t Lj = op.w & ~kLitFlag;
                    const uint32_t rem = Lj - k4;
                    const uint32_t len = live ? (rem < 4u ? rem : 4u) : 0u;
                    const uint32_t nl = c_end - C < (uint32_t)kWave ? c_end - C : (uint32_t)kWave;
                    const uint32_t xs = lane_read(x, 0);
                    const uint32_t step_end = lane_read(x + len, nl - 1);
                    STAMP(PH_FLAGS);
                    // ring space: the slots of [xs, step_end) must be flushed
                    // (and HBM reads below need flushed >= step_end - kRing + kRingSlack).
                    for (uint32_t spin = 0; step_end > flushed_seen + kRing - kRingSlack; spin++) {
                        if (spin > (1u << 22)) {       // writer stuck: let the exact path redo it
                            refuse = true;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                        flushed_seen = lds_load(&S.flushed);
                    }
                    if (refuse)
                        break;
                    STAMP(PH_SPACE);
                    if (STAMPS)
                        acc[CN_STEPS] += 1;
                    {
                        // source offsets r_i = (k4 + i) mod p (p == 0: k4 + i)
                        const uint32_t p = pr.x;
                        uint32_t r[4];
                        r[0] = k4 - p * (uint32_t)__umulhi(k4, pr.y);
                        r[0] = min(r[0], r[0] - p);
#pragma unroll
                        for (uint32_t i = 1; i < 4; i++)
                            r[i] = min(r[i - 1] + 1u, r[i - 1] + 1u - p);
                        const bool lin = (op.y & kLitFlag) != 0;
                        const uint32_t bb = live ? op.y & ~kLitFlag : 0u;
                        // (linear sources past the staging read HBM below; masking
                        // keeps their LDS read inside the allocation)
                        const uint32_t amask = !live ? 0u : lin ? kLdsMask : kRingMask;
                        const uint8_t* lds = (const uint8_t*)&S;
                        uint32_t val = 0;
#pragma unroll
                        for (uint32_t i = 0; i < 4; i++)
                            val |= (uint32_t)lds[(bb + r[i]) & amask] << (8 * i);
                        if (gbatch) {                          // literal past staging / far match
                            const bool gj = (op.w & kLitFlag) != 0;
                            uint32_t gmask = 0;
#pragma unroll
                            for (uint32_t i = 0; i < 4; i++) {
                                const uint32_t sp = bb + r[i];
                                const bool isg = gj && i < len && (lin ? sp >= lin_end : sp + kRing < xs + 260u);
                                gmask |= isg ? (1u << i) : 0u;
                            }
                            if (wave_ballot(gmask != 0)) {
                                const uint32_t lin_in = kStageOff - k.P;     // LDS address - input position
                                for (uint32_t i = 0; i < 4; i++) {
                                    if (!(gmask & (1u << i)))
                                        continue;
                                    const uint32_t sp = bb + r[i];
                                    const uint32_t bv = lin
                                        ? (uint32_t)*((__attribute__((address_space(1))) const uint8_t*)(k.in + (sp - lin_in)))
                                        : global_byte_nt(k.out + sp);
                                    val = (val & ~(0xFFu << (8 * i))) | (bv << (8 * i));
                                }
                            }
                        }
                        uint8_t* ldsw = (uint8_t*)&S;
#pragma unroll
                        for (uint32_t i = 0; i < 4; i++)
                            ldsw[i < len ? ((x + i) & kRingMask) : kSinkOff + i] = (uint8_t)(val >> (8 * i));
                    }
                    wave_order();
                    STAMP(PH_GATHER);
                    lds_store(&S.produced, step_end);  // bytes below are final: hand them over
                    STAMP(PH_PUB);
                }
                if (refuse)
                    break;
                s = e;
            }
            carry += wtotal;
            wave_order();
        }
        k.P += kPiece;
    }

    if (STAMPS && l == 0)
        for (int i = 0; i < PH_N; i++)
            stamps[(size_t)b * kStampSlots + i] = acc[i];
#undef STAMP
    if (l == 0) {
        if (refuse) {
            lds_store(&S.state, 2u);
            status[b] = kFallback;
            const uint32_t at = atomicAdd(&fallback[0], 1u);
            fallback[1 + at] = b;
        } else {
            lds_store(&S.produced, carry);
            lds_store(&S.state, 1u);
            out_len[b] = carry;
            status[b] = 0;
        }
    }
}

}  // namespace

extern "C" int lzo_mi355x_launch_decompress_fast(const uint8_t* src, const uint64_t* src_off,
                                                 const uint32_t* src_len, uint8_t* dst,
                                                 const uint64_t* dst_off, const uint32_t* dst_cap,
                                                 uint32_t* out_len, int32_t* status,
                                                 uint32_t* fallback, uint32_t nblocks,
                                                 hipStream_t stream)
{
    if (nblocks == 0)
        return 0;
    hipLaunchKernelGGL(lzo1x_decode_fast_kernel<false>, dim3(nblocks), dim3(2 * kWave), 0,
                       stream, src, src_off, src_len, dst, dst_off, dst_cap, out_len, status,
                       fallback, nblocks, nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Diagnostic: the same decoder with per-phase cycle stamps (kStampSlots x u64 per block).
extern "C" int lzo_mi355x_debug_decompress_fast_stamps(
    const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len, uint8_t* dst,
    const uint64_t* dst_off, const uint32_t* dst_cap, uint32_t* out_len, int32_t* status,
    uint32_t* fallback, uint32_t nblocks, uint64_t* stamps, hipStream_t stream)
{
    if (nblocks == 0)
        return 0;
    hipLaunchKernelGGL(lzo1x_decode_fast_kernel<true>, dim3(nblocks), dim3(2 * kWave), 0,
                       stream, src, src_off, src_len, dst, dst_off, dst_cap, out_len, status,
                       fallback, nblocks, stamps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
