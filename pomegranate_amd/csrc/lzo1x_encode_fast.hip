// lzo1x_encode_fast.hip -- the throughput LZO1X-1 encoder for MI355X (gfx950)
// for blocks of up to 16 MiB (ITB records are 12 KiB - 524 KiB).  Output is byte-identical to
// lib/minilzo.c:2922-3207 (lzo1x_1_compress) run with a zero-filled wrkmem;
// the parse is SURVEY.md Appendix A.1.  Larger blocks are left with status
// LZO_MI355X_ENC_PENDING for lzo1x_encode_kernel (lzo1x_kernels.hip).
//
// One workgroup per block, two waves:
//
//  * the PARSE wave walks the block 64 candidate positions at a time.  Every
//    lane probes its own position against the dictionary as it was before the
//    window (u16 positions in LDS, 0 = empty: the reference never stores
//    position 0).  A lane's probe is exact as long as no earlier lane of the
//    window that really probes writes a slot it reads.  Path lanes post
//    (window tag, lane) for the slot they write into a claim table with
//    ds_min, then read back the entries of the slots they read: an entry of
//    this window from a lower lane is such a write (or, rarely, another slot
//    hashing to the same entry), and the window is cut at the first lane that
//    finds one, so every lane before it is exact.  Within
//    the exact prefix the greedy parse proceeds as the reference does: the
//    first matching lane emits a match, the lanes it covers are skipped (they
//    neither probe nor update the dictionary), and the lane right after it
//    continues -- several matches per window.  Candidate bytes and a 28-byte
//    match compare come in one round trip per window; only matches of 28
//    bytes or more need a wave-parallel extension.  The parse wave only emits
//    tokens (literal run, match) into an LDS queue.
//
//  * the EMIT wave turns tokens into the LZO1X byte stream (lzo1x_emit.h) in
//    an LDS ring and stores it to HBM, off the parse wave's critical path.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdlib.h>
#include <stdint.h>

#include "lzo_mi355x_kernels.h"
#include "lzo1x_emit.h"

namespace {

constexpr int kWave = 64;
constexpr uint32_t kSlots = emit::kSlots;
// Dictionary entries are u16: v = position - base + 1 (0 = empty).  Before a
// window could store a value past 65535, the base moves up to a multiple of
// kRebase at least kM4MaxOffset + 1 below the window, and every entry is
// re-based: the ones below the new base are cleared -- their distance from
// every later probe exceeds M4_MAX_OFFSET, so the reference rejects them too
// (lib/minilzo.c:2878-2883) and the parse is unchanged.
constexpr uint32_t kRebase = 8192;
constexpr uint32_t kMaxN = 1u << 24;            // larger blocks: the general encoder
#ifndef POM_ENC_TOK
#define POM_ENC_TOK 64
#endif
#ifndef POM_ENC_CLAIM
#define POM_ENC_CLAIM 1024
#endif
#ifndef POM_ENC_STAGE
#define POM_ENC_STAGE 1024
#endif
constexpr uint32_t kTok = POM_ENC_TOK;          // token queue entries
constexpr uint32_t kClaim = POM_ENC_CLAIM;      // claim table entries (slots hashed)
constexpr uint32_t kStage = POM_ENC_STAGE;      // emitter output ring
constexpr uint32_t kM2MaxOffset = 0x800;        // lib/minilzo.c M2_MAX_OFFSET
constexpr uint32_t kM4MaxOffset = 0xBFFF;       // M4_MAX_OFFSET
constexpr uint32_t kFarPos = 0xC0000000u;        // a read position past every block (kMaxN)
#ifndef POM_EMIT_SLEEP
#define POM_EMIT_SLEEP 8
#endif
#ifndef POM_ENC_AHEAD
#define POM_ENC_AHEAD 2048                      // bytes the emit wave pulls into L2 ahead of the parse
#endif
#ifndef POM_ENC_AHEAD1
#define POM_ENC_AHEAD1 0                        // the one-wave kernel's own read-ahead (0: none)
#endif

// The dictionary lives in LDS (4 blocks per CU: it is 32 KiB) or, with
// scratch from the caller, in global memory: 32 KiB per resident workgroup,
// so 16 blocks per CU parse at once (4 parse waves per SIMD instead of one)
// at the price of a probe round trip through L2 instead of LDS.
#ifndef POM_ENC_RESIDENT
#define POM_ENC_RESIDENT 16                     // workgroups per CU with the global dictionary (2 waves each: the CU wave limit)
#endif
constexpr uint32_t kDictBytes = (kSlots + 2) * 2 + 60;   // per workgroup, 64-byte multiple
// Global dictionary: a bitmap in LDS (2 KiB per block) of the slots the block
// has written.  A probe of any other slot is EMPTY without a load (a buffer
// load out of range: no memory request), and the 32 KiB region needs no
// zeroing per block.  On C3's ITB blocks 27% of primary and 38% of secondary
// probes read unwritten slots, and a window's dictionary lines drop from 39
// to 15 (scripts/dbg/enc_empty_sim.c).
#ifndef POM_ENC_OCC
#define POM_ENC_OCC 1
#endif
#ifndef POM_ENC_OCC2
#define POM_ENC_OCC2 1                          // (with POM_ENC_OCC) the secondary slot only behind a written primary
#endif
static_assert(kDictBytes % 64 == 0, "dictionary regions stay 64-byte aligned");
// Scratch: [0, kScratchHead) the block ticket counter (u32, zeroed by the
// launcher when the grid is smaller than the batch), then one dictionary
// region per workgroup, then (batches of more blocks than resident
// workgroups) the start order, u32 per block.
constexpr uint32_t kScratchHead = 256;

template <bool GD>
struct __attribute__((aligned(16))) EncLdsT {
    // (the spare entry past the end of dict, claim and tok took the writes of
    // lanes with no part in them until round 5; those writes are exec-masked
    // now -- 50-odd lanes writing one LDS address serialised -- and the
    // entries stay only to keep the measured layout)
    uint16_t dict[GD ? 2 : kSlots + 2]; // last probe position per hash slot: position - base + 1 (0 = empty)
    uint32_t occ[GD && POM_ENC_OCC ? kSlots / 32 : 1];  // global dictionary: the slots this block wrote
    uint32_t claim[kClaim + 1];     // (window tag << 8 | lowest writing lane) per hashed slot
    uint4 tok[kTok + 1];            // {literal start, literal count, match length (0: tail), offset}
    uint8_t stage[kStage];          // emitter output ring
    uint32_t prod;                  // tokens published by the parse wave
    uint32_t cons;                  // tokens consumed by the emit wave
    uint32_t ip;                    // the parse wave's window start (a prefetch hint)
    uint32_t sink;                  // prefetched words end here
};
typedef EncLdsT<false> EncLds;
// four blocks (eight waves) per CU; with the global dictionary, twelve
static_assert(sizeof(EncLdsT<false>) * 4 <= 160 * 1024, "LDS budget");
static_assert(sizeof(EncLdsT<true>) * POM_ENC_RESIDENT <= 160 * 1024, "LDS budget");

// Dictionary access: S.dict (LDS) or the workgroup's region in global memory.
// Probes are agent-scope relaxed atomic loads (global_load_ushort sc1): served
// by L2, never by a stale vector-L1 line, so a probe sees this wave's earlier
// dictionary stores.  Non-temporal probes (round 2 until the last build) are as
// exact but mark the lines evict-first in L2: the 512 dictionaries of an XCD then
// miss L2 far more often, and the C3 compress kernel took 2.23 instead of 1.84 ms.
#ifndef POM_CAND_AUX
#define POM_CAND_AUX 0                          // cache policy of the candidate loads (buffer aux bits)
#endif
#ifndef POM_PW_AUX
#define POM_PW_AUX 0                            // cache policy of the probe-word loads
#endif
#ifndef POM_ENC_PRIO
#define POM_ENC_PRIO 1                          // one-wave kernel: wave priority by input bytes left
#endif
#ifndef POM_ENC_PRIO_STEP
#define POM_ENC_PRIO_STEP 8192
#endif
#ifndef POM_DICT_LOAD
#define POM_DICT_LOAD 2                         // probe loads: 0 non-temporal, 1 plain, 2 agent-scope atomic
#endif
typedef __attribute__((address_space(1))) uint16_t gu16;
template <bool GD>
struct Dict {
    uint16_t* lds;
    gu16* g;
    uint32_t* occ;                  // (POM_ENC_OCC) EncLdsT::occ
    __amdgpu_buffer_rsrc_t rs;      // (POM_ENC_OCC) the region g, kSlots u16
    __device__ __forceinline__ bool written(uint32_t slot) const
    {
        return (occ[slot >> 5] >> (slot & 31u)) & 1u;
    }
    // (POM_ENC_OCC) the slot's entry if rd, else 0 with no memory request (a
    // buffer load out of range); sc1: L1 bypassed, as the atomic loads below
    __device__ __forceinline__ uint32_t get_if(uint32_t slot, bool rd) const
    {
        return __builtin_amdgcn_raw_buffer_load_b16(rs, rd ? 2u * slot : 0x80000000u, 0, 16);
    }
    __device__ __forceinline__ uint32_t get(uint32_t slot) const
    {
        if (GD && POM_ENC_OCC)
            return get_if(slot, written(slot));
        if (GD) {
#if POM_DICT_LOAD == 1
            return g[slot];
#elif POM_DICT_LOAD == 2
            return __hip_atomic_load((uint16_t*)(g + slot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
            return __builtin_nontemporal_load(g + slot);
#endif
        }
        return lds[slot];
    }
    __device__ __forceinline__ void put(uint32_t slot, uint32_t v) const
    {
        if (GD && POM_ENC_OCC)
            __hip_atomic_fetch_or(occ + (slot >> 5), 1u << (slot & 31u), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
        if (GD)
            g[slot] = (uint16_t)v;
        else
            lds[slot] = (uint16_t)v;
    }
    // dwords 2i, 2i+1 of the table as one u32 (zeroing, re-basing)
    __device__ __forceinline__ uint32_t get2(uint32_t i) const
    {
        if (GD)
            return __hip_atomic_load((uint32_t*)g + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return ((uint32_t*)lds)[i];
    }
    __device__ __forceinline__ void put2(uint32_t i, uint32_t v) const
    {
        if (GD)
            ((__attribute__((address_space(1))) uint32_t*)g)[i] = v;
        else
            ((uint32_t*)lds)[i] = v;
    }
};

__device__ __forceinline__ uint32_t lane_id() { return emit::lane(); }
__device__ __forceinline__ uint32_t claim_index(uint32_t slot) { return (slot ^ (slot >> 9)) & (kClaim - 1); }

// Inclusive prefix sum over the wave: DPP row shifts inside each 16-lane row,
// then the row totals via readlane (no LDS round trip; lzo1x_decode_fast.hip
// scans the same way).
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);   // row_shr:8
    const uint32_t r0 = __builtin_amdgcn_readlane(v, 15), r1 = __builtin_amdgcn_readlane(v, 31),
                   r2 = __builtin_amdgcn_readlane(v, 47);
    const uint32_t row = lane_id() >> 4;
    v += (row >= 1 ? r0 : 0u) + (row >= 2 ? r1 : 0u) + (row >= 3 ? r2 : 0u);
    return v;
}
__device__ __forceinline__ uint32_t lane_read(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint64_t wave_ballot(bool p) { return __ballot(p); }
// Lane masks straight from a v_cmp (a ballot of a compound bool costs a
// v_cndmask and a v_cmp more): active lanes with a == b, a < b, a >= b.
__device__ __forceinline__ uint64_t mask_eq(uint32_t a, uint32_t b) { return __builtin_amdgcn_uicmp(a, b, 32); }
__device__ __forceinline__ uint64_t mask_lt(uint32_t a, uint32_t b) { return __builtin_amdgcn_uicmp(a, b, 36); }
__device__ __forceinline__ uint64_t mask_ge(uint32_t a, uint32_t b) { return __builtin_amdgcn_uicmp(a, b, 35); }
__device__ __forceinline__ void wave_order() { emit::order(); }

__device__ __forceinline__ uint32_t lds_load(const uint32_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store(uint32_t* p, uint32_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

typedef __attribute__((address_space(1))) const uint32_t gdword;

// The block as a raw buffer: the aligned dwords from the one holding byte 0
// through the one holding byte n-1.  Reads past it return 0 in hardware (the
// range check), so every probe, candidate and extension load is unconditional
// -- no exec branches, and the loads of one round trip share one wait.
struct BlockSrc {
    __amdgpu_buffer_rsrc_t rs;
    uint32_t sh0;                                   // in & 3
};

__device__ __forceinline__ BlockSrc block_src(const uint8_t* in, uint32_t n)
{
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)in);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)in >> 32));
    const uint32_t nn = __builtin_amdgcn_readfirstlane(n);
    const uintptr_t base = (((uintptr_t)hi << 32) | lo) & ~(uintptr_t)3;
    const uint32_t sh0 = lo & 3u;
    const uint32_t bytes = nn ? ((sh0 + nn - 1) & ~3u) + 4u : 0u;
    return {__builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)bytes, 0x00020000), sh0};
}

// NW little-endian dwords of the block starting at byte pos (any alignment).
// Aligned dwords lying wholly past the block's last byte read as 0: callers
// cap every comparison at the block end.
template <int NW, int AUX = 0>
__device__ __forceinline__ void load_at(const BlockSrc& B, uint32_t pos, uint32_t (&w)[NW])
{
    const uint32_t a = pos + B.sh0;
    const uint32_t a0 = a & ~3u;
    uint32_t r[NW + 1];
#pragma unroll
    for (int i = 0; i <= NW; i++)
        r[i] = __builtin_amdgcn_raw_buffer_load_b32(B.rs, a0 + 4 * i, 0, AUX);
#pragma unroll
    for (int i = 0; i < NW; i++)
        w[i] = __builtin_amdgcn_alignbyte(r[i + 1], r[i], a & 3u);
}

#ifndef POM_ENC_CMP
#define POM_ENC_CMP 7                            // dwords compared in the window round trip (A/B r05q: 6 / 7 / 8 / 10)
#endif
#ifndef POM_ENC_PATHMAX
#define POM_ENC_PATHMAX 6                        // matches the path walk takes per window
#endif
#ifndef POM_ENC_BATCH
#define POM_ENC_BATCH 1                          // the emit wave writes up to 64 tokens per pass
#endif
#ifndef POM_ENC_FWD
#define POM_ENC_FWD 8                            // claim conflicts resolved in place per window
#endif
constexpr int kCmpW = POM_ENC_CMP;
constexpr uint32_t kCmpB = 4 * kCmpW;            // match bytes known without an extension

// Bits [off, off + width) of a 64-bit mask, width < 64 (one s_bfm_b64:
// ((1 << width) - 1) << off; the compiler's form takes four instructions).
__device__ __forceinline__ uint64_t bit_range(uint32_t off, uint32_t width)
{
    uint64_t m;
    asm("s_bfm_b64 %0, %1, %2" : "=s"(m) : "s"(width), "s"(off));
    return m;
}

// Index of the first differing byte of two NW-dword strings (4 * NW: none).
// v_ffbl_b32 of 0 is 0xFFFFFFFF, which a saturating add of 32i keeps, so the
// minimum over the dwords of ffbl + 32i is the first differing bit: xor,
// ffbl, add and a min3 half of the time per dword, no compare or select.
template <int NW>
__device__ __forceinline__ uint32_t first_diff(const uint32_t (&a)[NW], const uint32_t (&b)[NW])
{
    uint32_t m = 32 * NW;                           // (bit index of the first difference)
#pragma unroll
    for (int i = 0; i < NW; i++) {
        uint32_t f;                                  // (asm: the compiler rebuilds selects from ctz)
        asm("v_ffbl_b32 %0, %1" : "=v"(f) : "v"(a[i] ^ b[i]));           // 0xFFFFFFFF: equal
        m = min(m, __builtin_elementwise_add_sat(f, 32u * i));          // (saturates: equal stays max)
    }
    return m >> 3;
}

// Match length from index k0 on (the first k0 bytes match), wave-parallel,
// 256 bytes per round trip, capped at the block end (lib/minilzo.c:3090-3102).
__device__ uint32_t extend_match(const BlockSrc& B, uint32_t n, uint32_t mc, uint32_t mp,
                                 uint32_t k0, uint32_t l)
{
    const uint32_t lim = n - mp;
    for (uint32_t k = k0;; k += 4 * kWave) {
        const uint32_t idx = k + 4 * l;
        uint32_t a[1], b[1];
        load_at<1>(B, mc + idx, a);
        load_at<1>(B, mp + idx, b);
        const uint32_t x = a[0] ^ b[0];
        uint32_t e = idx < lim && x ? idx + ((uint32_t)__builtin_ctz(x) >> 3) : 0xFFFFFFFFu;
        if (idx + 4 > lim)
            e = e < lim ? e : lim;
        const uint64_t mis = wave_ballot(e != 0xFFFFFFFFu);
        if (mis)
            return lane_read(e, (uint32_t)__builtin_ctzll(mis));
    }
}

// ---------------------------------------------------------------------------
// Emitter: tokens -> the LZO1X byte stream (lzo1x_emit.h) in an LDS ring,
// stored to HBM.  Run by the emit wave (two-wave kernels) or, in the fused
// kernel, by the parse wave itself after each window.
// ---------------------------------------------------------------------------
template <bool GD>
struct Emitter {
    EncLdsT<GD>& S;
    emit::Enc e;
    BlockSrc B;
    uint32_t n;
    uint32_t ct;                                     // tokens consumed
    uint32_t pos;                                    // input covered by the tokens so far
    bool poisoned;                                   // a token the parse cannot have meant
    bool prio;                                       // (one-wave kernel) wave priority by input left
    uint32_t* olen;                                  // out_len / status / block of drain(prod)
    int32_t* ost;
    uint32_t blk;

    __device__ __forceinline__ Emitter(EncLdsT<GD>& S_, const uint8_t* in, uint32_t n_, uint8_t* out,
                                       uint32_t cap)
        : S(S_), B(block_src(in, n_)), n(n_), ct(0), pos(0), poisoned(false), prio(false), olen(nullptr),
          ost(nullptr), blk(0)
    {
        e.in = in;
        e.n = n_;
        e.out = out;
        e.cap = cap;
        e.stage = S_.stage;
        e.smask = kStage - 1;
        e.sflush = kStage / 2;
        e.op = e.flushed = 0;
    }

    // Lane-parallel emission of the pending tokens, lane k writing token
    // ct + k: the byte offsets are a prefix sum of the token sizes, a short
    // literal run's length goes into the previous match's second-to-last
    // byte (lib/minilzo.c:3027-3030: lane k-1's, or the staged byte before
    // the batch), and the literal bytes of all lanes come in one load round
    // trip.  The batch ends before the first token that is the tail, has more
    // than kLitMax literals, needs extension zeros, fails the checks below,
    // or would overrun the ring; that token takes the one-at-a-time path.
    // Returns the number of tokens written.
    static constexpr uint32_t kLitMax = 16;
    __device__ uint32_t batch(uint32_t prod)
    {
        const uint32_t k = lane_id();
        const uint32_t avail = prod - ct < (uint32_t)kWave ? prod - ct : (uint32_t)kWave;
        const uint4 t = S.tok[(ct + (k < avail ? k : 0u)) % kTok];
        const uint32_t r = t.y, L = t.z, d = t.w;
        const uint32_t hdr = r >= 4 ? 1u : 0u;             // r <= kLitMax: one byte r - 3
        const bool m2 = L <= 8 && d <= 0x800;
        const bool near = d <= 0x4000;
        const uint32_t lim = near ? 33u : 9u;               // longest length of the short form
        const bool shortlen = L <= 8 || L <= lim;
        const uint32_t msz = m2 ? 2u : shortlen ? 3u : 4u;
        const uint32_t sz = hdr + r + msz;
        const uint32_t adv = r + L;
        const uint32_t iadv = wave_incl_sum(adv);
        const uint32_t isz = wave_incl_sum(sz);
        const uint32_t pk = pos + iadv - adv;              // input position of token k
        const uint32_t budget = e.smask + 1 - (e.op - e.flushed) - 4 - kLitMax;   // (- kLitMax: see the literals)
        // (every test evaluated: no short-circuit exec-mask cascade)
        const bool fits = (k < avail) & (L != 0) & (r <= kLitMax) & (shortlen | (L - lim <= 255)) &
                          (t.x == pk) & (r <= n - pk) & (L <= n - pk - r) & (d != 0) & (d <= pk + r) &
                          (d <= kM4MaxOffset) & (isz <= budget);
        const uint64_t bad = wave_ballot(!fits);
        const uint32_t nb = bad ? (uint32_t)__builtin_ctzll(bad) : (uint32_t)kWave;
        if (nb == 0)
            return 0;
        const bool act = k < nb;
        const uint32_t m = e.smask;
        uint8_t* const st = e.stage;
        const uint32_t o = e.op + isz - sz;                // token k's first byte
        const uint32_t rn = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((k + 1) & 63u) << 2), (int)r);
        const uint32_t pbits = k + 1 < nb && rn <= 3 ? rn : 0u;
        if (k == 0 && r >= 1 && r <= 3)
            st[(e.op - 2) & m] |= (uint8_t)r;
        wave_order();
        uint32_t lw[kLitMax / 4];
        {
            const uint32_t a = (act && r ? t.x : kFarPos) + B.sh0;
            uint32_t raw[kLitMax / 4 + 1];
#pragma unroll
            for (uint32_t i = 0; i <= kLitMax / 4; i++)
                raw[i] = __builtin_amdgcn_raw_buffer_load_b32(B.rs, (a & ~3u) + 4 * i, 0, 0);
#pragma unroll
            for (uint32_t i = 0; i < kLitMax / 4; i++)
                lw[i] = __builtin_amdgcn_alignbyte(raw[i + 1], raw[i], a & 3u);
        }
        const uint32_t ol = o + hdr;
        // Literals: kLitMax bytes per lane whatever the run's length, highest
        // first, so no write is exec-masked per byte.  A byte past a lane's run
        // belongs to a later token: its owner writes it later in this loop (a
        // smaller index), or the headers and match bytes below do; the last
        // lane's extra bytes land in the ring's free space (the budget keeps
        // kLitMax spare).
        if (act) {
#pragma unroll
            for (int i = (int)kLitMax - 1; i >= 0; i--)
                st[(ol + i) & m] = (uint8_t)(lw[i >> 2] >> (8 * (i & 3)));
        }
        wave_order();
        if (act && hdr)
            st[o & m] = (uint8_t)(r - 3);
        // the match (lib/minilzo.c:3064-3145), the next run's length ORed in
        const uint32_t oo = near ? d - 1 : d - 0x4000;
        const uint32_t dlo = (oo & 63) << 2, dhi = oo >> 6;
        const uint32_t tagb = near ? 0x20u : 0x10u | ((oo & 0x4000) >> 11);
        uint32_t b0, b1, b2 = 0, b3 = 0;
        if (m2) {
            b0 = ((L - 1) << 5) | ((oo & 7) << 2);
            b1 = oo >> 3;
        } else if (shortlen) {
            b0 = tagb | (L - 2);
            b1 = dlo;
            b2 = dhi;
        } else {
            b0 = tagb;
            b1 = L - lim;                                  // ext(L - lim), no zero bytes
            b2 = dlo;
            b3 = dhi;
        }
        b0 |= msz == 2 ? pbits : 0u;
        b1 |= msz == 3 ? pbits : 0u;
        b2 |= msz == 4 ? pbits : 0u;
        const uint32_t om = ol + r;
        if (act) {
            st[om & m] = (uint8_t)b0;
            st[(om + 1) & m] = (uint8_t)b1;
        }
        if (act && msz >= 3)
            st[(om + 2) & m] = (uint8_t)b2;
        if (act && msz == 4)
            st[(om + 3) & m] = (uint8_t)b3;
        wave_order();
        e.op += lane_read(isz, nb - 1);
        pos += lane_read(iadv, nb - 1);
        emit::maybe_flush(e);
        return nb;
    }

    // Emits the tokens up to prod.  Returns true once the tail token (the
    // block's last) is written, with out_len[b] and status[b] set.
    __device__ bool drain(uint32_t prod, uint32_t* out_len, int32_t* status, uint32_t b)
    {
        while (ct < prod) {
#ifndef POM_ENC_NOEMIT
            if (POM_ENC_BATCH && !poisoned) {
                const uint32_t nb = batch(prod);
                if (nb) {
                    ct += nb;
                    lds_store(&S.cons, ct);
                    continue;
                }
            }
#endif
            const uint4 t = S.tok[ct % kTok];
            ct++;
            // Every token must continue where the last one ended and stay in
            // the block, a match must look back into it: otherwise nothing is
            // emitted (no read past the input), the queue is still drained so
            // the parse wave never blocks, and the block reports LZO_E_ERROR.
            poisoned = poisoned || t.x != pos || t.y > n - pos ||
                       (t.z != 0 && (t.z > n - pos - t.y || t.w == 0 || t.w > pos + t.y ||
                                     t.w > kM4MaxOffset));
            if (t.z == 0) {                          // tail literals + EOF: the block is done
                if (!poisoned && t.y == n - pos)
                    emit::tail_and_eof(e, t.x);
                if (lane_id() == 0) {
                    out_len[b] = e.op;
                    status[b] = poisoned || t.y != n - pos ? -1          // LZO_E_ERROR
                              : e.op <= e.cap ? 0 : -5;  // LZO_E_OK / LZO_E_OUTPUT_OVERRUN
                }
                return true;
            }
#ifdef POM_ENC_NOEMIT
            if (POM_ENC_NOEMIT) {                    // (timing experiment only: no output)
                pos += t.y + t.z;
                lds_store(&S.cons, ct);
                continue;
            }
#endif
            if (!poisoned) {
                if (t.y) {
                    emit::lit_header(e, t.y);
                    emit::lits(e, t.x, t.y);
                }
                emit::match(e, t.z, t.w);
                emit::maybe_flush(e);
                pos += t.y + t.z;
            }
            lds_store(&S.cons, ct);
        }
        return false;
    }
    __device__ bool drain(uint32_t prod) { return drain(prod, olen, ost, blk); }
};

// ---------------------------------------------------------------------------
// Parse wave
// ---------------------------------------------------------------------------
// Diagnostic build only (STAMPS): per-phase s_memtime cycle sums and counts of
// the parse wave go to stamps[b * kEncStampSlots + i]; no output depends on them.
enum { EP_SETUP, EP_PROBE, EP_CAND, EP_PATH, EP_CLAIM, EP_TOK, EP_DICT, EP_PUSHWAIT,
       EC_WINDOWS, EC_EXTEND, EC_TOKENS, EC_PATHIT, EC_EXTIT, EC_C2NEED, EC_C2MATCH, EC_FWD, EP_N };
constexpr int kEncStampSlots = 16;

// FUSED (one-wave kernel): the parse wave runs the emitter E itself -- it
// drains the token queue once POM_ENC_DRAIN tokens are pending (larger emit
// batches than an eager emit wave gets) or the queue has no room, and at the
// end.
#ifndef POM_ENC_DRAIN
#define POM_ENC_DRAIN 48
#endif
template <bool STAMPS, bool GD, bool FUSED = false>
__device__ void parse_wave(EncLdsT<GD>& S, const Dict<GD> D, const uint8_t* in, uint32_t n, uint32_t l,
                           uint64_t* acc, Emitter<GD>* E = nullptr)
{
    uint64_t tmark = STAMPS ? __builtin_amdgcn_s_memtime() : 0;
#define ESTAMP(ph)                                                  \
    do {                                                            \
        if (STAMPS) {                                               \
            const uint64_t now_ = __builtin_amdgcn_s_memtime();     \
            acc[ph] += now_ - tmark;                                \
            tmark = now_;                                           \
        }                                                           \
    } while (0)
    uint32_t tp = 0;                                // tokens produced
    uint32_t cons_seen = 0;
    // (FUSED, POM_ENC_AHEAD1) lines up to that many bytes past the window go
    // to L2, one dword per 128-B line.  Off by default: a wave's loads retire
    // in order, so the window after such a load waits for its miss, and the
    // distance (0 / 2 / 4 KiB) moved C3 by under 1%.
    const uintptr_t pf_lines = (uintptr_t)in & ~(uintptr_t)127;
    const uintptr_t pf_last = ((uintptr_t)in + n - 1) & ~(uintptr_t)3;
    uint32_t pf = 0, pf_acc = 0, pf_new = 0;
    auto prefetch = [&](uint32_t at) {
        pf_acc ^= pf_new;
        pf_new = 0;
        const uint32_t ahead = at + POM_ENC_AHEAD1;
        const uint32_t want = ahead < n + 127 ? ahead : n + 127;
        for (; pf < want; pf += 128 * kWave) {
            const uintptr_t a = pf_lines + pf + 128 * l;
            if (a <= pf_last)
                pf_new ^= *(gdword*)a;
        }
    };
    auto push = [&](uint32_t from, uint32_t nlit, uint32_t mlen, uint32_t off) {
        if (STAMPS)
            acc[EC_TOKENS] += 1;
        ESTAMP(EP_TOK);
        if (FUSED) {
            if (tp - E->ct >= kTok)
                E->drain(tp);
        } else {
            while (tp - cons_seen >= kTok) {         // the emit wave always drains
                __builtin_amdgcn_s_sleep(2);
                cons_seen = lds_load(&S.cons);
            }
        }
        ESTAMP(EP_PUSHWAIT);
        if (l == 0)
            S.tok[tp % kTok] = make_uint4(from, nlit, mlen, off);
        tp++;
        lds_store(&S.prod, tp);
    };

    const BlockSrc B = block_src(in, n);
    uint32_t ii = 0;                                // first byte not yet emitted
    if (n > 13) {                                   // lib/minilzo.c:3167-3173
        if (GD && POM_ENC_OCC) {
            for (uint32_t s = l; s < kSlots / 32; s += kWave)
                S.occ[s] = 0;                       // zero-filled wrkmem: all EMPTY
        } else {
            for (uint32_t s = l; s < kSlots / 2; s += kWave)
                D.put2(s, 0);                       // zero-filled wrkmem: all EMPTY
        }
        for (uint32_t s = l; s < kClaim; s += kWave)
            S.claim[s] = 0xFFFFFFFFu;               // (tag 0xFFFFFF: no window has it)
        if (GD && !POM_ENC_OCC)
            __builtin_amdgcn_s_waitcnt(0x0F70);     // vmcnt(0): the table is zero in L2
        wave_order();
        const uint32_t ip_end = n - 13;             // lib/minilzo.c:2929
        uint32_t ip = 4;
        uint32_t base = 0;                          // dictionary position base
        uint32_t wtag = 0xFFFFFEu;                  // claim tag of the window (one per window, > 0)
        // (FUSED priority) next ip at which it steps down; never without priority
        uint32_t prio_ip = FUSED && E->prio ? 0u : 0xFFFFFFFFu;
        // Probe words of the window (position ip + l): the next window's are
        // read as soon as its start is known, ahead of the token and
        // dictionary writes.
        uint32_t pw[kCmpW];
        load_at<kCmpW>(B, ip + l, pw);
        ESTAMP(EP_SETUP);
        for (;;) {
            if (STAMPS)
                acc[EC_WINDOWS] += 1;
#if POM_ENC_PRIO
            // (one-wave kernel, one block per workgroup) blocks that are behind
            // (more input left) get the issue slots first, so the workgroups of
            // a CU finish together.  The priority steps down at most three
            // times a block: it is set again only once ip passes prio_ip.
            if (FUSED && ip >= prio_ip) {
                const uint32_t left = n - ip, st = POM_ENC_PRIO_STEP;
                const uint32_t q = __builtin_amdgcn_readfirstlane(left >= 3u * st ? 3u : left >= 2u * st ? 2u
                                                                  : left >= st ? 1u : 0u);
                switch (q) {
                case 3: __builtin_amdgcn_s_setprio(3); break;
                case 2: __builtin_amdgcn_s_setprio(2); break;
                case 1: __builtin_amdgcn_s_setprio(1); break;
                default: __builtin_amdgcn_s_setprio(0); break;
                }
                prio_ip = q ? n - q * st + 1 : 0xFFFFFFFFu;     // left < q * st from there on
            }
#endif
            if (ip + kWave - base >= 0xFFFFu) {     // this window's positions would not fit
                const uint32_t nb = (ip - (kM4MaxOffset + 1)) / kRebase * kRebase;
                const uint32_t delta = nb - base;
                for (uint32_t s2 = l; s2 < kSlots / 2; s2 += kWave) {
                    const uint32_t pr = D.get2(s2);
                    const uint32_t lo = pr & 0xFFFFu, hi = pr >> 16;
                    const uint32_t nlo = lo > delta ? lo - delta : 0u;
                    const uint32_t nhi = hi > delta ? hi - delta : 0u;
                    D.put2(s2, nlo | (nhi << 16));
                }
                if (GD)
                    __builtin_amdgcn_s_waitcnt(0x0F70);
                wave_order();
                base = nb;
            }
            if (FUSED && POM_ENC_AHEAD1)
                prefetch(ip);
            else if (!FUSED && POM_ENC_AHEAD)
                S.ip = ip;
            const uint32_t p = ip + l;
            const bool active = l == 0 || p < ip_end;   // the first probe always runs
            // (every lane probes; an inactive one ends with no candidate)
            const uint32_t h1 = emit::slot_primary(pw[0] & 0xFF, (pw[0] >> 8) & 0xFF,
                                                   (pw[0] >> 16) & 0xFF, pw[0] >> 24);
            const uint32_t h2 = emit::slot_secondary(h1);
            uint32_t e1, e2;
            if (GD && POM_ENC_OCC) {
                // (no load for a slot never written, for an inactive lane, or
                // for the secondary slot of an empty primary: v1 is false then)
                const bool r1 = active && D.written(h1);
                e1 = D.get_if(h1, r1);
                e2 = D.get_if(h2, POM_ENC_OCC2 ? r1 && D.written(h2) : D.written(h2));
            } else {
                e1 = D.get(h1);
                e2 = D.get(h2);
            }
            const uint32_t w1 = active && e1 ? base + e1 - 1 : 0u;   // (positions >= 4: 0 stays "empty")
            const uint32_t w2 = active && e2 ? base + e2 - 1 : 0u;
            const uint64_t am = mask_lt(p, ip_end) | 1ull;      // (active)
            const uint32_t nact = (uint32_t)__builtin_popcountll(am);
            if (STAMPS)
                __builtin_amdgcn_s_waitcnt(0);       // (attribute the probe loads here)
            ESTAMP(EP_PROBE);

            // Probe decision of every active lane with the pre-window
            // dictionary, lib/minilzo.c:2940-2971 (exact up to the cut below).
            const bool v1 = active && w1 != 0 && p - w1 <= kM4MaxOffset;
            const bool v2 = v1 && w2 != 0 && p - w2 <= kM4MaxOffset;
            uint32_t c1w[kCmpW], c2w[kCmpW];        // (read unconditionally; used only if valid)
            // (lanes without a valid candidate read past the block: range
            // checked, no memory request; the secondary candidate is only
            // ever compared when the primary one is more than M2_MAX_OFFSET
            // back, lib/minilzo.c:2946-2949)
            load_at<kCmpW, POM_CAND_AUX>(B, v1 ? w1 : kFarPos, c1w);
            load_at<kCmpW, POM_CAND_AUX>(B, v2 && p - w1 > kM2MaxOffset ? w2 : kFarPos, c2w);
            const uint32_t b3 = pw[0] >> 24;
            // (selects, no branches)
            const bool c1pass = v1 && (p - w1 <= kM2MaxOffset || (c1w[0] >> 24) == b3);
            const bool use2 = v1 && !c1pass;         // the secondary slot is read and written
            const bool c2pass = use2 && v2 && (p - w2 <= kM2MaxOffset || (c2w[0] >> 24) == b3);
            const bool tm = c1pass || c2pass;
            uint32_t slot = use2 ? h2 : h1, cand = c2pass ? w2 : w1;
            uint32_t cw[kCmpW];
#pragma unroll
            for (int i = 0; i < kCmpW; i++)
                cw[i] = c2pass ? c2w[i] : c1w[i];
            // try_match (:2962-2971), then the match length as far as kCmpB bytes
            const bool ok = tm && ((cw[0] ^ pw[0]) & 0xFFFFFFu) == 0;
            uint32_t mlen = first_diff<kCmpW>(cw, pw);
            mlen = mlen < n - p ? mlen : n - p;

            // ---- the greedy path through the window, speculatively ----------
            // From lane 0: a matching lane jumps over its match, any other
            // lane is a literal.  Lanes inside matches neither probe nor
            // update the dictionary (:3051-3150).
            uint64_t okm = wave_ballot(ok);
            if (STAMPS) {
                __builtin_amdgcn_s_waitcnt(0);       // (attribute the candidate loads here)
                acc[EC_C2NEED] += 0;
                acc[EC_C2MATCH] += 0;
            }
            ESTAMP(EP_CAND);
            uint64_t path = 0, mstart = 0;
            uint32_t end = 0;                        // lane where the path leaves the window
            uint32_t nmatch = 0;
            // The path through the window from lane `from` on (lanes below it
            // stay as they are): from `end`, the next match lane q -- the
            // literal lanes end .. q-1 before it -- then on from q + its
            // length.  rem: the ok lanes at or after `end` (empty once the path
            // leaves the window: ok lanes are active ones).
            auto walk = [&](uint32_t from) {
                end = from;
                uint64_t rem = okm & (~0ull << from);            // (from < 64)
                uint32_t nm = nmatch;
#pragma unroll
                for (int it = 0; it < POM_ENC_PATHMAX; it++) {
                    if (nm >= POM_ENC_PATHMAX)
                        break;
                    if (!rem) {
                        if (end < nact) {            // literal lanes to the last active one
                            path |= nact - end >= 64 ? ~0ull : bit_range(end, nact - end);
                            end = nact;
                        }
                        break;
                    }
                    if (STAMPS)
                        acc[EC_PATHIT] += 1;
                    const uint32_t q = (uint32_t)__builtin_ctzll(rem);
                    path |= bit_range(end, q - end) | (1ull << q);        // (q - end < 64)
                    mstart |= 1ull << q;
                    uint32_t len = lane_read(mlen, q);
                    if (len == kCmpB && n - (ip + q) > kCmpB) {
                        if (STAMPS)
                            acc[EC_EXTEND] += 1;
                        len = extend_match(B, n, lane_read(cand, q), ip + q, kCmpB, l);
                        if (STAMPS)
                            acc[EC_EXTIT] += (len - kCmpB) / (4 * kWave) + 1;
                        mlen = l == q ? len : mlen;
                    }
                    end = q + len;
                    nm++;                            // (the window ends after the last one)
                    const uint32_t e = end < 64u ? end : 64u;   // (past the window: a width-0 mask)
                    rem &= bit_range(e, 64u - e);
                }
                nmatch = nm;
            };
            walk(0);
            // The next window's probe words.  One-wave kernel: issued from this
            // first walk's end (again below only if forwarding moves the end),
            // ahead of the claims (C3 compress -1%).  The lone-block kernels
            // issue them after the claims: there an early load holds up the
            // re-walks' extension loads behind it (lone 64 KiB 655 -> 675 us).
            uint32_t npw[kCmpW];
            const uint32_t end0 = end;
            if (FUSED)
                load_at<kCmpW, POM_PW_AUX>(B, ip + end0 + l, npw);
            ESTAMP(EP_PATH);
            // ---- exactness: claims among the path lanes, and forwarding ------
            // Path lane l read h1 (and h2 when use2) and writes slot.  The
            // table keeps, per hashed slot, the lowest lane of this window
            // writing it (ds_min of tag|lane; a wave's LDS operations complete
            // in order, so the reads below see every post).  A path lane is
            // inexact only if a lower path lane writes a slot it read.  Such a
            // lane c, lowest first, is decided again: its entry is the position
            // of the last lower path lane j writing that slot -- less than 64
            // back, so the candidate passes the M2_MAX_OFFSET test -- and j's
            // probe words are the candidate's bytes.  The path is walked again
            // from c and the claims re-posted under a new tag.  After
            // POM_ENC_FWD rounds the window ends at the next conflicting lane.
            uint64_t resolved = 0, superseded = 0;   // (superseded: a later lane writes its slot)
            uint64_t um2 = wave_ballot(use2);        // lanes that read the secondary slot
            for (uint32_t round = 0;; round++) {
                const bool onpath = (path >> l) & 1ull;
                const uint32_t mine = (wtag << 8) | l;
                // (off-path lanes post nothing: sent to one spare entry, their
                // atomics serialised on it -- lone 64 KiB 655 -> 640 us)
                if (onpath)
                    atomicMin(&S.claim[claim_index(slot)], mine);
                wave_order();
                const uint32_t t1 = S.claim[claim_index(h1)];
                const uint32_t t2 = S.claim[claim_index(h2)];
                // path lanes not yet resolved that read a slot a lower lane of
                // this window writes (h1, or h2 when use2)
                const uint64_t cf1 = mask_eq(t1 >> 8, wtag) & mask_lt(t1 & 0xFFu, l);
                const uint64_t cf2 = um2 & mask_eq(t2 >> 8, wtag) & mask_lt(t2 & 0xFFu, l);
                uint64_t cm = path & ~resolved & (cf1 | cf2);
                wtag--;
                if (!cm)
                    break;
                if (round >= POM_ENC_FWD) {
                    end = (uint32_t)__builtin_ctzll(cm);   // the window ends at a path lane
                    break;
                }
                const uint32_t c = (uint32_t)__builtin_ctzll(cm);   // never lane 0
                if (STAMPS)
                    acc[EC_FWD] += 1;
                resolved |= 1ull << c;
                const uint64_t below_c = (1ull << c) - 1;
                const uint64_t pm = path & below_c;      // exact path lanes below c
                const uint32_t h1c = lane_read(h1, c), h2c = lane_read(h2, c);
                const bool u2c = ((um2 >> c) & 1ull) != 0;
                const uint64_t wm1 = wave_ballot(slot == h1c) & pm;
                const uint64_t wm2 = wave_ballot(slot == h2c) & pm & (u2c ? ~0ull : 0ull);
                if (!wm1 && !wm2)                        // a claim-table alias: c was exact
                    continue;                            // (claims again)
                const bool via2 = wm1 == 0;              // h1 unchanged, its test failed again: h2
                const uint32_t j = 63u - (uint32_t)__builtin_clzll(via2 ? wm2 : wm1);
                superseded |= 1ull << j;                 // c writes j's slot after j
                uint32_t pj[kCmpW];
#pragma unroll
                for (int i = 0; i < kCmpW; i++)
                    pj[i] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(j << 2), (int)pw[i]);
                uint32_t mc = first_diff<kCmpW>(pj, pw);
                mc = mc < n - p ? mc : n - p;
                const bool isc = l == c;
                const uint64_t bitc = 1ull << c;
                // (lane c's new decision goes into the lane masks; ok and use2
                // themselves are not read again)
                const uint64_t nokm = __builtin_amdgcn_uicmp((pj[0] ^ pw[0]) & 0xFFFFFFu, 0u, 32);
                okm = (okm & ~bitc) | (nokm & bitc);
                um2 = via2 ? um2 | bitc : um2 & ~bitc;
                mlen = isc ? mc : mlen;
                cand = isc ? ip + j : cand;
                slot = isc ? (via2 ? h2 : h1) : slot;
                path &= below_c;
                mstart &= below_c;
                nmatch = (uint32_t)__builtin_popcountll(mstart);
                walk(c);
            }
            if (STAMPS) {                            // (why the window ended)
                acc[EC_C2NEED] += end > 64 ? 1 : 0;  // a match crossing its last lane
                acc[EC_C2MATCH] += nmatch >= POM_ENC_PATHMAX ? 1 : 0;   // the path cap
            }
            const uint64_t keep = end >= 64 ? ~0ull : ((1ull << end) - 1);
            if (!FUSED || end != end0)
                load_at<kCmpW, POM_PW_AUX>(B, ip + end + l, npw);

            ESTAMP(EP_CLAIM);
            // ---- tokens for the matches before the cut ------------------------
            // Each match lane writes its own token: its literal run starts
            // after the highest lane below it that is not a literal path lane
            // (the last byte of the previous match), or at ii.  The parse
            // stops after the first match reaching ip_end (:3151-3152).
            uint64_t km = mstart & keep;
            const uint64_t dm = km & mask_ge(p + mlen, ip_end);   // (ism && p + mlen >= ip_end)
            const bool done = dm != 0;
            if (done) {
                const uint32_t d = (uint32_t)__builtin_ctzll(dm);
                km &= d >= 63 ? ~0ull : ((2ull << d) - 1);
            }
            if (km) {
                const uint32_t cnt = (uint32_t)__builtin_popcountll(km);
                if (STAMPS)
                    acc[EC_TOKENS] += cnt;
                ESTAMP(EP_TOK);
                if (FUSED) {
                    if (tp + cnt - E->ct > kTok)
                        E->drain(tp);
                } else {
                    while (tp + cnt - cons_seen > kTok) {    // the emit wave always drains
                        __builtin_amdgcn_s_sleep(2);
                        cons_seen = lds_load(&S.cons);
                    }
                }
                ESTAMP(EP_PUSHWAIT);
                const uint64_t below = (1ull << l) - 1;
                const uint64_t stop = ~(path & ~mstart) & below;
                const uint32_t from = stop ? ip + 64 - (uint32_t)__builtin_clzll(stop) : ii;
                const uint32_t r = (uint32_t)__builtin_popcountll(km & below);
                // (the other lanes write nothing: sent to a spare entry, their
                // writes to one address were serialised -- lone 64 KiB 641 -> 629
                // us, with the dictionary put below)
                if ((km >> l) & 1ull)
                    S.tok[(tp + r) % kTok] = make_uint4(from, p - from, mlen, p - cand);
                tp += cnt;
                lds_store(&S.prod, tp);
                const uint32_t last = 63 - (uint32_t)__builtin_clzll(km);
                ii = ip + last + lane_read(mlen, last);
                if (FUSED && tp - E->ct >= POM_ENC_DRAIN)
                    E->drain(tp);
            }
            // UPDATE_I of every path lane before the cut but the superseded ones: their slots are distinct
            ESTAMP(EP_TOK);
            if (GD) {
                if ((path & keep & ~superseded) >> l & 1ull)
                    D.put(slot, p - base + 1);
            } else {
                if ((path & keep & ~superseded) >> l & 1ull)
                    D.put(slot, p - base + 1);
            }
            wave_order();
            ESTAMP(EP_DICT);
            if (done)
                break;
            ip += end;
            if (ip >= ip_end)
                break;
#pragma unroll
            for (int i = 0; i < kCmpW; i++)
                pw[i] = npw[i];
        }
    }
    push(ii, n - ii, 0, 0);                          // tail + EOF
    if (FUSED) {
        E->drain(tp);                                // through the tail: out_len, status set
        if (pf_acc == 0x9E3779B9u)                   // (keeps the prefetch loads; never matters)
            S.sink = pf_acc;
    }
#undef ESTAMP
}

// Emit wave (two-wave kernels): drains the token queue as the parse wave
// fills it.
template <bool GD>
__device__ void emit_wave(EncLdsT<GD>& S, const uint8_t* in, uint32_t n, uint8_t* out, uint32_t cap,
                          uint32_t* out_len, int32_t* status, uint32_t b)
{
    Emitter<GD> E(S, in, n, out, cap);
    // Lines ahead of the parse wave go to L2 from this wave, so the parse
    // wave's probe, candidate and extension loads hit there: one dword per
    // 128-B line, 8 KiB per load instruction; waiting on them stalls only
    // this wave.
    const uintptr_t lines = (uintptr_t)in & ~(uintptr_t)127;
    const uintptr_t last = ((uintptr_t)in + n - 1) & ~(uintptr_t)3;
    uint32_t pf = 0;                                 // bytes from `lines` already touched
    auto prefetch = [&]() {
        if (!POM_ENC_AHEAD)
            return;
        const uint32_t ahead = *(volatile uint32_t*)&S.ip + POM_ENC_AHEAD;
        const uint32_t want = ahead < n + 127 ? ahead : n + 127;
        if (pf >= want)
            return;
        uint32_t x = 0;
        for (; pf < want; pf += 128 * kWave) {
            const uintptr_t a = lines + pf + 128 * lane_id();
            if (a <= last)
                x ^= *(gdword*)a;
        }
        if (x == 0x9E3779B9u)                        // (keeps the loads; never matters)
            S.sink = x;
    };
    for (;;) {
        prefetch();
        const uint32_t prod = lds_load(&S.prod);
        if (E.ct == prod) {
            __builtin_amdgcn_s_sleep(POM_EMIT_SLEEP);
            continue;
        }
        if (E.drain(prod, out_len, status, b))
            return;
    }
}

// One block: both waves, then the workgroup is ready for the next one.
template <bool STAMPS, bool GD>
__device__ __forceinline__ void encode_block(EncLdsT<GD>& S, const Dict<GD> D,
                                             const uint8_t* __restrict__ src,
                                             const uint64_t* __restrict__ src_off,
                                             const uint32_t* __restrict__ src_len,
                                             uint8_t* __restrict__ dst,
                                             const uint64_t* __restrict__ dst_off,
                                             const uint32_t* __restrict__ dst_cap,
                                             uint32_t* __restrict__ out_len,
                                             int32_t* __restrict__ status, uint32_t b,
                                             uint64_t* __restrict__ stamps)
{
    const uint32_t n = src_len[b];
    if (n > kMaxN) {                                 // (u32 positions, 16-bit token lengths kept small)
        if (threadIdx.x == 0)
            status[b] = LZO_MI355X_ENC_PENDING;
        return;
    }
    const uint32_t l = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x == 0) {
        S.prod = 0;
        S.cons = 0;
        S.ip = 0;
    }
    __syncthreads();
    const uint8_t* in = src + src_off[b];
    if (wave == 0) {
        uint64_t acc[EP_N] = {};
        parse_wave<STAMPS, GD>(S, D, in, n, l, acc);
        if (STAMPS && l == 0)
            for (int i = 0; i < EP_N; i++)
                stamps[(size_t)b * kEncStampSlots + i] = acc[i];
    } else
        emit_wave<GD>(S, in, n, dst + dst_off[b], dst_cap[b], out_len, status, b);
}

template <bool STAMPS>
__global__ __launch_bounds__(2 * kWave) void lzo1x_encode_fast_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ src_len, uint8_t* __restrict__ dst,
    const uint64_t* __restrict__ dst_off, const uint32_t* __restrict__ dst_cap,
    uint32_t* __restrict__ out_len, int32_t* __restrict__ status, uint32_t nblocks,
    uint64_t* __restrict__ stamps)
{
    __shared__ EncLds S;
    const uint32_t b = blockIdx.x;
    if (b >= nblocks)
        return;
    Dict<false> D;
    D.lds = S.dict;
    D.g = nullptr;
    D.occ = nullptr;
    encode_block<STAMPS, false>(S, D, src, src_off, src_len, dst, dst_off, dst_cap, out_len, status,
                                b, stamps);
}

// Global-dictionary encoders: a grid of resident workgroups, each with its
// own dictionary region.  Workgroup g codes block g, then (when the batch has
// more blocks than the grid) takes block gridDim.x + ticket++ until none is
// left: a workgroup that drew small blocks takes more of them, so mixed sizes
// (C4: 4-256 KiB) finish together instead of with the unluckiest stride.
__device__ __forceinline__ uint32_t next_block(uint32_t* ticket)
{
    uint32_t t = 0;
    if (lane_id() == 0)
        t = atomicAdd(ticket, 1u);
    return gridDim.x + __builtin_amdgcn_readfirstlane(t);
}

template <bool STAMPS>
__global__ __launch_bounds__(2 * kWave, POM_ENC_RESIDENT / 2) void lzo1x_encode_gdict_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ src_len, uint8_t* __restrict__ dst,
    const uint64_t* __restrict__ dst_off, const uint32_t* __restrict__ dst_cap,
    uint32_t* __restrict__ out_len, int32_t* __restrict__ status, uint32_t nblocks,
    uint8_t* __restrict__ dicts, uint64_t* __restrict__ stamps)
{
    __shared__ EncLdsT<true> S;
    __shared__ uint32_t next;
    Dict<true> D;
    D.lds = nullptr;
    D.g = (gu16*)(dicts + kScratchHead + (size_t)blockIdx.x * kDictBytes);
    D.occ = S.occ;
    D.rs = __builtin_amdgcn_make_buffer_rsrc((void*)D.g, 0, (int)(kSlots * 2), 0x00020000);
    const bool dyn = nblocks > gridDim.x;
    for (uint32_t b = blockIdx.x; b < nblocks;) {
        encode_block<STAMPS, true>(S, D, src, src_off, src_len, dst, dst_off, dst_cap, out_len,
                                   status, b, stamps);
        if (!dyn)
            break;
        if (threadIdx.x < kWave) {
            const uint32_t nb = next_block((uint32_t*)dicts);
            if (threadIdx.x == 0)
                next = nb;
        }
        __syncthreads();                             // both waves done with the block; `next` set
        b = next;
        __syncthreads();                             // (read before the next block overwrites it)
    }
}

// One-wave global-dictionary encoder: the parse wave emits its own tokens
// (parse_wave<..., FUSED>), so a CU holds POM_ENC_RESIDENT1 blocks in flight
// instead of 16 -- more independent parse chains per SIMD to hide the probe
// and candidate round trips.
#ifndef POM_ENC_RESIDENT1
#define POM_ENC_RESIDENT1 16                    // one-wave workgroups per CU (4 waves per SIMD: 128 VGPRs, no spills)
#endif
static_assert(sizeof(EncLdsT<true>) * POM_ENC_RESIDENT1 <= 160 * 1024, "LDS budget");

template <bool STAMPS>
__device__ __forceinline__ void gdict1_body(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ src_len, uint8_t* __restrict__ dst,
    const uint64_t* __restrict__ dst_off, const uint32_t* __restrict__ dst_cap,
    uint32_t* __restrict__ out_len, int32_t* __restrict__ status, uint32_t nblocks,
    uint8_t* __restrict__ dicts, const uint32_t* __restrict__ order, uint64_t* __restrict__ stamps)
{
    __shared__ EncLdsT<true> S;
    Dict<true> D;
    D.lds = nullptr;
    D.g = (gu16*)(dicts + kScratchHead + (size_t)blockIdx.x * kDictBytes);
    D.occ = S.occ;
    D.rs = __builtin_amdgcn_make_buffer_rsrc((void*)D.g, 0, (int)(kSlots * 2), 0x00020000);
    const uint32_t l = lane_id();
    const bool dyn = nblocks > gridDim.x;
    for (uint32_t t = blockIdx.x; t < nblocks; t = dyn ? next_block((uint32_t*)dicts) : nblocks) {
        const uint32_t b = order ? order[t] : t;      // (largest first: lzo_mi355x_launch_order_by_size)
        const uint32_t n = src_len[b];
        if (n > kMaxN) {                             // the general encoder's
            if (l == 0)
                status[b] = LZO_MI355X_ENC_PENDING;
            continue;
        }
        const uint8_t* in = src + src_off[b];
        Emitter<true> E(S, in, n, dst + dst_off[b], dst_cap[b]);
        E.olen = out_len;
        E.ost = status;
        E.blk = b;
        E.prio = !dyn;                               // (block tickets: mixed sizes, no priority)
        uint64_t acc[EP_N] = {};
        parse_wave<STAMPS, true, true>(S, D, in, n, l, acc, &E);
        if (STAMPS && l == 0)
            for (int i = 0; i < EP_N; i++)
                stamps[(size_t)b * kEncStampSlots + i] = acc[i];
        wave_order();
    }
}

__global__ __launch_bounds__(kWave, POM_ENC_RESIDENT1 / 4) void lzo1x_encode_gdict1_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ src_len, uint8_t* __restrict__ dst,
    const uint64_t* __restrict__ dst_off, const uint32_t* __restrict__ dst_cap,
    uint32_t* __restrict__ out_len, int32_t* __restrict__ status, uint32_t nblocks,
    uint8_t* __restrict__ dicts, const uint32_t* __restrict__ order)
{
    gdict1_body<false>(src, src_off, src_len, dst, dst_off, dst_cap, out_len, status, nblocks, dicts,
                       order, nullptr);
}

// (diagnostic) the same with the parse wave's phase stamps
__global__ __launch_bounds__(kWave, POM_ENC_RESIDENT1 / 4) void lzo1x_encode_gdict1_stamps_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ src_len, uint8_t* __restrict__ dst,
    const uint64_t* __restrict__ dst_off, const uint32_t* __restrict__ dst_cap,
    uint32_t* __restrict__ out_len, int32_t* __restrict__ status, uint32_t nblocks,
    uint8_t* __restrict__ dicts, uint64_t* __restrict__ stamps)
{
    gdict1_body<true>(src, src_off, src_len, dst, dst_off, dst_cap, out_len, status, nblocks, dicts,
                      nullptr, stamps);
}

}  // namespace

// Waves per block of the global-dictionary encoder: debug key enc_waves of
// POM_LZO_DEBUG (1 or 2, read at every launch, for the tests of both
// kernels), default 1.
static int enc_waves(void)
{
    return pom_dbg_int("enc_waves", 1) == 2 ? 2 : 1;
}

static uint32_t enc_resident(void)
{
    static int cus[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64)
        return 256 * POM_ENC_RESIDENT;
    if (!cus[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        cus[dev] = n;
    }
    return (uint32_t)cus[dev] * (enc_waves() == 1 ? POM_ENC_RESIDENT1 : POM_ENC_RESIDENT);
}

// Start order of a batch with more blocks than resident workgroups (bytes at
// the end of the scratch, after the dictionary regions).
static size_t enc_order_bytes(uint32_t nblocks)
{
    return nblocks > enc_resident() ? ((size_t)4 * nblocks + 255) / 256 * 256 : 0;
}

// Grid of the global-dictionary encoders: one workgroup per dictionary region
// of the scratch, at most one per block and one per resident slot, and at
// most the debug key enc_grid.
static uint32_t enc_grid(size_t scratch_bytes, uint32_t nblocks)
{
    const size_t ob = enc_order_bytes(nblocks);
    if (scratch_bytes >= kScratchHead + kDictBytes + ob)
        scratch_bytes -= ob;                         // (room for the start order)
    uint32_t grid = scratch_bytes > kScratchHead ? (uint32_t)((scratch_bytes - kScratchHead) / kDictBytes) : 0u;
    grid = grid < nblocks ? grid : nblocks;
    grid = grid < enc_resident() ? grid : enc_resident();
    const uint32_t cap = (uint32_t)pom_dbg_int("enc_grid", 0);   // (tests: a grid smaller than the batch)
    return cap && cap < grid ? cap : grid;
}

extern "C" size_t lzo_mi355x_compress_scratch(uint32_t nblocks)
{
    const uint32_t g = nblocks < enc_resident() ? nblocks : enc_resident();
    return kScratchHead + (size_t)g * kDictBytes + enc_order_bytes(nblocks);
}

extern "C" int lzo_mi355x_launch_compress_fast(const uint8_t* src, const uint64_t* src_off,
                                               const uint32_t* src_len, uint8_t* dst,
                                               const uint64_t* dst_off, const uint32_t* dst_cap,
                                               uint32_t* out_len, int32_t* status,
                                               uint32_t nblocks, void* scratch, size_t scratch_bytes,
                                               hipStream_t stream)
{
    if (nblocks == 0)
        return 0;
    const uint32_t grid = scratch ? enc_grid(scratch_bytes, nblocks) : 0u;
    if (grid && grid < nblocks && hipMemsetAsync(scratch, 0, sizeof(uint32_t), stream) != hipSuccess)
        return -1;                                   // (the block ticket)
    // largest first when the blocks outnumber the workgroups and the scratch
    // has room for the order after the grid's dictionaries
    const size_t ob = enc_order_bytes(nblocks);
    const size_t order_at = kScratchHead + (size_t)grid * kDictBytes;
    uint32_t* order = grid && grid < nblocks && ob && order_at + ob <= scratch_bytes
                          ? (uint32_t*)((uint8_t*)scratch + order_at) : nullptr;
    if (order && enc_waves() == 1 && lzo_mi355x_launch_order_by_size(src_len, nblocks, order, stream) != 0)
        return -1;
    if (grid && enc_waves() == 1)
        hipLaunchKernelGGL(lzo1x_encode_gdict1_kernel, dim3(grid), dim3(kWave), 0, stream, src, src_off,
                           src_len, dst, dst_off, dst_cap, out_len, status, nblocks, (uint8_t*)scratch,
                           (const uint32_t*)order);
    else if (grid)
        hipLaunchKernelGGL(lzo1x_encode_gdict_kernel<false>, dim3(grid), dim3(2 * kWave), 0, stream,
                           src, src_off, src_len, dst, dst_off, dst_cap, out_len, status, nblocks,
                           (uint8_t*)scratch, nullptr);
    else
        hipLaunchKernelGGL(lzo1x_encode_fast_kernel<false>, dim3(nblocks), dim3(2 * kWave), 0, stream,
                           src, src_off, src_len, dst, dst_off, dst_cap, out_len, status, nblocks,
                           nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Diagnostic: the same encoder with parse-wave phase stamps (16 x u64 per block).
extern "C" int lzo_mi355x_debug_compress_fast_stamps(const uint8_t* src, const uint64_t* src_off,
                                                     const uint32_t* src_len, uint8_t* dst,
                                                     const uint64_t* dst_off,
                                                     const uint32_t* dst_cap, uint32_t* out_len,
                                                     int32_t* status, uint32_t nblocks,
                                                     uint64_t* stamps, hipStream_t stream)
{
    if (nblocks == 0)
        return 0;
    hipLaunchKernelGGL(lzo1x_encode_fast_kernel<true>, dim3(nblocks), dim3(2 * kWave), 0, stream,
                       src, src_off, src_len, dst, dst_off, dst_cap, out_len, status, nblocks,
                       stamps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Diagnostic: the global-dictionary encoder with parse-wave phase stamps.
extern "C" int lzo_mi355x_debug_compress_gdict_stamps(const uint8_t* src, const uint64_t* src_off,
                                                      const uint32_t* src_len, uint8_t* dst,
                                                      const uint64_t* dst_off,
                                                      const uint32_t* dst_cap, uint32_t* out_len,
                                                      int32_t* status, uint32_t nblocks,
                                                      void* scratch, size_t scratch_bytes,
                                                      uint64_t* stamps, hipStream_t stream)
{
    const uint32_t grid = enc_grid(scratch_bytes, nblocks);
    if (grid == 0 || (grid < nblocks && hipMemsetAsync(scratch, 0, sizeof(uint32_t), stream) != hipSuccess))
        return -1;
    hipLaunchKernelGGL(lzo1x_encode_gdict_kernel<true>, dim3(grid), dim3(2 * kWave), 0, stream,
                       src, src_off, src_len, dst, dst_off, dst_cap, out_len, status, nblocks,
                       (uint8_t*)scratch, stamps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Diagnostic: the one-wave global-dictionary encoder (the bench's) with
// parse-wave phase stamps (16 x u64 per block; no start order).
extern "C" int lzo_mi355x_debug_compress_gdict1_stamps(const uint8_t* src, const uint64_t* src_off,
                                                       const uint32_t* src_len, uint8_t* dst,
                                                       const uint64_t* dst_off,
                                                       const uint32_t* dst_cap, uint32_t* out_len,
                                                       int32_t* status, uint32_t nblocks,
                                                       void* scratch, size_t scratch_bytes,
                                                       uint64_t* stamps, hipStream_t stream)
{
    const uint32_t grid = enc_grid(scratch_bytes, nblocks);
    if (grid == 0 || (grid < nblocks && hipMemsetAsync(scratch, 0, sizeof(uint32_t), stream) != hipSuccess))
        return -1;
    hipLaunchKernelGGL(lzo1x_encode_gdict1_stamps_kernel, dim3(grid), dim3(kWave), 0, stream,
                       src, src_off, src_len, dst, dst_off, dst_cap, out_len, status, nblocks,
                       (uint8_t*)scratch, stamps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
