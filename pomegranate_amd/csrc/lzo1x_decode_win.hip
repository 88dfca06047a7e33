// lzo1x_decode_win.hip -- the windowed LZO1X decoder for MI355X (gfx950).
//
// One workgroup of 8 waves per block; the block's last 64 KiB of output stay
// resident in an LDS ring (every LZO1X match distance, <= 0xBFFF, reaches into
// it), so a block never reads its own output back from HBM.  Two workgroups
// share a CU (80 KB of LDS each).  The block is decoded as an alternation of
//
//  * PIECES of compressed input (kZH = 2 KiB, staged in one half of a 4 KiB
//    LDS ring): 128 parse lanes, each owning a 16-byte segment, find the
//    instruction starts of the LZO1X grammar (lib/minilzo.c:3308-3699,
//    SURVEY.md Appendix A.2) as a state machine over (position, state):
//      - every lane walks speculatively from 16 bytes before its segment and
//        keeps the starts it visits inside the segment as per-state bitmaps;
//      - a lane whose true entry (its predecessor's exit) is not one of its
//        speculative starts walks exactly from it until it lands on one; the
//        exits settle by Jacobi iteration over the lanes (one barrier each,
//        about two rounds per piece on ITB streams);
//      - a counting walk, a scan over the lanes, and an emitting walk write
//        the piece's ops (output start, literal zin offset or match distance)
//        to an LDS op table of kOpCap entries;
//  * WINDOWS of output (kW = 4 KiB, lane = 8 output bytes): every output byte
//    gets a source pointer, encoded as e = B - t for a source at output
//    position t (B = window end - 1); literal bytes are written into the ring
//    first and point at themselves as final (e = kFin + offset).  Matches that overlap themselves (distance d < length) are reduced
//    to the last period before max(op start, window start).  A source inside
//    the window (e <= T) is followed through the window's pointer table
//    (e = tab[W - 1 - e], with write-back, so chains shorten as they are
//    walked) until it is a literal or lies before the window.  Then every
//    byte is one independent LDS gather, written to the ring and to HBM.
//    The pointer table (2 bytes per window byte) lives in the ring itself,
//    just past the window: those slots hold output older than any match can
//    reach (kW <= 8 KiB).
//
// Blocks it does not finish exactly (malformed input, lookbehind/capacity
// errors, instructions longer than a piece, misaligned destinations) are
// appended to the fallback list for lzo1x_decode_exact_kernel
// (lzo1x_kernels.hip), which produces the reference's output and LZO_E_* code
// bit for bit.  The algorithm was checked first as a sequential C model
// (scripts/dbg/win_model.c) against the oracle.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lzo_mi355x_kernels.h"

namespace {

constexpr uint32_t kWave = 64;
constexpr uint32_t kNT = 512;                    // threads per workgroup (8 waves)
constexpr uint32_t kW = 4096;                    // window bytes (8 per thread)
constexpr uint32_t kZH = 2048;                   // compressed bytes per piece (instruction starts)
constexpr uint32_t kZS = kZH + 64;               // bytes staged per piece (headers past its end)
constexpr uint32_t kZR = 2 * kZS;                // zin ring (two pieces)
constexpr uint32_t kOpCap = 1024;                // ops held at once
constexpr uint32_t kG = 32;                      // parse segment bytes
constexpr uint32_t kNPL = kZH / kG;              // parse lanes (wave 0)
constexpr uint32_t kLook = 32;                   // speculative lead-in
constexpr uint32_t kFin = 53248u;                // e >= kFin: final byte at ring[A + e - kFin]
constexpr uint32_t kLitF = 0x80000000u;          // op source: literal ...
constexpr uint32_t kLitG = 0x40000000u;          // ... at an input position (else a zin offset)
constexpr int32_t kFallback = 0x7FFF0001;
static_assert(kW * 8 == kNT * 64, "window: 8 bytes per thread");
static_assert(kW + 2 * kW <= 65536u - 0xBFFFu - 1u, "pointer table [A+W, A+3W) in dead ring slots");
static_assert(0xBFFFu + kW < kFin && kFin + kW <= 65536u, "e encoding: match pointers below final ones");
static_assert(kNPL == kWave, "one parse wave");

enum : uint32_t { ST_A = 0, ST_B = 1, ST_C = 2, ST_F = 3 };
enum : uint32_t { TK_EOF = 1, TK_BAD = 2 };
// piece results
enum : uint32_t { PR_OK = 0, PR_EOF = 1, PR_FULL = 2, PR_REFUSE = 3 };
// control words
enum : uint32_t { C_REFUSE = 0, C_SPOS, C_SST, C_SKIND, C_TOPS, C_TBYTES, C_N = 16 };

struct __attribute__((aligned(16))) WinLds {
    uint8_t ring[65536];
    uint32_t zin[kZR / 4 + 4];                   // + pad: 4-byte reads past the end
    uint32_t opp[kOpCap + 4];                    // op output start; opp[nops] = end
    uint32_t ops[kOpCap];                        // kLitF | zin offset, or match distance
    uint32_t bmap[2][kW / 32];                   // op starts of the window
    uint32_t ctl[C_N];
    uint64_t stamp[16];                          // diagnostics (STAMPS builds)
};
static_assert(sizeof(WinLds) <= 81920, "two workgroups per CU");

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Inclusive prefix sum over the wave (DPP row shifts, then row totals).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);
    const uint32_t r0 = __builtin_amdgcn_readlane(v, 15), r1 = __builtin_amdgcn_readlane(v, 31),
                   r2 = __builtin_amdgcn_readlane(v, 47);
    const uint32_t row = lane_id() >> 4;
    v += (row >= 1 ? r0 : 0u) + (row >= 2 ? r1 : 0u) + (row >= 3 ? r2 : 0u);
    return v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) { return __builtin_amdgcn_readlane(wave_incl_scan(v), 63); }

// ---- compressed input (staged piece) --------------------------------------
struct Piece {
    uint32_t I;          // input position of zin byte zb
    uint32_t zb;         // byte offset of the piece's half in zin
    uint32_t sEnd;       // I + kZS: [I, sEnd) is staged (zero past z)
    uint32_t z;
    const uint8_t* in;   // the whole compressed block (HBM)
};

__device__ __forceinline__ uint32_t zbyte(const WinLds& L, uint32_t off)
{
    return (L.zin[off >> 2] >> (8u * (off & 3u))) & 0xFFu;
}

// input byte p < z: from the staged piece, or from HBM past it
__device__ __forceinline__ uint32_t in_byte(const WinLds& L, const Piece& k, uint32_t p)
{
    return p < k.sEnd ? zbyte(L, k.zb + (p - k.I)) : (uint32_t)k.in[p];
}

struct Tok {
    uint32_t pos, st;    // next instruction start
    uint32_t aL, aS;     // op A: length, source (kLitF | input pos, or distance)
    uint32_t bL, bS;     // op B: trailing literals (bL == 0: none)
    uint32_t fl;         // TK_*
};

constexpr uint32_t kMaxExtZeros = 64;            // zero length-extension bytes a lane reads at most
constexpr uint32_t kMaxRunZeros = 1u << 24;      // zero bytes the true path takes in one extension

// One instruction at (pos, st), general form: long length extensions and
// instructions that run past the staged piece (bytes read from HBM).  Bytes
// at or past z read as 0 and make the instruction TK_BAD.
__device__ __noinline__ Tok tok_slow(const WinLds& L, const Piece k, uint32_t pos, uint32_t st, bool spec)
{
    Tok r;
    r.aL = r.bL = r.aS = r.bS = 0;
    r.fl = 0;
    uint32_t far = 0;    // furthest byte read + 1
    auto rd = [&](uint32_t p) -> uint32_t {
        far = p + 1 > far ? p + 1 : far;
        return p < k.z ? in_byte(L, k, p) : 0u;
    };
    // (spec: a lane decoding speculatively from inside a long zero run would
    // scan the rest of it, for every start in the run; after kMaxExtZeros zero
    // bytes its guess is refused instead.  The true path -- the frontier,
    // counting and emitting walks -- scans each run once: linear time)
    // (the true path too: a run of 2^24 zero bytes or more is refused, so the
    // block goes to the exact decoder, which keeps the reference's 64-bit
    // length, lib/minilzo.c:3805 -- from 16,843,009 zeros on, 255 per zero
    // passes 2^32 and this u32 sum would wrap to a small, valid-looking length)
    bool capped = false;
    auto ext = [&](uint32_t& p, uint32_t base) -> uint32_t {
        uint32_t v = 0;
        while (p < k.z) {
            if (v >= 255u * kMaxRunZeros) {
                capped = true;
                break;
            }
            // (past the staged piece, aligned 16-byte reads take a long zero
            // run 16 bytes at a time: such a read never leaves the page of the
            // block's byte at p)
            if (!spec && p >= k.sEnd && p + 16 <= k.z && ((uintptr_t)(k.in + p) & 15u) == 0) {
                const uint4 w = *(const uint4*)(k.in + p);
                if ((w.x | w.y | w.z | w.w) == 0) {
                    v += 255u * 16;
                    p += 16;
                    far = p > far ? p : far;
                    continue;
                }
            }
            if (rd(p) != 0)
                break;
            v += 255;
            p++;
            if (spec && v > 255u * kMaxExtZeros) {
                capped = true;
                break;
            }
        }
        v += base + rd(p);
        p++;
        return v;
    };
    uint32_t t = rd(pos);
    if (st == ST_F) {
        if (t > 17) {
            const uint32_t n = t - 17;
            r.aL = n;
            r.aS = kLitF | (pos + 1);
            r.pos = pos + 1 + n;
            r.st = n < 4 ? ST_C : ST_B;
            goto done;
        }
        st = ST_A;
    }
    {
        uint32_t Ln, d;
        if (t < 16 && st == ST_A) {
            pos++;
            if (t == 0)
                t = ext(pos, 15);
            r.aL = t + 3;
            r.aS = kLitF | pos;
            r.pos = pos + t + 3;
            r.st = ST_B;
            goto done;
        }
        if (t < 16) {
            d = (st == ST_B ? 0x801u : 1u) + (t >> 2) + (rd(pos + 1) << 2);
            Ln = st == ST_B ? 3u : 2u;
            pos += 2;
        } else if (t >= 64) {
            d = 1 + ((t >> 2) & 7) + (rd(pos + 1) << 3);
            Ln = (t >> 5) + 1;
            pos += 2;
        } else if (t >= 32) {
            Ln = t & 31;
            pos++;
            if (Ln == 0)
                Ln = ext(pos, 31);
            Ln += 2;
            d = 1 + ((rd(pos) | (rd(pos + 1) << 8)) >> 2);
            pos += 2;
        } else {
            uint32_t dd = (t & 8) << 11;
            Ln = t & 7;
            pos++;
            if (Ln == 0)
                Ln = ext(pos, 7);
            Ln += 2;
            dd += (rd(pos) | (rd(pos + 1) << 8)) >> 2;
            pos += 2;
            if (dd == 0) {
                r.fl = TK_EOF;
                r.pos = pos;
                r.st = ST_A;
                goto done;
            }
            d = dd + 0x4000;
        }
        r.aL = Ln;
        r.aS = d;
        const uint32_t tl = rd(pos - 2) & 3;
        if (tl) {
            r.bL = tl;
            r.bS = kLitF | pos;
            pos += tl;
            r.st = ST_C;
        } else
            r.st = ST_A;
        r.pos = pos;
    }
done:
    {
        const uint32_t need = far > r.pos ? far : r.pos;
        if (need > k.z || r.pos < pos || capped)
            r.fl = TK_BAD;                       // runs past the input (INPUT_OVERRUN), or a capped zero run
        else if ((r.fl & TK_EOF) && r.pos != k.z)
            r.fl = TK_BAD;                       // EOF not at the end (INPUT_NOT_CONSUMED)
    }
    return r;
}

// Branch-free form for the common case: the instruction's fields lie in its
// first 4 bytes (no 255-chunk length extension) inside the staged piece.
// One zin round trip.
__device__ __forceinline__ Tok tok(const WinLds& L, const Piece& k, uint32_t pos, uint32_t st, bool spec = false)
{
    const uint32_t off = k.zb + (pos - k.I);
    const uint32_t lo = __builtin_amdgcn_alignbyte(L.zin[(off >> 2) + 1], L.zin[off >> 2], off & 3u);
    const uint32_t t = lo & 0xFFu, b1 = __builtin_amdgcn_ubfe(lo, 8, 8);
    const bool flit = st == ST_F && t > 17;
    const uint32_t se = st == ST_F ? ST_A : st;
    const bool lit = !flit && se == ST_A && t < 16;
    const bool m1 = !flit && !lit && t < 16;
    const bool m2 = !flit && t >= 64;
    const bool m3 = !flit && t >= 32 && t < 64;
    const bool m4 = !flit && t >= 16 && t < 32;
    const bool ext = (lit && t == 0) || (m3 && (t & 31) == 0) || (m4 && (t & 7) == 0);
    if (__builtin_expect((ext && b1 == 0) || pos + 4 > k.sEnd, 0))
        return tok_slow(L, k, pos, st, spec);
    const uint32_t e = ext ? 1u : 0u;
    const uint32_t o16 = __builtin_amdgcn_ubfe(lo, 8u + 8u * e, 16);
    const uint32_t dd4 = ((t & 8u) << 11) + (o16 >> 2);
    const uint32_t used = (m1 || m2) ? 2u : 3u + e;
    const uint32_t tl = __builtin_amdgcn_ubfe(lo, 8u * (used - 2u), 2);
    const uint32_t nlit = flit ? t - 17 : (ext ? 15u + b1 : t) + 3u;
    const uint32_t Ln = m1 ? (se == ST_B ? 3u : 2u)
                      : m2 ? (t >> 5) + 1u
                      : m3 ? (ext ? 31u + b1 : (t & 31u)) + 2u
                           : (ext ? 7u + b1 : (t & 7u)) + 2u;
    const uint32_t d = m1 ? (se == ST_B ? 0x801u : 1u) + (t >> 2) + (b1 << 2)
                     : m2 ? 1u + ((t >> 2) & 7u) + (b1 << 3)
                     : m3 ? 1u + (o16 >> 2) : dd4 + 0x4000u;
    const bool eof = m4 && dd4 == 0;
    const bool islit = flit || lit;
    const uint32_t hdr = flit ? 1u : 1u + e;
    Tok r;
    r.aL = eof ? 0u : islit ? nlit : Ln;
    r.aS = islit ? kLitF | (pos + hdr) : d;
    r.bL = (islit || eof) ? 0u : tl;
    r.bS = kLitF | (pos + used);
    r.pos = islit ? pos + hdr + nlit : pos + used + (eof ? 0u : tl);
    r.st = islit ? (flit && nlit < 4 ? ST_C : ST_B) : (tl && !eof ? ST_C : ST_A);
    // the instruction (header, then literals) ends at r.pos
    r.fl = r.pos > k.z ? TK_BAD : eof ? (r.pos != k.z ? TK_BAD : TK_EOF) : 0u;
    return r;
}

__device__ __forceinline__ uint32_t pack_pt(const Piece& k, uint32_t pos, uint32_t st) { return ((pos - k.I) << 2) | st; }

// ---- diagnostics: per-phase cycle stamps (STAMPS builds only) ----------------
// (thread 0 accumulates into L.stamp; L.stamp[15] holds the last time)
#define STAMP(i)                                                   \
    do {                                                           \
        if (STAMPS && threadIdx.x == 0) {                          \
            const uint64_t _t = clock64();                         \
            L.stamp[(i)] += _t - L.stamp[15];                      \
            L.stamp[15] = _t;                                      \
        }                                                          \
    } while (0)
#define COUNT(i, n)                                                \
    do {                                                           \
        if (STAMPS && threadIdx.x == 0)                            \
            L.stamp[(i)] += (n);                                   \
    } while (0)

// ---- block state ----------------------------------------------------------
struct Blk {
    const uint8_t* in;
    uint8_t* out;
    uint32_t z, cap;
};

// ---- piece parse ------------------------------------------------------------
struct PieceOut {
    uint32_t result;     // PR_*
    uint32_t I, st;      // next piece entry
    uint32_t nops, E;    // op count and output end after the piece
};

template <bool STAMPS>
__device__ PieceOut parse_piece(WinLds& L, const Blk& blk, uint32_t I, uint32_t st_in,
                                uint32_t nops, uint32_t E, uint32_t half)
{
    const uint32_t tid = threadIdx.x;
    Piece k;
    k.I = I;
    k.zb = half * kZS;
    k.z = blk.z;
    k.sEnd = I + kZS;
    k.in = blk.in;

    // stage kZS bytes from I (0 past z): thread t the dwords t and t + kNT
    {
        const uintptr_t base = (uintptr_t)(blk.in + I);
        const uint32_t sh = (uint32_t)(base & 3u);
        const uint32_t* aw = (const uint32_t*)(base - sh);
        for (uint32_t w = tid; w < kZS / 4; w += kNT) {
            const uint32_t p = I + 4 * w;
            uint32_t v = 0;
            if (p - sh + 8 <= blk.z) {            // both aligned dwords inside the input
                v = __builtin_amdgcn_alignbyte(aw[w + 1], aw[w], sh);
            } else {
                for (uint32_t i = 0; i < 4; i++)
                    if (p + i < blk.z)
                        v |= (uint32_t)blk.in[p + i] << (8 * i);
            }
            L.zin[(k.zb >> 2) + w] = v;
        }
    }
    __syncthreads();
    STAMP(0);

    PieceOut r;
    if (tid < kWave) {
        // ---- wave 0: the parse; lane j owns input segment [a, b) ------------
        const uint32_t j = tid;
        const uint32_t a = I + kG * j, b = a + kG;
        const uint32_t entry0 = pack_pt(k, I, st_in);
        uint32_t bm0 = 0, bm1 = 0, bm2 = 0, sx;

        // P1: speculative walk from kLook bytes before the segment
        if (a >= blk.z && j) {
            sx = pack_pt(k, b, ST_A);
        } else {
            uint32_t pos = j ? (a >= I + kLook ? a - kLook : I) : I;
            uint32_t st = j ? (uint32_t)ST_A : st_in;
            uint32_t restart = pos;
            while (pos < b) {
                const Tok t = tok(L, k, pos, st, j != 0);   // (lane 0 starts at the true entry)
                if (t.fl) {
                    if (j == 0 || (t.fl & TK_EOF))
                        break;                   // stop point
                    restart++;                   // impossible guess: start one byte later
                    pos = restart;
                    st = ST_A;
                    bm0 = bm1 = bm2 = 0;
                    continue;
                }
                if (pos >= a) {
                    const uint32_t bit = 1u << (pos - a);
                    const uint32_t s2 = st == ST_F ? ST_A : st;
                    bm0 |= s2 == ST_A ? bit : 0u;
                    bm1 |= s2 == ST_B ? bit : 0u;
                    bm2 |= s2 == ST_C ? bit : 0u;
                }
                pos = t.pos;
                st = t.st;
            }
            if (pos >= a && pos < b) {           // stopped inside: the stop point is a start
                const uint32_t bit = 1u << (pos - a);
                const uint32_t s2 = st == ST_F ? ST_A : st;
                bm0 |= s2 == ST_A ? bit : 0u;
                bm1 |= s2 == ST_B ? bit : 0u;
                bm2 |= s2 == ST_C ? bit : 0u;
            }
            sx = pack_pt(k, pos, st);
        }
        STAMP(1);

        auto in_bm = [&](uint32_t key) -> bool {
            const uint32_t pos = I + (key >> 2), st = key & 3u;
            if (pos < a || pos >= b)
                return false;
            const uint32_t s2 = st == ST_F ? ST_A : st;
            const uint32_t m = s2 == ST_A ? bm0 : s2 == ST_B ? bm1 : bm2;
            return (m >> (pos - a)) & 1u;
        };

        // P2: settle the exits from the true entries.  ok: this lane's exit is
        // its speculative one whenever its predecessor's is.  A frontier f
        // moves over the lanes: runs of ok lanes are taken at once (ballot),
        // entries past a segment pass over it, and only a lane whose true
        // entry is not one of its speculative starts walks.
        const uint32_t psx = (uint32_t)__shfl_up((int)sx, 1, kWave);
        const uint64_t okm = __ballot(j > 0 && in_bm(psx));
        uint32_t x = sx;
        uint32_t f = 1, cur = uni(__builtin_amdgcn_readlane(sx, 0));
        while (f < kWave) {
            const uint32_t cpos = I + (cur >> 2);
            const uint32_t af = I + kG * f;
            if (cpos < af) {                     // a stop point: no starts after it
                x = j >= f ? cur : x;
                break;
            }
            if (cpos >= af + kG) {               // passes over lanes f .. g-1
                uint32_t g = (cpos - I) / kG;
                g = g < kWave ? g : kWave;
                x = (j >= f && j < g) ? cur : x;
                f = g;
                continue;
            }
            COUNT(12, 1);
            const uint64_t hit = __ballot(in_bm(cur));
            if ((hit >> f) & 1ull) {
                // lanes f .. g-1 keep their speculative exits
                const uint64_t rest = f + 1 < kWave ? ~okm & (~0ull << (f + 1)) : 0ull;
                const uint32_t g = rest ? (uint32_t)__builtin_ctzll(rest) : kWave;
                cur = uni(__builtin_amdgcn_readlane(sx, g - 1));
                f = g;
            } else {
                const uint64_t tw0 = STAMPS ? clock64() : 0;
                uint32_t w = 0, nwt = 0;
                if (j == f) {                    // walk from the true entry
                    uint32_t pos = cpos, st = cur & 3u;
                    for (;;) {
                        const Tok t = tok(L, k, pos, st);
                        nwt++;
                        if (t.fl) {
                            w = pack_pt(k, pos, st);
                            break;
                        }
                        pos = t.pos;
                        st = t.st;
                        if (pos >= b) {
                            w = pack_pt(k, pos, st);
                            break;
                        }
                        const uint32_t key = pack_pt(k, pos, st);
                        if (in_bm(key)) {
                            w = sx;
                            break;
                        }
                    }
                    x = w;
                }
                cur = uni(__builtin_amdgcn_readlane(w, f));
                if (STAMPS && threadIdx.x == 0) {
                    L.stamp[13] += clock64() - tw0;
                    L.stamp[14] += __builtin_amdgcn_readlane(nwt, f);
                }
                f++;
            }
        }
        STAMP(2);

        // P3: count ops and bytes on the true path
        uint32_t ent = (uint32_t)__shfl_up((int)x, 1, kWave);
        if (j == 0)
            ent = entry0;
        uint32_t c_ops = 0, c_bytes = 0, skind = 0, spos = 0, sst = 0;
        {
            uint32_t pos = I + (ent >> 2), st = ent & 3u;
            if (pos >= a) {
                while (pos < b) {
                    const Tok t = tok(L, k, pos, st);
                    if (t.fl) {
                        skind = t.fl;
                        spos = pos;
                        sst = st;
                        break;
                    }
                    c_ops += (t.aL ? 1u : 0u) + (t.bL ? 1u : 0u);
                    c_bytes += t.aL + t.bL;
                    pos = t.pos;
                    st = t.st;
                }
            }
        }
        const uint32_t i_ops = wave_incl_scan(c_ops), i_bytes = wave_incl_scan(c_bytes);
        const uint32_t b_ops = i_ops - c_ops, b_bytes = i_bytes - c_bytes;
        const uint32_t t_ops = uni(__builtin_amdgcn_readlane(i_ops, kWave - 1));
        const uint32_t t_bytes = uni(__builtin_amdgcn_readlane(i_bytes, kWave - 1));
        const uint64_t stops = __ballot(skind != 0);
        STAMP(3);

        // literal source: a zin offset when the bytes are staged, else the input
        // position (long literal runs past the piece are read from HBM)
        auto lit_src = [&](uint32_t q, uint32_t n) -> uint32_t {
            return q + n <= k.sEnd ? kLitF | (k.zb + (q - I)) : kLitF | kLitG | q;
        };
        // P4: emit ops; at the op cap the instruction that does not fit starts
        // the next piece
        const uint32_t avail = kOpCap - nops;
        const uint64_t over = __ballot(b_ops + c_ops > avail);
        uint32_t cut_pos = 0, cut_st = 0, cut_n = 0, cut_out = 0;
        if (c_ops && b_ops <= avail) {
            uint32_t pos = I + (ent >> 2), st = ent & 3u;
            uint32_t n = b_ops, outp = E + b_bytes;
            while (pos < b) {
                const Tok t = tok(L, k, pos, st);
                if (t.fl)
                    break;
                const uint32_t need = (t.aL ? 1u : 0u) + (t.bL ? 1u : 0u);
                if (n + need > avail) {
                    cut_pos = pos;
                    cut_st = st;
                    cut_n = n;
                    cut_out = outp;
                    break;
                }
                if (t.aL) {
                    L.opp[nops + n] = outp;
                    L.ops[nops + n] = (t.aS & kLitF) ? lit_src(t.aS & ~kLitF, t.aL) : t.aS;
                    n++;
                    outp += t.aL;
                }
                if (t.bL) {
                    L.opp[nops + n] = outp;
                    L.ops[nops + n] = lit_src(t.bS & ~kLitF, t.bL);
                    n++;
                    outp += t.bL;
                }
                pos = t.pos;
                st = t.st;
            }
        }
        if (over) {
            const uint32_t cl = (uint32_t)__builtin_ctzll(over);
            r.result = PR_FULL;
            r.I = uni(__builtin_amdgcn_readlane(cut_pos, cl));
            r.st = uni(__builtin_amdgcn_readlane(cut_st, cl));
            r.nops = nops + uni(__builtin_amdgcn_readlane(cut_n, cl));
            r.E = uni(__builtin_amdgcn_readlane(cut_out, cl));
        } else {
            r.nops = nops + t_ops;
            r.E = E + t_bytes;
            if (stops) {
                const uint32_t sl = (uint32_t)__builtin_ctzll(stops);
                const uint32_t sk = uni(__builtin_amdgcn_readlane(skind, sl));
                r.I = uni(__builtin_amdgcn_readlane(spos, sl));
                r.st = uni(__builtin_amdgcn_readlane(sst, sl));
                r.result = (sk & TK_BAD) ? PR_REFUSE : PR_EOF;
                if (sk & TK_EOF)
                    r.I = blk.z;
            } else {
                const uint32_t xl = uni(__builtin_amdgcn_readlane(x, kWave - 1));
                r.I = I + (xl >> 2);
                r.st = xl & 3u;
                r.result = PR_OK;
            }
        }
        if (r.result == PR_OK && r.I == I)
            r.result = PR_REFUSE;                // (never: a piece always starts an instruction)
        if (j == 0) {
            L.opp[r.nops] = r.E;                 // sentinel
            L.ctl[C_SPOS] = r.I;
            L.ctl[C_SST] = r.st;
            L.ctl[C_TOPS] = r.nops;
            L.ctl[C_TBYTES] = r.E;
            L.ctl[C_SKIND] = r.result;
        }
    }
    COUNT(10, 1);
    __syncthreads();
    STAMP(4);
    r.I = uni(L.ctl[C_SPOS]);
    r.st = uni(L.ctl[C_SST]);
    r.nops = uni(L.ctl[C_TOPS]);
    r.E = uni(L.ctl[C_TBYTES]);
    r.result = uni(L.ctl[C_SKIND]);
    return r;
}

// ---- window -------------------------------------------------------------------
// Op starts in (S, A + W) into the bitmap bm (positions relative to A).
__device__ __forceinline__ void scatter_starts(WinLds& L, uint32_t* bm, uint32_t A, uint32_t iS,
                                               uint32_t nops)
{
    for (uint32_t i = iS + 1 + threadIdx.x; i < nops; i += kNT) {
        const uint32_t p = L.opp[i];
        if (p >= A + kW)
            break;
        atomicOr(&bm[(p - A) >> 5], 1u << ((p - A) & 31u));
    }
}

// Output [S, Ew) with the thread grid anchored at A = S & ~15 (bytes of the grid
// below S or at/after Ew are rewritten with their own ring bytes).  Returns
// false on a lookbehind error.  iS: index of the op covering S, updated to the
// op covering Ew.  Two barriers: after the pointer table (and the literal
// bytes) are written, and at the end; the op-start bitmap of the next window
// is filled during this one when that window follows in the same piece
// (next_same), else at the start of the next one (prepped false).
template <bool STAMPS>
__device__ bool run_window(WinLds& L, const Blk& blk, uint32_t S, uint32_t Ew, uint32_t& iS,
                           uint32_t nops, uint32_t& cur, bool& prepped, bool next_same)
{
    const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const uint32_t A = S & ~15u, B = A + kW - 1, T = B - S;
    const uint32_t tabb = A + kW;               // tab[i] at ring[(tabb + 2i) & 0xFFFF]
    uint32_t* const bm = L.bmap[cur];

    if (!prepped) {
        scatter_starts(L, bm, A, iS, nops);
        __syncthreads();
    }
    STAMP(5);

    const uint32_t o = wave * 512 + lane * 8;    // this thread's 8 bytes: A + o ..
    const uint32_t x0 = A + o;
    // ops before the wave's sub-window and in the whole window
    const uint32_t d0 = bm[lane], d1 = bm[lane + 64];
    const uint32_t pc0 = __builtin_popcount(d0), pc1 = __builtin_popcount(d1);
    const uint32_t before = wave_sum((lane < 16 * wave ? pc0 : 0u) + (lane + 64 < 16 * wave ? pc1 : 0u));
    const uint32_t total = wave_sum(pc0 + pc1);
    const uint32_t bits8 = (bm[o >> 5] >> (o & 31u)) & 0xFFu;
    const uint32_t lc = __builtin_popcount(bits8);
    const uint32_t excl = wave_incl_scan(lc) - lc;
    const uint32_t obase = iS + before + excl;

    // source pointers; literal bytes go straight into the ring (final).
    // Branch-free: every load is issued unconditionally from a clamped address
    // and the results selected afterwards, so the loads of the 8 bytes share one
    // wait (a load under a divergent condition becomes a branch with its own
    // s_waitcnt, and 8 of them serialise).
    uint32_t e[8], pv[8], sv[8];
#pragma unroll
    for (uint32_t i = 0; i < 8; i++) {
        uint32_t oi = obase + __builtin_popcount(bits8 & ((2u << i) - 1u));
        oi = oi < kOpCap ? oi : kOpCap - 1;
        pv[i] = L.opp[oi];
        sv[i] = L.ops[oi];
    }
    uint32_t lmask = 0, gmask = 0, lv0 = 0, lv1 = 0;
    bool bad = false;
    uint32_t zv[8];
#pragma unroll
    for (uint32_t i = 0; i < 8; i++) {
        const uint32_t x = x0 + i;
        const bool valid = x >= S && x < Ew;
        const bool lit = valid && (sv[i] & kLitF) != 0;
        lmask |= lit ? 1u << i : 0u;
        gmask |= lit && (sv[i] & kLitG) ? 1u << i : 0u;
        const uint32_t zoff = (sv[i] & 0xFFFFu) + (x - pv[i]);        // (garbage unless a zin literal)
        zv[i] = L.zin[(zoff >> 2) < kZR / 4 ? zoff >> 2 : 0u] >> (8u * (zoff & 3u));
    }
    if (__builtin_expect(gmask != 0, 0)) {          // literal runs longer than a piece (HBM)
#pragma unroll
        for (uint32_t i = 0; i < 8; i++)
            if ((gmask >> i) & 1u)
                zv[i] = blk.in[(sv[i] & 0xFFFFFFu) + (x0 + i - pv[i])];
    }
#pragma unroll
    for (uint32_t i = 0; i < 8; i++) {
        const uint32_t x = x0 + i;
        const bool valid = x >= S && x < Ew;
        const uint32_t p = pv[i], d = sv[i];
        const uint32_t c = zv[i] & 0xFFu;
        if (i < 4)
            lv0 |= ((lmask >> i) & 1u) ? c << (8 * i) : 0u;
        else
            lv1 |= ((lmask >> i) & 1u) ? c << (8 * (i - 4)) : 0u;
        // match: x - d, or for a match of period d < length the last period
        // before max(op start, window start)
        const uint32_t q0 = p > S ? p : S;
        const uint32_t kk = x - q0;                 // < kW + 16
        const uint32_t dd = d & 0xFFFFu ? d & 0xFFFFu : 1u;
        const uint32_t qq = (uint32_t)((float)kk * __builtin_amdgcn_rcpf((float)dd));
        int32_t rr = (int32_t)(kk - qq * dd);
        rr += rr < 0 ? (int32_t)dd : 0;
        rr -= rr >= (int32_t)dd ? (int32_t)dd : 0;
        const uint32_t t = q0 - dd + (uint32_t)rr;
        const bool match = valid && !((lmask >> i) & 1u);
        bad |= match && (d > p || t >= x);          // lookbehind (lib/minilzo.c:3628); t >= x never
        e[i] = !valid ? B - x : ((lmask >> i) & 1u) ? kFin + (x - A) : B - t;
    }
    if (bad)
        L.ctl[C_REFUSE] = 1;
    // pointer table slice (8 x u16 = 16 B, 16-aligned)
    {
        uint4 w;
        w.x = e[0] | (e[1] << 16);
        w.y = e[2] | (e[3] << 16);
        w.z = e[4] | (e[5] << 16);
        w.w = e[6] | (e[7] << 16);
        *(uint4*)&L.ring[(tabb + 2 * o) & 0xFFFFu] = w;
    }
    if (lmask) {
        uint2* const slot = (uint2*)&L.ring[x0 & 0xFFFFu];
        uint2 w = *slot;
        uint32_t m0 = 0, m1 = 0;
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) {
            m0 |= (lmask >> i) & 1u ? 0xFFu << (8 * i) : 0u;
            m1 |= (lmask >> (i + 4)) & 1u ? 0xFFu << (8 * i) : 0u;
        }
        w.x = (w.x & ~m0) | (lv0 & m0);
        w.y = (w.y & ~m1) | (lv1 & m1);
        *slot = w;
    }
    // op covering Ew; the next window's op starts
    uint32_t nx = iS + total;
    if (nx + 1 < nops && L.opp[nx + 1] <= Ew)
        nx++;
    nx = uni(nx);
    if (next_same)
        scatter_starts(L, L.bmap[cur ^ 1u], Ew & ~15u, nx, nops);
    __syncthreads();
    STAMP(6);
    if (L.ctl[C_REFUSE])
        return false;
    // this window's bitmap is read: clear it for the window after next
    if (tid < kW / 32)
        bm[tid] = 0;

    // chase in-window sources (pointer table shared, written back as we go;
    // relaxed LDS atomics: another lane's entry is read as it is, old or new,
    // and every value ever stored there is a valid source for its byte)
    {
        uint32_t* const t32 = (uint32_t*)L.ring;
        const uint32_t myw = ((tabb + 2 * o) & 0xFFFFu) >> 2;
        bool any = true;
        while (__ballot(any) != 0ull) {
            any = false;
            uint32_t w8[8];
#pragma unroll
            for (uint32_t i = 0; i < 8; i++) {            // unconditional loads, one wait
                const uint32_t x = x0 + i;
                const bool pend = x >= S && x < Ew && e[i] <= T;
                const uint32_t byteoff = (tabb + 2 * (kW - 1 - (pend ? e[i] : 0u))) & 0xFFFFu;
                w8[i] = __hip_atomic_load(&t32[byteoff >> 2], __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP) >> (8 * (byteoff & 2));
            }
#pragma unroll
            for (uint32_t i = 0; i < 8; i++) {
                const uint32_t x = x0 + i;
                const bool pend = x >= S && x < Ew && e[i] <= T;
                e[i] = pend ? w8[i] & 0xFFFFu : e[i];
                any |= pend && e[i] <= T;
            }
            COUNT(11, 1);
#pragma unroll
            for (uint32_t q = 0; q < 4; q++)
                __hip_atomic_store(&t32[myw + q], e[2 * q] | (e[2 * q + 1] << 16), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    STAMP(7);

    // gather (no barrier after the chase: a lane's final sources are literal
    // bytes, written before the barrier above, or bytes before S; the ring
    // bytes written below are never a final source of this window)
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (uint32_t i = 0; i < 8; i++) {
        const uint32_t x = x0 + i;
        const bool valid = x >= S && x < Ew;
        const uint32_t y = !valid ? x : e[i] >= kFin ? A + (e[i] - kFin) : B - e[i];
        const uint32_t v = L.ring[y & 0xFFFFu];
        if (i < 4)
            lo |= v << (8 * i);
        else
            hi |= v << (8 * (i - 4));
    }
    *(uint2*)&L.ring[x0 & 0xFFFFu] = make_uint2(lo, hi);
    if (x0 >= S && x0 + 8 <= Ew) {
        *(uint2*)(blk.out + x0) = make_uint2(lo, hi);
    } else {
#pragma unroll
        for (uint32_t i = 0; i < 8; i++) {
            const uint32_t x = x0 + i;
            if (x >= S && x < Ew)
                blk.out[x] = (uint8_t)((i < 4 ? lo >> (8 * i) : hi >> (8 * (i - 4))) & 0xFFu);
        }
    }
    iS = nx;
    cur ^= 1u;
    prepped = next_same;
    COUNT(9, 1);
    __syncthreads();          // ring bytes final; every chase done before the next table
    STAMP(8);
    return true;
}

__device__ void close_block(uint32_t b, bool ok, uint32_t len, uint32_t* out_len, int32_t* status,
                            uint32_t* fallback, uint32_t* fallback_ids)
{
    if (threadIdx.x != 0)
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

template <bool STAMPS>
__global__ __launch_bounds__(kNT, 4) void lzo1x_decode_win_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ src_len, uint8_t* __restrict__ dst,
    const uint64_t* __restrict__ dst_off, const uint32_t* __restrict__ dst_cap,
    uint32_t* __restrict__ out_len, int32_t* __restrict__ status,
    uint32_t* __restrict__ fallback, uint32_t* __restrict__ fallback_ids, uint32_t nblocks,
    uint64_t* __restrict__ dbg)
{
    __shared__ WinLds L;
    if (STAMPS && threadIdx.x < 16)
        L.stamp[threadIdx.x] = threadIdx.x == 15 ? clock64() : 0;
    const uint32_t b = blockIdx.x;
    if (b >= nblocks)
        return;
    const uint32_t tid = threadIdx.x;
    Blk blk;
    blk.in = src + src_off[b];
    blk.z = src_len[b];
    blk.out = dst + dst_off[b];
    blk.cap = dst_cap[b];
    // the exact decoder takes: empty or huge inputs, destinations not 8-aligned
    if (blk.z == 0 || blk.z >= (1u << 24) || ((uintptr_t)blk.out & 7u)) {
        close_block(b, false, 0, out_len, status, fallback, fallback_ids);
        return;
    }
    if (tid < kW / 32) {
        L.bmap[0][tid] = 0;
        L.bmap[1][tid] = 0;
    }
    if (tid == 0)
        L.ctl[C_REFUSE] = 0;
    __syncthreads();

    uint32_t I = 0, st = ST_F, E = 0, S = 0, iS = 0, nops = 0, cur = 0;
    bool ok = true;
    for (uint32_t k = 0;; k++) {
        // carry the ops that still cover [S, E) to the front of the table
        if (k) {
            const uint32_t keep = nops - iS;      // ops iS .. nops-1, plus the sentinel
            uint32_t v0 = 0, s0 = 0, v1 = 0, s1 = 0;
            if (tid <= keep) {
                v0 = L.opp[iS + tid];
                s0 = tid < keep ? L.ops[iS + tid] : 0u;
            }
            if (tid + kNT <= keep) {
                v1 = L.opp[iS + tid + kNT];
                s1 = tid + kNT < keep ? L.ops[iS + tid + kNT] : 0u;
            }
            __syncthreads();
            if (tid <= keep) {
                L.opp[tid] = v0;
                L.ops[tid] = s0;
            }
            if (tid + kNT <= keep) {
                L.opp[tid + kNT] = v1;
                L.ops[tid + kNT] = s1;
            }
            nops = keep;
            iS = 0;
        }
        const uint32_t Pk = E;
        const PieceOut r = parse_piece<STAMPS>(L, blk, I, st, nops, E, k & 1u);
        if (r.result == PR_REFUSE || r.E > blk.cap) {
            ok = false;
            break;
        }
        I = r.I;
        st = r.st;
        nops = r.nops;
        E = r.E;
        const bool eof = r.result == PR_EOF;
        auto full_next = [&](uint32_t s2) { return s2 < E && ((s2 & ~15u) + kW <= E || eof); };
        bool prepped = false;
        while (full_next(S)) {
            const uint32_t Ew = (S & ~15u) + kW < E ? (S & ~15u) + kW : E;
            if (!run_window<STAMPS>(L, blk, S, Ew, iS, nops, cur, prepped, full_next(Ew))) {
                ok = false;
                break;
            }
            S = Ew;
        }
        if (!ok)
            break;
        if (eof)
            break;
        if (S < E && (S < Pk || r.result == PR_FULL)) {
            bool prepped2 = false;
            if (!run_window<STAMPS>(L, blk, S, E, iS, nops, cur, prepped2, false)) {
                ok = false;
                break;
            }
            S = E;
        }
    }
    close_block(b, ok, E, out_len, status, fallback, fallback_ids);
    if (STAMPS && tid == 0)
        for (int i = 0; i < 16; i++)
            dbg[(size_t)b * 16 + i] = L.stamp[i];
}

}  // namespace

extern "C" int lzo_mi355x_launch_decompress_win(const uint8_t* src, const uint64_t* src_off,
                                                const uint32_t* src_len, uint8_t* dst,
                                                const uint64_t* dst_off, const uint32_t* dst_cap,
                                                uint32_t* out_len, int32_t* status,
                                                uint32_t* fallback, uint32_t* fallback_ids,
                                                uint32_t nblocks, hipStream_t stream)
{
    if (nblocks == 0)
        return 0;
    hipLaunchKernelGGL(lzo1x_decode_win_kernel<false>, dim3(nblocks), dim3(kNT), 0, stream, src,
                       src_off, src_len, dst, dst_off, dst_cap, out_len, status, fallback,
                       fallback_ids, nblocks, nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Diagnostic: the same decoder with per-phase cycle stamps (16 x u64 per block,
// thread 0's view): 0 stage, 1 speculative walks, 2 settle, 3 count + scan,
// 4 emit, 5 window op bitmap, 6 pointers, 7 chase, 8 gather + stores;
// counts: 9 windows, 10 pieces, 11 chase rounds (wave 0), 12 settle rounds (wave 0).
extern "C" int lzo_mi355x_debug_decompress_win_stamps(const uint8_t* src, const uint64_t* src_off,
                                                      const uint32_t* src_len, uint8_t* dst,
                                                      const uint64_t* dst_off, const uint32_t* dst_cap,
                                                      uint32_t* out_len, int32_t* status,
                                                      uint32_t* fallback, uint32_t* fallback_ids,
                                                      uint32_t nblocks, uint64_t* stamps,
                                                      hipStream_t stream)
{
    if (nblocks == 0)
        return 0;
    hipLaunchKernelGGL(lzo1x_decode_win_kernel<true>, dim3(nblocks), dim3(kNT), 0, stream, src,
                       src_off, src_len, dst, dst_off, dst_cap, out_len, status, fallback,
                       fallback_ids, nblocks, stamps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
