// lzo1x_decode_lat.hip -- the latency decoder for MI355X (gfx950): one block,
// or up to 8 side by side, decoded by the whole GPU as a pipeline of
// data-parallel kernels, with no per-window chain.  For single
// calls and small batches of ITBs up to 536,192 B (include/xtable.h:136-144),
// where every throughput decoder is one workgroup's serial chain.  With
// several blocks every kernel runs over the flattened node and output spaces;
// jumps, marks and origins never leave a block (END and BAD absorb, look-behind
// is checked), and each element finds its block in the kernel argument.
//
// Grammar: lib/minilzo.c:3308-3699.  Stages:
//  1. NODES: every (position, state class) of the compressed stream -- class
//     A (top of the loop: t < 16 is a literal run) or N (after literals: t < 16
//     is an M1 match) -- gets the node of the instruction that follows it,
//     one thread per node (node 0 is the first byte, state F; END and BAD are
//     absorbing: EOF exactly at the input's end, or a refused instruction).
//  2. PATH: pointer doubling (levels J_k = J_{k-1} o J_{k-1}), then marking
//     from node 0 down the levels: the marked nodes are the block's
//     instructions, in node order = stream order.
//  3. FIELDS: each instruction's exact state (B or C decides an M1's length
//     and distance) is its predecessor's next state, found by a running
//     maximum of marked node ids; it is decoded again with it, and a running
//     sum of output lengths gives every instruction's output position.  The
//     capacity, look-behind and end checks hand the block to the exact
//     decoder (fallback list) exactly as the other decoders do.
//  4. ORIGINS: output byte p is covered by the instruction whose start is the
//     running maximum of starts at p; its origin is an input position (a
//     literal) or p - d (a match byte).
//  5. DOUBLING: origin[p] = origin applied 8 times, until every origin is a
//     literal (chains on ITB blocks are at most ~600 hops: <= 4 rounds; a
//     round that finds nothing left ends the rest early).
//  6. GATHER: out[p] = in[origin[p]].
// Every stage is a plain grid over nodes or output bytes; the scans are
// two-level (tiles of 4096, then the tile totals).
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "lzo_mi355x_kernels.h"

namespace {

constexpr uint32_t ST_A = 0, ST_B = 1, ST_C = 2, ST_F = 3;
constexpr uint32_t kLitO = 0x80000000u;          // origin: an input position
constexpr int32_t kFallback = 0x7FFF0001;
constexpr uint32_t kT = 256;                     // threads per workgroup (grids)
constexpr uint32_t kScanT = 1024;                // scan tile: kScanT threads x 4
constexpr uint32_t kTile = 4 * kScanT;
constexpr uint32_t kMaxTiles = kTile;            // one tile of tile totals
constexpr uint32_t kRounds = 24;                 // doubling rounds at most (chains < 2^24)

// control words in scratch
constexpr uint32_t kMaxBlk = 8;                  // blocks one pipeline decodes side by side
// control words in scratch: C_ROUND + r: round r found work; per block b:
// C_BADB + b handed over, C_TOTB + b output length, C_BASEB + b output sum
// before its first node
enum { C_ROUND = 0, C_BADB = 24, C_TOTB = C_BADB + 8, C_BASEB = C_TOTB + 8, C_WORDS = C_BASEB + 8 };
static_assert(C_BADB >= 24 && kMaxBlk == 8, "control layout");

// The blocks of one pipeline (kernel argument): node ids no .. no + 2z + 2
// (0 the first byte in state F, 1 + 2i + c position i class c, 2z + 1 END,
// 2z + 2 BAD), output slots oo .. oo + cap of the flattened output space,
// input and output at src + in_off, dst + out_off.
struct BlkMeta {
    uint32_t no, z, oo, cap;
    uint64_t in_off, out_off;
};
struct Blks {
    uint32_t nb, N, C, pad;
    BlkMeta m[kMaxBlk];
};

__device__ __forceinline__ uint32_t blk_of_node(const Blks& B, uint32_t id)
{
    uint32_t b = 0;
    for (uint32_t i = 1; i < B.nb; i++)
        b = id >= B.m[i].no ? i : b;
    return b;
}

__device__ __forceinline__ uint32_t blk_of_out(const Blks& B, uint32_t p)
{
    uint32_t b = 0;
    for (uint32_t i = 1; i < B.nb; i++)
        b = p >= B.m[i].oo ? i : b;
    return b;
}

struct Ins {
    uint32_t L, d, lit, lsrc, next, nst, kind;   // kind: 0 ok, 1 EOF exactly at z, 2 refuse
};

__device__ __forceinline__ uint32_t ib(const uint8_t* in, uint32_t z, uint32_t q)
{
    return q < z ? (uint32_t)in[q] : 0u;
}

// One instruction at p in state s (lib/minilzo.c:3357-3414 literal runs,
// 3418-3443 / 3588-3613 M1, 3447-3498 M2, 3500-3537 M3, 3538-3587 M4 / EOF,
// 3650-3667 trailing literals).
__device__ Ins decode_at(const uint8_t* in, uint32_t z, uint32_t p, uint32_t s)
{
    Ins x{0, 0, 0, 0, 0, ST_A, 2};
    uint32_t q = p;
    if (q >= z)
        return x;
    const uint32_t t = ib(in, z, q++);
    // A length extension: zero bytes count 255 each.  Every node of a zero run
    // would scan the rest of the run, so a node gives up after kExtMax zero
    // bytes (a length past ~16 K): refused here, the block goes to the exact
    // decoder, which decodes such a stream in linear time.
    constexpr uint32_t kExtMax = 64;
    auto ext = [&](uint32_t base, uint32_t& n) -> bool {
        uint32_t v = 0;
        for (;;) {
            if (q >= z || v >= kExtMax * 255u)
                return false;
            const uint32_t b = ib(in, z, q++);
            if (b) {
                n = v + base + b;
                return true;
            }
            v += 255;
        }
    };
    if (s == ST_F) {
        if (t > 17) {
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
        if (s == ST_A) {
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
        const uint32_t b1 = ib(in, z, q++);
        x.L = s == ST_B ? 3u : 2u;
        x.d = (s == ST_B ? 0x801u : 1u) + (t >> 2) + (b1 << 2);
        w = t;
    } else if (t >= 64) {
        const uint32_t b1 = ib(in, z, q++);
        x.L = (t >> 5) + 1;
        x.d = 1 + ((t >> 2) & 7) + (b1 << 3);
        w = t;
    } else if (t >= 32) {
        uint32_t n = t & 31;
        if (n == 0 && !ext(31, n))
            return x;
        x.L = n + 2;
        w = ib(in, z, q) | (ib(in, z, q + 1) << 8);
        q += 2;
        x.d = 1 + (w >> 2);
    } else {
        uint32_t n = t & 7;
        if (n == 0 && !ext(7, n))
            return x;
        x.L = n + 2;
        w = ib(in, z, q) | (ib(in, z, q + 1) << 8);
        q += 2;
        const uint32_t dd = ((t & 8) << 11) + (w >> 2);
        if (dd == 0) {
            x.L = 0;
            x.next = q;
            x.kind = q == z ? 1 : 2;
            return x;
        }
        x.d = dd + 0x4000;
    }
    const uint32_t T = w & 3;
    x.lit = T;
    x.lsrc = q;
    x.next = q + T;
    x.nst = T ? ST_C : ST_A;
    x.kind = x.next < z ? 0 : 2;
    return x;
}

__device__ __forceinline__ uint32_t umax32(uint32_t a, uint32_t b) { return a > b ? a : b; }

// node ids: 0 = position 0 in state F; 1 + 2i + c = position i, class c (0 A,
// 1 B/C); END = 2z + 1; BAD = 2z + 2
__device__ __forceinline__ void node_pos(uint32_t id, uint32_t& p, uint32_t& s)
{
    p = id ? (id - 1) >> 1 : 0u;
    s = id ? (((id - 1) & 1u) ? ST_B : ST_A) : ST_F;
}

__global__ __launch_bounds__(kT) void lat_nodes(const uint8_t* __restrict__ src, const Blks B, uint32_t* __restrict__ J0,
                                                uint32_t* __restrict__ nst, uint32_t* __restrict__ mark,
                                                uint32_t* __restrict__ ctl, uint32_t* __restrict__ cover)
{
    const uint32_t g = blockIdx.x * kT + threadIdx.x, step = gridDim.x * kT;
    if (g < C_WORDS)
        ctl[g] = 0;
    for (uint32_t p = g; p < B.C; p += step)
        cover[p] = 0;
    for (uint32_t id = g; id < B.N; id += step) {
        const uint32_t b = blk_of_node(B, id), no = B.m[b].no, z = B.m[b].z, l = id - no;
        uint32_t j = id, ns = ST_A;
        if (l < 2 * z + 1) {
            uint32_t p, s;
            node_pos(l, p, s);
            const Ins x = decode_at(src + B.m[b].in_off, z, p, s);
            j = no + (x.kind == 2 ? 2 * z + 2 : x.kind == 1 ? 2 * z + 1 : 1 + 2 * x.next + (x.nst != ST_A ? 1u : 0u));
            ns = x.nst;
        }
        J0[id] = j;
        nst[id] = ns;
        mark[id] = l == 0 ? 1u : 0u;
    }
}

// levels k + 1 .. k + nl (nl <= 3) from level k: J_{k+i} = J_k applied 2^i
// times (one launch per three levels: launches, not work, bound this path)
__global__ __launch_bounds__(kT) void lat_jump(const uint32_t* __restrict__ Jk, uint32_t* __restrict__ Jn, uint32_t N,
                                               uint32_t nl)
{
    for (uint32_t id = blockIdx.x * kT + threadIdx.x; id < N; id += gridDim.x * kT) {
        uint32_t x = Jk[Jk[id]];
        Jn[id] = x;
        if (nl > 1) {
            x = Jk[Jk[x]];
            Jn[(size_t)N + id] = x;
        }
        if (nl > 2) {
            x = Jk[Jk[Jk[Jk[x]]]];
            Jn[2 * (size_t)N + id] = x;
        }
    }
}

// levels k, k - 1, k - 2 (nl of them, from the top): every node reached from a
// marked node by any combination of those jumps is marked (marks made in the
// same pass may propagate further: still nodes of the path)
__global__ __launch_bounds__(kT) void lat_mark(const uint32_t* __restrict__ J, uint32_t* mark, uint32_t N, uint32_t k,
                                               uint32_t nl)
{
    const uint32_t* J0 = J + (size_t)k * N;
    const uint32_t* J1 = J0 - (nl > 1 ? N : 0);
    const uint32_t* J2 = J1 - (nl > 2 ? N : 0);
    auto set = [&](uint32_t x) { __hip_atomic_store(mark + x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    for (uint32_t id = blockIdx.x * kT + threadIdx.x; id < N; id += gridDim.x * kT) {
        if (!__hip_atomic_load(mark + id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            continue;
        const uint32_t a = J0[id];
        set(a);
        if (nl > 1) {
            const uint32_t b = J1[id], c = J1[a];
            set(b);
            set(c);
            if (nl > 2) {
                set(J2[id]);
                set(J2[a]);
                set(J2[b]);
                set(J2[c]);
            }
        }
    }
}

// running-maximum input: the id of every instruction node, 0 elsewhere; a
// block whose path ends anywhere but its END is handed over
__global__ __launch_bounds__(kT) void lat_pred_in(const Blks B, const uint32_t* __restrict__ mark,
                                                  uint32_t* __restrict__ v, uint32_t* __restrict__ ctl)
{
    const uint32_t g = blockIdx.x * kT + threadIdx.x;
    for (uint32_t id = g; id < B.N; id += gridDim.x * kT) {
        const uint32_t b = blk_of_node(B, id);
        v[id] = (id - B.m[b].no < 2 * B.m[b].z + 1 && mark[id]) ? id : 0u;
    }
    if (g < B.nb) {
        const uint32_t e = B.m[g].no + 2 * B.m[g].z + 1;
        if (mark[e + 1] || !mark[e])
            ctl[C_BADB + g] = 1;
    }
}

// exact state, fields and output length of every instruction node
__global__ __launch_bounds__(kT) void lat_fields(const uint8_t* __restrict__ src, const Blks B,
                                                 const uint32_t* __restrict__ mark, const uint32_t* __restrict__ pmax,
                                                 const uint32_t* __restrict__ nst, uint4* __restrict__ fld,
                                                 uint32_t* __restrict__ tot, uint32_t* __restrict__ ctl)
{
    for (uint32_t id = blockIdx.x * kT + threadIdx.x; id < B.N; id += gridDim.x * kT) {
        const uint32_t b = blk_of_node(B, id), z = B.m[b].z, l = id - B.m[b].no;
        uint32_t n = 0;
        if (l < 2 * z + 1 && mark[id]) {
            uint32_t p, s;
            node_pos(l, p, s);
            if (l != 0)
                s = nst[pmax[id - 1]];           // the predecessor's next state
            const Ins x = decode_at(src + B.m[b].in_off, z, p, s);
            const bool cls_a = ((l - 1) & 1u) == 0u;
            if (x.kind == 2 || (l != 0 && (s == ST_A) != cls_a))
                ctl[C_BADB + b] = 1;             // (a path is consistent by construction)
            fld[id] = make_uint4(x.L, x.d, x.lit, x.lsrc);
            n = x.L + x.lit;
        }
        tot[id] = n;
    }
}

// checks (capacity, look-behind), each block's length, and the start marker
// of every instruction
__global__ __launch_bounds__(kT) void lat_starts(const Blks B, const uint32_t* __restrict__ mark,
                                                 const uint4* __restrict__ fld, const uint32_t* __restrict__ tot,
                                                 const uint32_t* __restrict__ osum, uint32_t* __restrict__ cover,
                                                 uint32_t* __restrict__ ctl)
{
    const uint32_t g = blockIdx.x * kT + threadIdx.x;
    if (g < B.nb) {
        const uint32_t no = B.m[g].no, base = osum[no] - tot[no];
        const uint32_t total = osum[no + 2 * B.m[g].z + 2] - base;
        ctl[C_TOTB + g] = total;
        ctl[C_BASEB + g] = base;
        if (total > B.m[g].cap)
            ctl[C_BADB + g] = 1;
    }
    for (uint32_t id = g; id < B.N; id += gridDim.x * kT) {
        const uint32_t b = blk_of_node(B, id), no = B.m[b].no;
        if (id - no < 2 * B.m[b].z + 1 && mark[id] && tot[id]) {
            const uint32_t o = osum[id] - tot[id] - (osum[no] - tot[no]);   // output position
            const uint4 f = fld[id];
            if (f.x && f.y > o)
                ctl[C_BADB + b] = 1;             // look-behind (lib/minilzo.c TEST_LB)
            if (o < B.m[b].cap)
                cover[B.m[b].oo + o] = id;
        }
    }
}

__global__ __launch_bounds__(kT) void lat_origins(const Blks B, const uint32_t* __restrict__ cover,
                                                  const uint32_t* __restrict__ tiles, const uint4* __restrict__ fld,
                                                  const uint32_t* __restrict__ tot, const uint32_t* __restrict__ osum,
                                                  uint32_t* __restrict__ org, const uint32_t* __restrict__ ctl)
{
    for (uint32_t p = blockIdx.x * kT + threadIdx.x; p < B.C; p += gridDim.x * kT) {
        const uint32_t b = blk_of_out(B, p), pl = p - B.m[b].oo;
        if (ctl[C_BADB + b] || pl >= ctl[C_TOTB + b]) {
            org[p] = kLitO;                      // (outside every block's output: never gathered)
            continue;
        }
        uint32_t id = cover[p];
        if (p >= kTile)
            id = umax32(tiles[p / kTile], id);   // (the cover scan's add pass)
        const uint4 f = fld[id];
        const uint32_t o = osum[id] - tot[id] - ctl[C_BASEB + b];
        const uint32_t r = pl - o;
        org[p] = r < f.x ? p - f.y : kLitO | (uint32_t)(B.m[b].in_off + f.w + (r - f.x));
    }
}

// one doubling round, in place (a partly updated source only shortens the
// chain); a round after one that found nothing left returns at once
__global__ __launch_bounds__(kT) void lat_double(uint32_t* org, uint32_t C, uint32_t* __restrict__ ctl, uint32_t r)
{
    if (r > 0 && ctl[C_ROUND + r - 1] == 0)
        return;
    bool left = false;
    for (uint32_t p = blockIdx.x * kT + threadIdx.x; p < C; p += gridDim.x * kT) {
        uint32_t o = __hip_atomic_load(org + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!(o & kLitO)) {
            // seven dereferences a pass: a chain shrinks 8x per launch
#pragma unroll
            for (int i = 0; i < 7; i++)
                if (!(o & kLitO))
                    o = __hip_atomic_load(org + o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(org + p, o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            left = left || !(o & kLitO);
        }
    }
    if (__any(left) && (threadIdx.x & 63u) == 0)
        ctl[C_ROUND + r] = 1;
}

__global__ __launch_bounds__(kT) void lat_gather(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, const Blks B,
                                                 const uint32_t* __restrict__ org, const uint32_t* __restrict__ ctl,
                                                 uint32_t* __restrict__ out_len, int32_t* __restrict__ status,
                                                 uint32_t* __restrict__ fallback, uint32_t* __restrict__ fallback_ids,
                                                 uint32_t b0, uint32_t rounds)
{
    const bool stuck = ctl[C_ROUND + rounds - 1] != 0;   // (chains longer than the rounds: never on valid data)
    const uint32_t g = blockIdx.x * kT + threadIdx.x;
    if (g < B.nb) {
        const uint32_t b = b0 + g;
        if (ctl[C_BADB + g] || stuck) {
            out_len[b] = 0xFA110000u;
            status[b] = kFallback;
            fallback_ids[atomicAdd(&fallback[0], 1u)] = b;
        } else {
            out_len[b] = ctl[C_TOTB + g];
            status[b] = 0;
        }
    }
    if (stuck)
        return;
    for (uint32_t p = g; p < B.C; p += gridDim.x * kT) {
        const uint32_t b = blk_of_out(B, p), pl = p - B.m[b].oo;
        if (!ctl[C_BADB + b] && pl < ctl[C_TOTB + b])
            dst[B.m[b].out_off + pl] = src[org[p] & ~kLitO];
    }
}

// ---- scans (inclusive; MAX = running maximum, else running sum) -------------
template <bool MAX>
__device__ __forceinline__ uint32_t op2(uint32_t a, uint32_t b)
{
    return MAX ? (a > b ? a : b) : a + b;
}

template <bool MAX>
__device__ uint32_t block_scan(uint32_t v, uint32_t* sh)
{
    // inclusive scan of one value per thread over kScanT threads
    const uint32_t t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (uint32_t o = 1; o < kScanT; o <<= 1) {
        const uint32_t a = t >= o ? sh[t - o] : (MAX ? 0u : 0u);
        __syncthreads();
        sh[t] = op2<MAX>(sh[t], a);
        __syncthreads();
    }
    return sh[t];
}

template <bool MAX>
__global__ __launch_bounds__(kScanT) void scan_tiles(const uint32_t* in, uint32_t* out,   // (in == out: in-place scans)
                                                     uint32_t n, uint32_t* __restrict__ tiles)
{
    __shared__ uint32_t sh[kScanT];
    const uint32_t base = blockIdx.x * kTile + 4 * threadIdx.x;
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; j++)
        v[j] = base + j < n ? in[base + j] : 0u;
    v[1] = op2<MAX>(v[0], v[1]);
    v[2] = op2<MAX>(v[1], v[2]);
    v[3] = op2<MAX>(v[2], v[3]);
    const uint32_t inc = block_scan<MAX>(v[3], sh);
    const uint32_t pre = threadIdx.x ? sh[threadIdx.x - 1] : 0u;
    (void)inc;
#pragma unroll
    for (int j = 0; j < 4; j++)
        if (base + j < n)
            out[base + j] = op2<MAX>(pre, v[j]);
    if (threadIdx.x == kScanT - 1)
        tiles[blockIdx.x] = sh[kScanT - 1];
}

template <bool MAX>
__global__ __launch_bounds__(kScanT) void scan_tile_totals(uint32_t* tiles, uint32_t ntiles)
{
    // exclusive scan of the tile totals in place (ntiles <= kMaxTiles)
    __shared__ uint32_t sh[kScanT];
    const uint32_t base = 4 * threadIdx.x;
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; j++)
        v[j] = base + j < ntiles ? tiles[base + j] : 0u;
    uint32_t s[4];
    s[0] = v[0];
    s[1] = op2<MAX>(s[0], v[1]);
    s[2] = op2<MAX>(s[1], v[2]);
    s[3] = op2<MAX>(s[2], v[3]);
    block_scan<MAX>(s[3], sh);
    const uint32_t pre = threadIdx.x ? sh[threadIdx.x - 1] : 0u;
    const uint32_t ex[4] = {pre, op2<MAX>(pre, s[0]), op2<MAX>(pre, s[1]), op2<MAX>(pre, s[2])};
#pragma unroll
    for (int j = 0; j < 4; j++)
        if (base + j < ntiles)
            tiles[base + j] = ex[j];
}

template <bool MAX>
__global__ __launch_bounds__(kT) void scan_add(uint32_t* out, uint32_t n, const uint32_t* __restrict__ tiles)
{
    for (uint32_t i = blockIdx.x * kT + threadIdx.x; i < n; i += gridDim.x * kT)
        if (i >= kTile)
            out[i] = op2<MAX>(tiles[i / kTile], out[i]);
}

// add = false: the tiles are scanned and their exclusive prefixes left in
// tiles[] for the consumer to apply (element i: op(tiles[i / kTile], out[i])
// from the second tile on)
template <bool MAX>
int scan(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* tiles, uint32_t grid, hipStream_t s,
         bool add = true)
{
    const uint32_t nt = (n + kTile - 1) / kTile;
    if (nt > kMaxTiles)
        return -1;
    hipLaunchKernelGGL(scan_tiles<MAX>, dim3(nt), dim3(kScanT), 0, s, in, out, n, tiles);
    if (nt > 1) {
        hipLaunchKernelGGL(scan_tile_totals<MAX>, dim3(1), dim3(kScanT), 0, s, tiles, nt);
        if (add)
            hipLaunchKernelGGL(scan_add<MAX>, dim3(grid), dim3(kT), 0, s, out, n, (const uint32_t*)tiles);
    }
    return 0;
}

uint32_t levels_for(uint32_t z)
{
    // the path has at most z + 1 instructions: 2^K > z + 2
    uint32_t k = 1;
    while ((1ull << k) <= (uint64_t)z + 2)
        k++;
    return k;
}

struct Lay {
    size_t J, nst, mark, v, pmax, fld, tot, osum, tiles, ctl, cover, org, end;
};

Lay layout(uint64_t N, uint64_t C, uint32_t K)
{
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    Lay L;
    size_t o = 0;
    L.J = o;     o = up(o + K * N * 4);
    L.nst = o;   o = up(o + N * 4);
    L.mark = o;  o = up(o + N * 4);
    L.v = o;     o = up(o + N * 4);
    L.pmax = o;  o = up(o + N * 4);
    L.fld = o;   o = up(o + N * 16);
    L.tot = o;   o = up(o + N * 4);
    L.osum = o;  o = up(o + N * 4);
    L.tiles = o; o = up(o + (size_t)kMaxTiles * 4);
    L.ctl = o;   o = up(o + C_WORDS * 4);
    L.cover = o; o = up(o + C * 4);
    L.org = o;   o = up(o + C * 4);
    L.end = o;
    return L;
}

// N, C and K of nb blocks, or false outside the decoder's range
bool shape(const uint64_t* src_off, const uint32_t* z, const uint32_t* cap, uint32_t nb, uint64_t& N,
           uint64_t& C, uint32_t& K)
{
    const uint64_t lim = (uint64_t)kMaxTiles * kTile;   // elements one two-level scan takes
    if (nb == 0 || nb > kMaxBlk)
        return false;
    N = C = 0;
    uint32_t zmax = 0;
    for (uint32_t b = 0; b < nb; b++) {
        if (z[b] == 0 || cap[b] == 0 || src_off[b] + z[b] >= (1ull << 31))
            return false;
        N += 2 * (uint64_t)z[b] + 3;
        C += cap[b];
        zmax = z[b] > zmax ? z[b] : zmax;
    }
    K = levels_for(zmax);
    return N <= lim && C <= lim;
}

}  // namespace

// Scratch for nb <= 8 blocks decoded by one pipeline (host arrays); 0 when
// they are outside the decoder's range (an empty input or room, more than 8
// blocks, more than 16 Mi nodes or output slots).
extern "C" size_t lzo_mi355x_decompress_lat_scratch_n(const uint64_t* src_off, const uint32_t* z,
                                                      const uint32_t* cap, uint32_t nb)
{
    uint64_t N, C;
    uint32_t K;
    return shape(src_off, z, cap, nb, N, C, K) ? layout(N, C, K).end : 0;
}

extern "C" size_t lzo_mi355x_decompress_lat_scratch(uint32_t z, uint32_t cap)
{
    const uint64_t off = 0;
    return lzo_mi355x_decompress_lat_scratch_n(&off, &z, &cap, 1);
}

// nb <= 8 blocks side by side: block b's z[b] bytes at src + src_off[b] into
// dst + dst_off[b] (capacity cap[b]); out_len / status / fallback entries at
// b0 + b (host arrays; src_off[b] + z[b] < 2^31).
extern "C" int lzo_mi355x_launch_decompress_lat_n(const uint8_t* src, const uint64_t* src_off, const uint32_t* z,
                                                  uint8_t* dst, const uint64_t* dst_off, const uint32_t* cap,
                                                  uint32_t nb, uint32_t* out_len, int32_t* status,
                                                  uint32_t* fallback, uint32_t* fallback_ids, uint32_t b0,
                                                  void* scratch, size_t scratch_bytes, hipStream_t s)
{
    uint64_t N64, C64;
    uint32_t K;
    if (!shape(src_off, z, cap, nb, N64, C64, K))
        return -1;
    const Lay L = layout(N64, C64, K);
    if (L.end > scratch_bytes)
        return -1;
    const uint32_t N = (uint32_t)N64, C = (uint32_t)C64;
    Blks B{};
    B.nb = nb;
    B.N = N;
    B.C = C;
    uint32_t no = 0, oo = 0;
    for (uint32_t b = 0; b < nb; b++) {
        B.m[b] = BlkMeta{no, z[b], oo, cap[b], src_off[b], dst_off[b]};
        no += 2 * z[b] + 3;
        oo += cap[b];
    }
    uint8_t* S = (uint8_t*)scratch;
    uint32_t* J = (uint32_t*)(S + L.J);
    uint32_t* nst = (uint32_t*)(S + L.nst);
    uint32_t* mark = (uint32_t*)(S + L.mark);
    uint32_t* v = (uint32_t*)(S + L.v);
    uint32_t* pmax = (uint32_t*)(S + L.pmax);
    uint4* fld = (uint4*)(S + L.fld);
    uint32_t* tot = (uint32_t*)(S + L.tot);
    uint32_t* osum = (uint32_t*)(S + L.osum);
    uint32_t* tiles = (uint32_t*)(S + L.tiles);
    uint32_t* ctl = (uint32_t*)(S + L.ctl);
    uint32_t* cover = (uint32_t*)(S + L.cover);
    uint32_t* org = (uint32_t*)(S + L.org);
    auto grid = [](uint32_t n) { uint32_t g = (n + kT - 1) / kT; return g < 1 ? 1u : (g > 4096u ? 4096u : g); };
    const uint32_t gN = grid(N), gC = grid(C);
    hipLaunchKernelGGL(lat_nodes, dim3(gN > gC ? gN : gC), dim3(kT), 0, s, src, B, J, nst, mark, ctl, cover);
    for (uint32_t k = 0; k + 1 < K; k += 3) {
        const uint32_t nl = K - 1 - k < 3 ? K - 1 - k : 3u;
        hipLaunchKernelGGL(lat_jump, dim3(gN), dim3(kT), 0, s, (const uint32_t*)(J + (size_t)k * N),
                           J + (size_t)(k + 1) * N, N, nl);
    }
    for (uint32_t top = K; top > 0;) {
        const uint32_t nl = top < 3 ? top : 3u;
        hipLaunchKernelGGL(lat_mark, dim3(gN), dim3(kT), 0, s, (const uint32_t*)J, mark, N, top - 1, nl);
        top -= nl;
    }
    hipLaunchKernelGGL(lat_pred_in, dim3(gN), dim3(kT), 0, s, B, (const uint32_t*)mark, v, ctl);
    if (scan<true>(v, pmax, N, tiles, gN, s) != 0)
        return -1;
    hipLaunchKernelGGL(lat_fields, dim3(gN), dim3(kT), 0, s, src, B, (const uint32_t*)mark, (const uint32_t*)pmax,
                       (const uint32_t*)nst, fld, tot, ctl);
    if (scan<false>(tot, osum, N, tiles, gN, s) != 0)
        return -1;
    hipLaunchKernelGGL(lat_starts, dim3(gN), dim3(kT), 0, s, B, (const uint32_t*)mark, (const uint4*)fld,
                       (const uint32_t*)tot, (const uint32_t*)osum, cover, ctl);
    if (scan<true>(cover, cover, C, tiles, gC, s, false) != 0)
        return -1;
    hipLaunchKernelGGL(lat_origins, dim3(gC), dim3(kT), 0, s, B, (const uint32_t*)cover, (const uint32_t*)tiles,
                       (const uint4*)fld, (const uint32_t*)tot, (const uint32_t*)osum, org, (const uint32_t*)ctl);
    // chains are shorter than any block's room: 8^R > the largest cap
    uint32_t cmax = 0;
    for (uint32_t b = 0; b < nb; b++)
        cmax = cap[b] > cmax ? cap[b] : cmax;
    uint32_t R = 1;
    while (R < kRounds && (1ull << (3 * R)) <= (uint64_t)cmax)
        R++;
    for (uint32_t r = 0; r < R; r++)
        hipLaunchKernelGGL(lat_double, dim3(gC), dim3(kT), 0, s, org, C, ctl, r);
    hipLaunchKernelGGL(lat_gather, dim3(gC), dim3(kT), 0, s, src, dst, B, (const uint32_t*)org, (const uint32_t*)ctl,
                       out_len, status, fallback, fallback_ids, b0, R);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// One block (the single-call path): out_len[b] / status[b] and the fallback
// list as the other decoders (0, or 0x7FFF0001 with b appended).
extern "C" int lzo_mi355x_launch_decompress_lat(const uint8_t* in, uint32_t z, uint8_t* out, uint32_t cap,
                                                uint32_t* out_len, int32_t* status, uint32_t* fallback,
                                                uint32_t* fallback_ids, uint32_t b, void* scratch,
                                                size_t scratch_bytes, hipStream_t s)
{
    const uint64_t off = 0;
    return lzo_mi355x_launch_decompress_lat_n(in, &off, &z, out, &off, &cap, 1, out_len, status, fallback,
                                              fallback_ids, b, scratch, scratch_bytes, s);
}
