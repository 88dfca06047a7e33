/*
 * win_model.c -- sequential C model of the round-3 windowed decoder
 * (lzo1x_decode_win_kernel).  Every "for lane" loop below is a parallel step of
 * the kernel; the model exists to check the algorithm (piece parse with
 * speculative segments, carried ops, window pointer chasing through the
 * e-encoding, tab-in-ring placement) against the oracle on the CPU before the
 * HIP transcription.  Not product code; test infrastructure only.
 *
 * Build: gcc -O2 -shared -fPIC -o win_model.so win_model.c
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { W = 4096, ZH = 2048, ZR = 2 * ZH, OPCAP = 1024, RING = 65536, GMAX = 64, NPLMAX = ZH / 4,
       LITBASE = RING - ZR, NT = 512 };
static uint32_t G = 16, NPL = ZH / 16, LOOK = 16;
static long st_spec_tokens, st_fix_tokens, st_rounds, st_lanes, st_div;
void win_params(uint32_t g, uint32_t look) { G = g; NPL = ZH / g; LOOK = look; st_spec_tokens = st_fix_tokens = st_rounds = st_lanes = st_div = 0; }
void win_pstats(long out[5]) { out[0] = st_spec_tokens; out[1] = st_fix_tokens; out[2] = st_rounds; out[3] = st_lanes; out[4] = st_div; }
enum { ST_A = 0, ST_B = 1, ST_C = 2, ST_F = 3 };
#define LITF 0x80000000u

typedef struct {
    const uint8_t *in; uint32_t z;
    uint8_t ring[RING];
    uint8_t zin[ZR];
    uint32_t opp[OPCAP + 1], ops[OPCAP];
    uint32_t nops;
    /* stats */
    long windows, chase_iters, pieces, flushes, walks_fix;
} M;

/* ---- token decode (mirrors decode_one of lzo1x_decode_fast.hip) ---------- */
typedef struct { uint32_t pos, st, aL, aS, bL, bS; int eof, bad, cut; } Tok;

static uint32_t zb(const M *m, uint32_t I, uint32_t pos, int *oob)
{
    /* byte at input pos from the staged piece starting at I (half h implicit) */
    if (pos >= m->z) { *oob |= 1; return 0; }
    if (pos - I >= ZH) { *oob |= 2; return 0; }
    return m->in[pos];     /* model: read the input directly; kernel reads zin */
}

static Tok decode(const M *m, uint32_t I, uint32_t pos, uint32_t st)
{
    Tok r = { 0 };
    int oob = 0;
    uint32_t t = zb(m, I, pos, &oob);
    if (st == ST_F) {
        if (t > 17) {
            uint32_t n = t - 17;
            r.aL = n; r.aS = LITF | (pos + 1);
            r.pos = pos + 1 + n; r.st = n < 4 ? ST_C : ST_B;
            goto check;
        }
        st = ST_A;
    }
    uint32_t L, d;
    if (t < 16 && st == ST_A) {
        pos++;
        if (t == 0) {
            uint32_t v = 0;
            while (zb(m, I, pos, &oob) == 0 && !oob) { v += 255; pos++; }
            t = v + 15 + zb(m, I, pos, &oob); pos++;
        }
        r.aL = t + 3; r.aS = LITF | pos; r.pos = pos + t + 3; r.st = ST_B;
        goto check;
    }
    if (t < 16) {
        d = (st == ST_B ? 0x801u : 1u) + (t >> 2) + (zb(m, I, pos + 1, &oob) << 2);
        L = st == ST_B ? 3 : 2; pos += 2;
    } else if (t >= 64) {
        d = 1 + ((t >> 2) & 7) + (zb(m, I, pos + 1, &oob) << 3);
        L = (t >> 5) + 1; pos += 2;
    } else if (t >= 32) {
        L = t & 31; pos++;
        if (L == 0) {
            uint32_t v = 0;
            while (zb(m, I, pos, &oob) == 0 && !oob) { v += 255; pos++; }
            L = v + 31 + zb(m, I, pos, &oob); pos++;
        }
        L += 2;
        d = 1 + ((zb(m, I, pos, &oob) | (zb(m, I, pos + 1, &oob) << 8)) >> 2); pos += 2;
    } else {
        uint32_t dd = (t & 8) << 11;
        L = t & 7; pos++;
        if (L == 0) {
            uint32_t v = 0;
            while (zb(m, I, pos, &oob) == 0 && !oob) { v += 255; pos++; }
            L = v + 7 + zb(m, I, pos, &oob); pos++;
        }
        L += 2;
        dd += (zb(m, I, pos, &oob) | (zb(m, I, pos + 1, &oob) << 8)) >> 2; pos += 2;
        if (dd == 0) {
            r.eof = 1; r.pos = pos; r.st = ST_A;
            if (pos != m->z) r.bad = 1;
            goto check;
        }
        d = dd + 0x4000;
    }
    r.aL = L; r.aS = d;
    {
        uint32_t tl = zb(m, I, pos - 2, &oob) & 3;
        if (tl) { r.bL = tl; r.bS = LITF | pos; pos += tl; r.st = ST_C; }
        else r.st = ST_A;
    }
    r.pos = pos;
check:
    /* the whole instruction (with its literals) must lie in [I, I+ZH) and in z */
    if (r.pos > m->z) r.bad = 1;
    else if (r.pos - I > ZH) r.cut = 1;
    if (oob & 1) r.bad = 1;
    else if (oob & 2) r.cut = 1;
    if (r.cut) r.bad = r.eof = 0;
    return r;
}

static int in_bm(const uint32_t bm[6], uint32_t a, uint32_t pos, uint32_t st)
{
    if (pos < a || pos >= a + G) return 0;
    uint32_t q = pos - a;
    return (bm[(st == ST_F ? ST_A : st) * 2 + (q >> 5)] >> (q & 31)) & 1;
}

/* ---- piece parse --------------------------------------------------------- */
/* returns: 0 ok, 1 eof reached, -1 refuse.  Appends ops to m->opp/ops from
 * index m->nops, advancing *I, *st, *E. */
static int parse_piece(M *m, uint32_t *pI, uint32_t *pst, uint32_t *pE, uint32_t half)
{
    const uint32_t I = *pI;
    /* stage */
    for (uint32_t i = 0; i < ZH; i++)
        m->zin[half * ZH + i] = (I + i < m->z) ? m->in[I + i] : 0;
    /* P1 speculative walks */
    static uint32_t bm[NPLMAX][6], xpos[NPLMAX], xst[NPLMAX], spos[NPLMAX], sst[NPLMAX];
    for (uint32_t j = 0; j < NPL; j++) {
        uint32_t a = I + G * j, b = a + G;
        uint32_t pos = j ? (a >= I + LOOK ? a - LOOK : I) : I, st = j ? ST_A : *pst;
        memset(bm[j], 0, sizeof(bm[j]));
        uint32_t restart = pos;
        st_lanes++;
        for (;;) {
            if (pos >= b) break;
            Tok t = decode(m, I, pos, st);
            if (t.bad || t.cut || t.eof) {
                if (t.cut || t.eof || j == 0) break;      /* exit here (stopping point) */
                /* impossible guess: restart one byte later */
                restart++;
                pos = restart; st = ST_A;
                memset(bm[j], 0, sizeof(bm[j]));
                continue;
            }
            st_spec_tokens++;
            if (pos >= a) { uint32_t q = pos - a; bm[j][(st == ST_F ? ST_A : st) * 2 + (q >> 5)] |= 1u << (q & 31); }
            pos = t.pos; st = t.st;
        }
        xpos[j] = spos[j] = pos; xst[j] = sst[j] = st;
        if (pos >= a && pos < b) { /* stopped inside: mark the stop point as a start */
            uint32_t q = pos - a; bm[j][(st == ST_F ? ST_A : st) * 2 + (q >> 5)] |= 1u << (q & 31); }
    }
    /* P2 fix-up (kernel round 3b): exits as keys (pos - I) << 2 | st, + 1;
     * 0 = PASS (the lane has no instruction start on the true path: its entry
     * passes over it, or is a stop point from an earlier lane).  A lane's entry
     * is the prefix maximum of the exits below it (true exits increase along
     * the lanes), so pass-through and stop chains settle in one round. */
    static uint64_t xk[NPLMAX], ok_[NPLMAX], ent_[NPLMAX];
    for (uint32_t j = 0; j < NPL; j++) {
        uint32_t a = I + G * j;
        xk[j] = (j && a >= m->z) ? 0 : ((uint64_t)(spos[j] - I) << 2 | sst[j]) + 1;
        ent_[j] = ~0ull;
    }
    int changed = 1;
    while (changed) {
        changed = 0; st_rounds++;
        memcpy(ok_, xk, sizeof(uint64_t) * NPL);           /* Jacobi */
        uint64_t run = 0;
        for (uint32_t j = 1; j < NPL; j++) {
            run = ok_[j - 1] > run ? ok_[j - 1] : run;
            if (run == ent_[j]) continue;
            ent_[j] = run;
            uint32_t a = I + G * j, b = a + G;
            uint32_t pos = I + (uint32_t)((run - 1) >> 2), st = (uint32_t)((run - 1) & 3);
            uint64_t nk;
            if (run == 0 || pos < a || pos >= b) nk = 0;              /* pass / stop propagation */
            else if (in_bm(bm[j], a, pos, st)) nk = ((uint64_t)(spos[j] - I) << 2 | sst[j]) + 1;
            else {
                m->walks_fix++;
                int landed = 0;
                for (;;) {
                    if (pos >= b) break;
                    if (in_bm(bm[j], a, pos, st)) { landed = 1; break; }
                    Tok t = decode(m, I, pos, st);
                    st_fix_tokens++;
                    if (t.bad || t.cut || t.eof) break;
                    pos = t.pos; st = t.st;
                }
                nk = landed ? ((uint64_t)(spos[j] - I) << 2 | sst[j]) + 1 : ((uint64_t)(pos - I) << 2 | st) + 1;
            }
            if (nk != xk[j]) { xk[j] = nk; changed = 1; }
        }
    }
    /* resolved exits (prefix max) for the check below */
    {
        uint64_t run = 0;
        for (uint32_t j = 0; j < NPL; j++) {
            run = xk[j] > run ? xk[j] : run;
            xpos[j] = I + (uint32_t)((run - 1) >> 2); xst[j] = (uint32_t)((run - 1) & 3);
        }
    }
    /* P3/P4: walk true paths, emit ops in lane order (sequential here) */
    uint32_t pos = I, st = *pst, E = *pE;
    int rc = 0;
    for (uint32_t j = 0; j < NPL; j++) {
        uint32_t b = I + G * (j + 1);
        uint32_t lane_ent_pos = pos;
        while (pos < b) {
            Tok t = decode(m, I, pos, st);
            if (t.cut) goto done;            /* reads past the staged piece first */
            if (t.eof) {
                if (t.bad) { fprintf(stderr, "model: eof bad at %u (z=%u) I=%u\n", t.pos, m->z, I); return -1; }
                rc = 1; pos = t.pos; goto done;
            }
            if (t.bad) { fprintf(stderr, "model: bad token at %u st %u (I=%u)\n", pos, st, I); return -1; }
            if (t.cut) goto done;
            uint32_t need = (t.aL ? 1 : 0) + (t.bL ? 1 : 0);
            if (m->nops + need > OPCAP) { rc = 2; goto done; }
            if (t.aL) {
                m->opp[m->nops] = E;
                m->ops[m->nops] = (t.aS & LITF) ? LITF | (((t.aS & ~LITF) - I + half * ZH)) : t.aS;
                m->nops++; E += t.aL;
            }
            if (t.bL) {
                m->opp[m->nops] = E;
                m->ops[m->nops] = LITF | ((t.bS & ~LITF) - I + half * ZH);
                m->nops++; E += t.bL;
            }
            pos = t.pos; st = t.st;
        }
        { /* divergence: true exit differs from the speculative one (pass-through excluded) */
            uint32_t a = I + G * j;
            if (lane_ent_pos >= a && lane_ent_pos < b && (pos != spos[j] || st != sst[j])) st_div++;
        }
        /* check the parallel exits agree with the sequential walk */
        if (pos != xpos[j] || st != xst[j]) {
            fprintf(stderr, "model: lane %u exit mismatch (%u,%u) vs (%u,%u)\n", j, pos, st, xpos[j], xst[j]);
            return -2;
        }
    }
done:
    if (pos == I && rc != 1) { fprintf(stderr, "model: no progress at %u rc %d nops %u\n", I, rc, m->nops); return -1; }
    *pI = pos; *pst = st; *pE = E;
    m->opp[m->nops] = E;
    m->pieces++;
    return rc;
}

/* ---- window execution ---------------------------------------------------- */
static uint32_t urem(uint32_t k, uint32_t d) { return k % d; }

static int run_window(M *m, uint32_t S, uint32_t E, uint32_t *iS, uint8_t *out, uint32_t cap)
{
    const uint32_t A = S & ~15u, B = A + W - 1, T = B - S;
    const uint32_t tabbase = A + W;            /* tab[i] at ring[(tabbase + 2i) & 0xFFFF] */
    uint16_t e[W];
    /* op index per byte: i_S + #starts in (S, x] */
    uint32_t o = *iS;
    for (uint32_t i = 0; i < W; i++) {
        uint32_t x = A + i;
        if (x < S || x >= E) { e[i] = (uint16_t)(B - x); continue; }
        while (o + 1 < m->nops && m->opp[o + 1] <= x) o++;
        uint32_t p = m->opp[o], src = m->ops[o];
        if (src & LITF) {
            e[i] = (uint16_t)(LITBASE + (src & ~LITF) + (x - p));
        } else {
            uint32_t d = src, k = x - p, t;
            if (d > x) { fprintf(stderr, "model: lookbehind x=%u d=%u\n", x, d); return -1; }
            /* periodic reduction to the last period before max(p, S): the
             * source stays within 49151 bytes of the window (ring-resident) */
            const uint32_t q = p > S ? p : S;
            (void)k;
            t = q - d + urem(x - q, d);
            e[i] = (uint16_t)(B - t);
        }
    }
    for (uint32_t i = 0; i < W; i++) {
        uint32_t off = (tabbase + 2 * i) & 0xFFFF;
        m->ring[off] = (uint8_t)e[i];
        m->ring[off + 1] = (uint8_t)(e[i] >> 8);
    }
    /* chase */
    for (uint32_t i = 0; i < W; i++) {
        uint32_t x = A + i;
        if (x < S || x >= E) continue;
        uint32_t v = e[i];
        while (v <= T) {
            uint32_t off = (tabbase + 2 * (W - 1 - v)) & 0xFFFF;
            v = m->ring[off] | (m->ring[off + 1] << 8);
            m->chase_iters++;
        }
        e[i] = (uint16_t)v;
        uint32_t off = (tabbase + 2 * i) & 0xFFFF;
        m->ring[off] = (uint8_t)v;
        m->ring[off + 1] = (uint8_t)(v >> 8);
    }
    /* gather */
    uint8_t val[W];
    for (uint32_t i = 0; i < W; i++) {
        uint32_t x = A + i, v = e[i];
        if (x >= E) { val[i] = m->ring[x & 0xFFFF]; continue; }
        val[i] = v >= LITBASE ? m->zin[v - LITBASE] : m->ring[(B - v) & 0xFFFF];
    }
    for (uint32_t i = 0; i < W; i++) {
        uint32_t x = A + i;
        m->ring[x & 0xFFFF] = val[i];
        if (x >= S && x < E) {
            if (x >= cap) return -3;
            out[x] = val[i];
        }
    }
    /* op covering the next start */
    while (o + 1 < m->nops && m->opp[o + 1] <= E) o++;
    *iS = o;
    m->windows++;
    return 0;
}

/* Decode one block.  Returns 0 ok, negative: the kernel would refuse. */
int win_decode(const uint8_t *in, uint32_t z, uint8_t *out, uint32_t cap, uint32_t *olen,
               long stats[6])
{
    M *m = calloc(1, sizeof(M));
    if (!m) return -9;
    m->in = in; m->z = z;
    uint32_t I = 0, st = ST_F, E = 0, S = 0, iS = 0, k = 0;
    uint32_t Pk = 0;            /* output start of the current piece */
    int eof = 0, rc = 0;
    if (z == 0) { free(m); return -1; }
    m->nops = 0;
    while (!eof) {
        /* carry: keep ops that end after S */
        uint32_t keep = iS;
        if (m->nops) {
            uint32_t n = m->nops - keep;
            memmove(m->opp, m->opp + keep, (n + 1) * 4);
            memmove(m->ops, m->ops + keep, n * 4);
            m->nops = n; iS = 0;
        }
        Pk = E;
        int r = parse_piece(m, &I, &st, &E, k & 1);
        if (r < 0) { rc = r; goto out; }
        eof = r == 1;
        int opfull = r == 2;
        if (E > cap) { rc = -3; goto out; }
        /* full windows */
        while (S < E && ((S & ~15u) + W <= E || eof)) {
            uint32_t A = S & ~15u, e2 = A + W < E ? A + W : E;
            if ((rc = run_window(m, S, e2, &iS, out, cap))) goto out;
            S = e2;
        }
        /* flush if the pending bytes hold ops of the previous piece (its zin
         * half is overwritten by the next piece) */
        if (!eof && S < E && (S < Pk || opfull)) {
            if ((rc = run_window(m, S, E, &iS, out, cap))) goto out;
            m->flushes++;
            S = E;
        }
        k++;
    }
    *olen = E;
out:
    if (stats) {
        stats[0] = m->windows; stats[1] = m->chase_iters; stats[2] = m->pieces;
        stats[3] = m->flushes; stats[4] = m->walks_fix; stats[5] = 0;
    }
    free(m);
    return rc;
}
