/* CPU study: how many of the one-wave encoder's dictionary
 * probes read a slot that no earlier position of the block has written, i.e.
 * loads a per-block LDS occupancy bitmap would skip.  Restates the greedy
 * parse of oracle/lzo1x_oracle.c (lib/minilzo.c:2922-3157) and groups it into
 * windows the way lzo1x_encode_gdict1_kernel does (64 positions from the
 * window start, at most 6 matches; forwarding cuts ignored).  Every lane
 * probes h1 and h2 with the dictionary as it was at the window start.
 *   gcc -O2 -o /tmp/enc_empty_sim scripts/dbg/enc_empty_sim.c
 *   /tmp/enc_empty_sim FILE BLOCK_BYTES      (FILE: raw concatenated blocks)
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { SLOTS = 1u << 14, FAR = 0xBFFF, NEAR = 0x0800, GUARD = 13, WAVE = 64, PATHMAX = 6 };

static uint32_t h1_of(const uint8_t *p)
{
    uint32_t v = ((((uint32_t)p[3] << 6) ^ p[2]) << 5) ^ p[1];
    v = (v << 5) ^ p[0];
    return ((v * 33u) >> 5) & (SLOTS - 1);
}
static uint32_t h2_of(uint32_t h) { return (h & 0x7FFu) ^ 0x201Fu; }

struct st { double win, lanes, e1, e2, allempty1, allempty12, lines_all, lines_occ, lines_occ2, visited, cl_valid, cl_ok, n_valid, n_ok; };

static void block(const uint8_t *in, size_t n, struct st *S)
{
    static uint32_t dict[SLOTS];
    static uint8_t wr[SLOTS];          /* written at all (the bitmap) */
    memset(dict, 0, sizeof dict);
    memset(wr, 0, sizeof wr);
    if (n <= GUARD)
        return;
    const size_t ip_end = n - GUARD;
    size_t ip = 4;
    while (ip < ip_end) {
        /* window [ip, ip + 64): probes against the current dictionary */
        S->win++;
        int any1 = 0, any12 = 0;
        static uint8_t cand_lines[(1 << 17) / 128], ok_lines[(1 << 17) / 128];
        memset(cand_lines, 0, sizeof cand_lines);
        memset(ok_lines, 0, sizeof ok_lines);
        uint8_t line_all[SLOTS / 64] = {0}, line_occ[SLOTS / 64] = {0}, line_occ2[SLOTS / 64] = {0};
        for (size_t p = ip; p < ip + WAVE && (p < ip_end || p == ip); p++) {
            uint32_t a = h1_of(in + p), b = h2_of(a);
            S->lanes++;
            if (!wr[a]) S->e1++; else any1 = 1;
            if (!wr[b]) S->e2++; else any12 = 1;
            line_all[a / 64] = line_all[b / 64] = 1;
            if (wr[a]) line_occ[a / 64] = 1;
            if (wr[b]) line_occ[b / 64] = 1;
            if (wr[a]) line_occ2[a / 64] = 1;      /* h2 only behind a written h1 */
            if (wr[a] && wr[b]) line_occ2[b / 64] = 1;
            /* candidate loads (as the kernel: c1 when valid, c2 when the
             * primary is far and the secondary valid) against the lanes whose
             * candidate really passes try_match */
            size_t w1 = dict[a] ? dict[a] - 1 : 0, w2 = dict[b] ? dict[b] - 1 : 0;
            int v1 = dict[a] && p - w1 <= FAR, v2 = v1 && dict[b] && p - w2 <= FAR;
            int c1pass = v1 && (p - w1 <= NEAR || in[w1 + 3] == in[p + 3]);
            int c2pass = v1 && !c1pass && v2 && (p - w2 <= NEAR || in[w2 + 3] == in[p + 3]);
            size_t c = c2pass ? w2 : w1;
            int ok = (c1pass || c2pass) && in[c] == in[p] && in[c + 1] == in[p + 1] && in[c + 2] == in[p + 2];
            if (v1) { S->n_valid++; cand_lines[(w1 + 3) >> 7] = 1; cand_lines[(w1 + 31) >> 7] = 1; }
            if (v2 && p - w1 > NEAR) { cand_lines[(w2 + 3) >> 7] = 1; cand_lines[(w2 + 31) >> 7] = 1; }
            if (ok) { S->n_ok++; ok_lines[(c + 3) >> 7] = 1; ok_lines[(c + 31) >> 7] = 1; }
        }
        for (size_t i = 0; i < sizeof cand_lines; i++) { S->cl_valid += cand_lines[i]; S->cl_ok += ok_lines[i]; }
        any12 |= any1;
        S->allempty1 += !any1;
        S->allempty12 += !any12;
        for (int i = 0; i < SLOTS / 64; i++) {
            S->lines_all += line_all[i];
            S->lines_occ += line_occ[i];
            S->lines_occ2 += line_occ2[i];
        }
        /* the true parse through the window */
        const size_t wend = ip + WAVE;
        int nm = 0;
        while (ip < ip_end && ip < wend && nm < PATHMAX) {
            uint32_t slot = h1_of(in + ip), cand = dict[slot];
            size_t c = 0, off;
            int ok = 0;
            if (cand && ip - (cand - 1) <= FAR) {
                c = cand - 1; off = ip - c;
                if (off <= NEAR || in[c + 3] == in[ip + 3]) ok = 1;
                else {
                    slot = h2_of(slot); cand = dict[slot];
                    if (cand && ip - (cand - 1) <= FAR) {
                        c = cand - 1; off = ip - c;
                        if (off <= NEAR || in[c + 3] == in[ip + 3]) ok = 1;
                    }
                }
            }
            if (ok && !(in[c] == in[ip] && in[c + 1] == in[ip + 1] && in[c + 2] == in[ip + 2]))
                ok = 0;
            dict[slot] = (uint32_t)(ip + 1);
            wr[slot] = 1;
            S->visited++;
            if (!ok) { ip++; continue; }
            size_t len = 3;
            while (ip + len < n && in[c + len] == in[ip + len]) len++;
            ip += len;
            nm++;
        }
    }
}

int main(int argc, char **argv)
{
    if (argc < 3) { fprintf(stderr, "usage: %s FILE BLOCK_BYTES\n", argv[0]); return 2; }
    FILE *f = fopen(argv[1], "rb");
    size_t bs = strtoul(argv[2], 0, 0);
    uint8_t *buf = malloc(bs);
    struct st S = {0};
    size_t nb = 0;
    while (f && fread(buf, 1, bs, f) == bs) { block(buf, bs, &S); nb++; }
    if (!nb) { fprintf(stderr, "no blocks\n"); return 1; }
    printf("blocks %zu: windows/block %.1f, visited/block %.0f\n", nb, S.win / nb, S.visited / nb);
    printf("lane probes empty: h1 %.1f%%, h2 %.1f%%\n", 100 * S.e1 / S.lanes, 100 * S.e2 / S.lanes);
    printf("windows with every h1 empty %.1f%%, every h1 and h2 empty %.1f%%\n",
           100 * S.allempty1 / S.win, 100 * S.allempty12 / S.win);
    printf("dictionary lines per window: all probes %.1f, written slots only %.1f, "
           "and h2 only behind a written h1 %.1f\n",
           S.lines_all / S.win, S.lines_occ / S.win, S.lines_occ2 / S.win);
    printf("candidate lanes per window: valid %.1f, passing try_match %.1f; input lines: loaded %.1f, "
           "of passing lanes %.1f\n", S.n_valid / S.win, S.n_ok / S.win, S.cl_valid / S.win, S.cl_ok / S.win);
    return 0;
}
