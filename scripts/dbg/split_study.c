/* split_study.c -- CPU study (round 3): does a speculative split of the LZO1X-1
 * parse (SURVEY Appendix A.1 rules) converge to the true parse?  Not product code. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#define SLOTS 16384
static uint32_t h1f(const uint8_t *p) {
    uint32_t b0 = p[0], b1 = p[1], b2 = p[2], b3 = p[3];
    return ((((((b3 << 6) ^ b2) << 5) ^ b1) << 5 ^ b0) * 33 >> 5) & 0x3FFF;
}
/* parse [start, n) with an empty dictionary; rec[p]: 0 not visited, 1 visited h1, 2 visited h2 */
static void parse(const uint8_t *in, size_t n, size_t start, uint8_t *rec, size_t *ii_at, size_t stop_at)
{
    static uint32_t dict[SLOTS];
    memset(dict, 0, sizeof dict);
    size_t ip = start < 4 ? 4 : start, ii = start, ip_end = n - 13;
    memset(rec, 0, n);
    for (;;) {
        if (ip >= stop_at && ii_at) { *ii_at = ii; ii_at = NULL; }
        uint32_t slot = h1f(in + ip), cand = dict[slot]; size_t c = 0; int ok = 0, used2 = 0;
        if (cand && ip - (cand - 1) <= 0xBFFF) {
            c = cand - 1;
            if (ip - c <= 0x800 || in[c + 3] == in[ip + 3]) ok = 1;
            else {
                slot = (slot & 0x7FF) ^ 0x201F; used2 = 1; cand = dict[slot];
                if (cand && ip - (cand - 1) <= 0xBFFF) { c = cand - 1; if (ip - c <= 0x800 || in[c + 3] == in[ip + 3]) ok = 1; }
            }
        }
        if (ok && !(in[c] == in[ip] && in[c + 1] == in[ip + 1] && in[c + 2] == in[ip + 2])) ok = 0;
        dict[slot] = ip + 1;
        rec[ip] = 1 + used2;
        if (!ok) { if (++ip >= ip_end) break; continue; }
        size_t len = 3;
        while (len < 9 && in[c + len] == in[ip + len]) len++;
        if (len == 9) while (ip + len < n && in[c + len] == in[ip + len]) len++;
        ip += len; ii = ip;
        if (ip >= ip_end) break;
    }
    if (ii_at) *ii_at = ii;
}
void study(const uint8_t *in, size_t n, size_t seg, size_t D, long out[4])
{
    uint8_t *tr = malloc(n), *sp = malloc(n);
    size_t ii_t, ii_s;
    parse(in, n, 0, tr, NULL, n);
    long ok = 0, tot = 0, syncsum = 0;
    for (size_t s = seg; s + 16 < n; s += seg) {
        size_t w = s > 0xBFFF + D ? s - 0xBFFF - D : 0;
        if (w == 0) continue;
        /* first visited position >= s in the true parse */
        size_t v = s; while (v < n && !tr[v]) v++;
        parse(in, n, w, sp, NULL, n);
        parse(in, n, 0, tr, &ii_t, v);
        parse(in, n, w, sp, &ii_s, v);
        int eq = memcmp(tr + (v - 0xBFFF), sp + (v - 0xBFFF), 0xBFFF) == 0 && ii_t == ii_s && sp[v] == tr[v];
        /* earliest x such that tr and sp agree on [x, v) */
        size_t x = v; while (x > w && tr[x - 1] == sp[x - 1]) x--;
        syncsum += (long)(x - w);
        ok += eq; tot++;
    }
    out[0] = ok; out[1] = tot; out[2] = tot ? syncsum / tot : 0; out[3] = 0;
    free(tr); free(sp);
}
