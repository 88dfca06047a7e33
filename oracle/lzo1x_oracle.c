/*
 * oracle/lzo1x_oracle.c -- CPU restatement of miniLZO 2.04's LZO1X-1 codec.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the
 * MI355X LZO1X path.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product library (liblzo_mi355x.so)
 * never links, loads or calls anything in oracle/.
 *
 * Parity is PINNED: tests/golden/ holds vectors produced by the reference
 * itself (lib/minilzo.c compiled in place by oracle/Makefile into
 * oracle/_ref/), and tests/test_oracle.py checks this restatement against
 * every one of them.  The restatement is written from the behavioral spec in
 * SURVEY.md Appendix A; comments cite the reference lines each rule follows
 * (paths relative to the reference tree).
 *
 * Output-defining conventions (SURVEY.md finding 3):
 *   - compression is defined as lzo1x_1_compress() run with a zero-filled
 *     wrkmem, i.e. every dictionary slot starts EMPTY;
 *   - the bounds-checked decoder reproduces lzo1x_decompress_safe()
 *     (lib/minilzo.c:3703-4190) including its unsigned NEED_IP arithmetic;
 *     input bytes at or past in_len read as 0 (the fixture generator gives
 *     the reference the same zero padding).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define ORC_E_OK 0                   /* lib/lzoconf.h:309 */
#define ORC_E_INPUT_OVERRUN (-4)     /* lib/lzoconf.h:313 */
#define ORC_E_OUTPUT_OVERRUN (-5)    /* lib/lzoconf.h:314 */
#define ORC_E_LOOKBEHIND_OVERRUN (-6)/* lib/lzoconf.h:315 */
#define ORC_E_EOF_NOT_FOUND (-7)     /* lib/lzoconf.h:316 */
#define ORC_E_INPUT_NOT_CONSUMED (-8)/* lib/lzoconf.h:317 */

enum {
    DICT_SLOTS = 1u << 14,   /* D_BITS 14, lib/minilzo.c:2627 */
    FAR_LIMIT = 0xBFFF,      /* M4_MAX_OFFSET, lib/minilzo.c:2653 */
    NEAR_LIMIT = 0x0800,     /* M2_MAX_OFFSET, lib/minilzo.c:2622 */
    MID_LIMIT = 0x4000,      /* M3_MAX_OFFSET, lib/minilzo.c:2652 */
    TAIL_GUARD = 13          /* M2_MAX_LEN + 5, lib/minilzo.c:2929,3167 */
};

/* Primary slot of the 4 bytes at p: DX3(p,5,5,6) * 0x21 >> 5, masked to 14
 * bits (lib/minilzo.c:2629, 2697-2704). */
static inline uint32_t slot_primary(const uint8_t *p)
{
    uint32_t v = ((((uint32_t)p[3] << 6) ^ p[2]) << 5) ^ p[1];
    v = (v << 5) ^ p[0];
    return ((v * 33u) >> 5) & (DICT_SLOTS - 1);
}

/* Secondary slot derived from the primary (D_INDEX2, lib/minilzo.c:2630). */
static inline uint32_t slot_secondary(uint32_t h)
{
    return (h & 0x7FFu) ^ 0x201Fu;
}

/* Emit a run-length continuation: (x / 255) zero bytes, then the rest
 * (lib/minilzo.c:3034-3046, 3129-3139). */
static size_t put_ext(uint8_t *out, size_t op, size_t x)
{
    while (x > 255) {
        out[op++] = 0;
        x -= 255;
    }
    out[op++] = (uint8_t)x;
    return op;
}

/* Literal-run header for r pending literals in the middle of the stream
 * (lib/minilzo.c:3023-3048).  r <= 3 folds into the low bits of the byte
 * two positions back (the previous match's last-but-one byte). */
static size_t put_lit_header(uint8_t *out, size_t op, size_t r)
{
    if (r <= 3)
        out[op - 2] |= (uint8_t)r;
    else if (r <= 18)
        out[op++] = (uint8_t)(r - 3);
    else {
        out[op++] = 0;
        op = put_ext(out, op, r - 18);
    }
    return op;
}

/* Encode one match of length len at distance off (lib/minilzo.c:3064-3145). */
static size_t put_match(uint8_t *out, size_t op, size_t len, size_t off)
{
    if (len <= 8) {
        if (off <= NEAR_LIMIT) {                       /* M2 */
            size_t o = off - 1;
            out[op++] = (uint8_t)(((len - 1) << 5) | ((o & 7) << 2));
            out[op++] = (uint8_t)(o >> 3);
            return op;
        }
        if (off <= MID_LIMIT) {                        /* M3, short */
            size_t o = off - 1;
            out[op++] = (uint8_t)(0x20 | (len - 2));
            out[op++] = (uint8_t)((o & 63) << 2);
            out[op++] = (uint8_t)(o >> 6);
            return op;
        }
        size_t o = off - 0x4000;                       /* M4, short */
        out[op++] = (uint8_t)(0x10 | ((o & 0x4000) >> 11) | (len - 2));
        out[op++] = (uint8_t)((o & 63) << 2);
        out[op++] = (uint8_t)(o >> 6);
        return op;
    }
    size_t o;
    if (off <= MID_LIMIT) {                            /* M3, long */
        o = off - 1;
        if (len <= 33)
            out[op++] = (uint8_t)(0x20 | (len - 2));
        else {
            out[op++] = 0x20;
            op = put_ext(out, op, len - 33);
        }
    } else {                                           /* M4, long */
        o = off - 0x4000;
        uint8_t hi = (uint8_t)((o & 0x4000) >> 11);
        if (len <= 9)
            out[op++] = (uint8_t)(0x10 | hi | (len - 2));
        else {
            out[op++] = (uint8_t)(0x10 | hi);
            op = put_ext(out, op, len - 9);
        }
    }
    out[op++] = (uint8_t)((o & 63) << 2);
    out[op++] = (uint8_t)(o >> 6);
    return op;
}

/* Greedy parse over in[0..n), n > 13 (lib/minilzo.c:2922-3157).  Returns the
 * number of trailing bytes left for the tail literal run; *op_out receives
 * the bytes written.  The dictionary holds position+1 (0 = EMPTY), which is
 * how a zero-filled wrkmem of NULL pointers behaves under
 * LZO_CHECK_MPOS_NON_DET (lib/minilzo.c:2878-2883). */
static size_t parse_core(const uint8_t *in, size_t n, uint8_t *out,
                         size_t *op_out, uint32_t *dict)
{
    size_t op = 0, ii = 0, ip = 4;
    const size_t ip_end = n - TAIL_GUARD;

    for (;;) {
        uint32_t slot = slot_primary(in + ip);
        uint32_t cand = dict[slot];
        size_t c = 0, off = 0;
        int ok = 0;

        if (cand != 0 && ip - (cand - 1) <= FAR_LIMIT) {
            c = cand - 1;
            off = ip - c;
            if (off <= NEAR_LIMIT || in[c + 3] == in[ip + 3])
                ok = 1;
            else {
                slot = slot_secondary(slot);
                cand = dict[slot];
                if (cand != 0 && ip - (cand - 1) <= FAR_LIMIT) {
                    c = cand - 1;
                    off = ip - c;
                    if (off <= NEAR_LIMIT || in[c + 3] == in[ip + 3])
                        ok = 1;
                }
            }
        }
        /* try_match: the first three bytes must agree (lib/minilzo.c:2962-2971) */
        if (ok && !(in[c] == in[ip] && in[c + 1] == in[ip + 1] &&
                    in[c + 2] == in[ip + 2]))
            ok = 0;

        dict[slot] = (uint32_t)(ip + 1);  /* UPDATE_I, lib/minilzo.c:3015,3022 */
        if (!ok) {
            if (++ip >= ip_end)
                break;
            continue;
        }

        if (ip > ii) {                     /* pending literals */
            op = put_lit_header(out, op, ip - ii);
            memcpy(out + op, in + ii, ip - ii);
            op += ip - ii;
        }

        /* Match length: bytes 3..8 first, then open-ended extension
         * (lib/minilzo.c:3051-3102). */
        size_t len = 3;
        while (len < 9 && in[c + len] == in[ip + len])
            len++;
        if (len == 9)
            while (ip + len < n && in[c + len] == in[ip + len])
                len++;

        op = put_match(out, op, len, off);
        ip += len;
        ii = ip;
        if (ip >= ip_end)
            break;
    }
    *op_out = op;
    return n - ii;
}

/* lzo1x_1_compress with a zero-filled wrkmem (lib/minilzo.c:3159-3207).
 * out must hold n + n/16 + 67 bytes.  Always returns ORC_E_OK. */
int oracle_lzo1x_1_compress(const uint8_t *in, size_t n, uint8_t *out,
                            size_t *out_len)
{
    static __thread uint32_t dict[DICT_SLOTS];
    size_t op = 0, t;

    if (n <= TAIL_GUARD)
        t = n;
    else {
        memset(dict, 0, sizeof(dict));
        t = parse_core(in, n, out, &op, dict);
    }
    if (t > 0) {
        size_t ii = n - t;
        if (op == 0 && t <= 238)
            out[op++] = (uint8_t)(17 + t);
        else
            op = put_lit_header(out, op, t);
        memcpy(out + op, in + ii, t);
        op += t;
    }
    out[op++] = 0x11;                       /* M4_MARKER | 1, then 0 0 */
    out[op++] = 0;
    out[op++] = 0;
    *out_len = op;
    return ORC_E_OK;
}

/* ------------------------------------------------------------------------ */
/* Decoder: the LZO1X grammar with lzo1x_decompress_safe's checks           */
/* (lib/minilzo.c:3308-3699 compiled with LZO_TEST_OVERRUN, :3703-3761).    */
/* ------------------------------------------------------------------------ */

struct dstate {
    const uint8_t *in;
    size_t in_len;
    uint8_t *out;
    size_t cap;
    size_t ip, op;
    int unchecked;      /* lzo1x_decompress (no input checks) instead of _safe */
};

/* The unchecked decoder (lib/minilzo.c:3308-3699, LZO_TEST_OVERRUN undefined,
 * :3214) reads past the input end without looking; with the input zero padded
 * (the convention of every harness here) a stream that has not ended by then
 * would read zeros forever, so a walk more than this many bytes past the end
 * stops with INPUT_OVERRUN (the code :3676-3680 gives for ip > ip_end).
 * The GPU exact decoder uses the same bound (lzo1x_kernels.hip). */
#define ORC_UNCHECKED_SLACK 64

static inline uint32_t rd(const struct dstate *s, size_t i)
{
    return i < s->in_len ? s->in[i] : 0u;
}

/* NEED_IP(x): fails only when ip <= in_len and fewer than x bytes remain.
 * The reference computes (lzo_uint)(ip_end - ip), so once ip has run past the
 * end the check passes (lib/minilzo.c:3733-3734). */
static inline int need_ip(const struct dstate *s, size_t x)
{
    if (s->unchecked)
        return s->ip <= s->in_len + ORC_UNCHECKED_SLACK;
    return !(s->ip <= s->in_len && s->in_len - s->ip < x);
}

/* TEST_IP at the top of the instruction loop (:3367, :3667): the safe decoder
 * stops with EOF_NOT_FOUND at the input end; the unchecked one reads on. */
static inline int test_ip(const struct dstate *s)
{
    return s->unchecked ? 1 : s->ip < s->in_len;
}

static inline int need_op(const struct dstate *s, size_t x)
{
    return s->cap - s->op >= x;       /* lib/minilzo.c:3740-3741 */
}

static inline void copy_lits(struct dstate *s, size_t t)
{
    for (size_t k = 0; k < t; k++)
        s->out[s->op + k] = (uint8_t)rd(s, s->ip + k);
    s->ip += t;
    s->op += t;
}

/* Byte-serial forward copy; overlapping sources repeat with period dist. */
static inline void copy_back(struct dstate *s, size_t dist, size_t len)
{
    size_t from = s->op - dist;
    for (size_t k = 0; k < len; k++)
        s->out[s->op + k] = s->out[from + k];
    s->op += len;
}

/* Length continuation: 255 per zero byte, then base + next byte. */
static inline int read_ext(struct dstate *s, size_t base, size_t *t)
{
    if (!need_ip(s, 1))
        return 0;
    size_t v = 0;
    while (rd(s, s->ip) == 0) {
        v += 255;
        s->ip++;
        if (!need_ip(s, 1))
            return 0;
    }
    *t = v + base + rd(s, s->ip++);
    return 1;
}

static int decompress(const uint8_t *in, size_t in_len, uint8_t *out, size_t *out_len,
                      int unchecked)
{
    struct dstate s = { in, in_len, out, *out_len, 0, 0, unchecked };
    size_t t, dist;
    /* where: 0 = top of the instruction loop, 1 = right after a literal run,
     * 2 = a match opcode t is pending, 3 = trailing literals pending */
    int where;
    int rc;

    *out_len = 0;
    t = rd(&s, 0);
    if (t > 17) {                          /* first-byte literal run, :3357 */
        s.ip = 1;
        t -= 17;
        if (t < 4)
            where = 3;
        else {
            if (!need_op(&s, t)) goto out_over;
            if (!need_ip(&s, t + 1)) goto in_over;
            copy_lits(&s, t);
            where = 1;
        }
    } else
        where = 0;

    for (;;) {
        if (where == 0) {                  /* :3367-3414 */
            if (!test_ip(&s))
                goto no_eof;
            if (!need_ip(&s, 1))
                goto in_over;
            t = rd(&s, s.ip++);
            if (t >= 16) {
                where = 2;
                continue;
            }
            if (t == 0 && !read_ext(&s, 15, &t))
                goto in_over;
            if (!need_op(&s, t + 3)) goto out_over;
            if (!need_ip(&s, t + 4)) goto in_over;
            copy_lits(&s, t + 3);
            where = 1;
            continue;
        }
        if (where == 1) {                  /* first_literal_run, :3416-3443 */
            t = rd(&s, s.ip++);
            if (t >= 16) {
                where = 2;
                continue;
            }
            dist = 1 + 0x800 + (t >> 2) + (rd(&s, s.ip++) << 2);
            if (dist > s.op) goto lb_over;
            if (!need_op(&s, 3)) goto out_over;
            copy_back(&s, dist, 3);
        } else if (where == 2) {           /* match, :3446-3646 */
            size_t len;
            if (t >= 64) {                 /* M2 */
                dist = 1 + ((t >> 2) & 7) + (rd(&s, s.ip++) << 3);
                len = (t >> 5) + 1;
            } else if (t >= 32) {          /* M3 */
                len = t & 31;
                if (len == 0 && !read_ext(&s, 31, &len))
                    goto in_over;
                len += 2;
                dist = 1 + ((rd(&s, s.ip) | (rd(&s, s.ip + 1) << 8)) >> 2);
                s.ip += 2;
            } else if (t >= 16) {          /* M4 or EOF */
                size_t d = (t & 8) << 11;
                len = t & 7;
                if (len == 0 && !read_ext(&s, 7, &len))
                    goto in_over;
                len += 2;
                d += (rd(&s, s.ip) | (rd(&s, s.ip + 1) << 8)) >> 2;
                s.ip += 2;
                if (d == 0)
                    goto eof;
                dist = d + 0x4000;
            } else {                       /* M1: 2 bytes after trailing lits */
                dist = 1 + (t >> 2) + (rd(&s, s.ip++) << 2);
                len = 2;
            }
            if (dist > s.op) goto lb_over;
            if (!need_op(&s, len)) goto out_over;
            copy_back(&s, dist, len);
        } else {                           /* where == 3: trailing literals */
            goto match_next;
        }
        /* match_done, :3650-3653 */
        t = rd(&s, s.ip - 2) & 3;
        if (t == 0) {
            where = 0;
            continue;
        }
    match_next:                            /* :3654-3668 */
        if (!need_op(&s, t)) goto out_over;
        if (!need_ip(&s, t + 1)) goto in_over;
        copy_lits(&s, t);
        t = rd(&s, s.ip++);
        if (!test_ip(&s))
            goto no_eof;
        where = 2;
    }

eof:                                       /* :3676-3680 */
    *out_len = s.op;
    if (s.ip == s.in_len) return ORC_E_OK;
    return s.ip < s.in_len ? ORC_E_INPUT_NOT_CONSUMED : ORC_E_INPUT_OVERRUN;
no_eof:
    rc = ORC_E_EOF_NOT_FOUND;
    goto fin;
in_over:
    rc = ORC_E_INPUT_OVERRUN;
    goto fin;
out_over:
    rc = ORC_E_OUTPUT_OVERRUN;
    goto fin;
lb_over:
    rc = ORC_E_LOOKBEHIND_OVERRUN;
fin:
    *out_len = s.op;
    return rc;
}

/* lzo1x_decompress_safe (lib/minilzo.c:3703-4190): *out_len is the capacity
 * in, the produced length out. */
int oracle_lzo1x_decompress_safe(const uint8_t *in, size_t in_len,
                                 uint8_t *out, size_t *out_len)
{
    return decompress(in, in_len, out, out_len, 0);
}

/* lzo1x_decompress, the unchecked decoder Pomegranate calls (mds/itb.c:2964,
 * mdsl/gc.c:770, api/api.c:6438): no input checks, so trailing bytes and
 * back-to-back streams give INPUT_NOT_CONSUMED after the first EOF and a
 * stream whose EOF marker is cut short INPUT_OVERRUN (:3676-3680).  *out_len
 * is the output room in (the reference has none: the caller sizes it). */
int oracle_lzo1x_decompress_unchecked(const uint8_t *in, size_t in_len,
                                      uint8_t *out, size_t *out_len)
{
    return decompress(in, in_len, out, out_len, 1);
}

/* Worst-case compressed size used by every harness (lib/minilzo.h notes
 * n + n/16 + 64 + 3). */
size_t oracle_lzo1x_worst(size_t n)
{
    return n + n / 16 + 64 + 3;
}
