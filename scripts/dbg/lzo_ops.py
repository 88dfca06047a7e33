"""Debug helper: the op list of an LZO1X stream (pure Python)."""
def parse(z):
    """returns list of ops: ('L', out, len, inpos) or ('M', out, len, dist)"""
    ops = []
    ip = 0; op = 0
    state = 'F'
    def lit(n):
        nonlocal ip, op
        ops.append(('L', op, n, ip)); ip += n; op += n
    t = z[0]
    if t > 17:
        ip = 1
        lit(t - 17)
        state = 'C' if t - 17 < 4 else 'B'
    while True:
        t = z[ip]; ip += 1
        if state in ('A', 'F') and t < 16:
            if t == 0:
                t = 15
                while z[ip] == 0:
                    t += 255; ip += 1
                t += z[ip]; ip += 1
            lit(t + 3)
            state = 'B'
            continue
        if t < 16:
            if state == 'B':
                dist = 1 + 0x800 + (t >> 2) + (z[ip] << 2); ip += 1; ln = 3
            else:
                dist = 1 + (t >> 2) + (z[ip] << 2); ip += 1; ln = 2
        elif t >= 64:
            dist = 1 + ((t >> 2) & 7) + (z[ip] << 3); ip += 1; ln = (t >> 5) + 1
        elif t >= 32:
            ln = t & 31
            if ln == 0:
                ln = 31
                while z[ip] == 0:
                    ln += 255; ip += 1
                ln += z[ip]; ip += 1
            ln += 2
            dist = 1 + ((z[ip] | (z[ip + 1] << 8)) >> 2); ip += 2
        else:
            ln = t & 7
            if ln == 0:
                ln = 7
                while z[ip] == 0:
                    ln += 255; ip += 1
                ln += z[ip]; ip += 1
            ln += 2
            d = ((t & 8) << 11) + ((z[ip] | (z[ip + 1] << 8)) >> 2); ip += 2
            if d == 0:
                break
            dist = d + 0x4000
        ops.append(('M', op, ln, dist)); op += ln
        s = z[ip - 2] & 3
        if s == 0:
            state = 'A'
        else:
            lit(s); state = 'C'
    return ops, op

