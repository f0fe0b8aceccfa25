"""debug: token list of a raw deflate stream (pure Python inflate)"""
import sys

class Bits:
    def __init__(s, b): s.b = b; s.p = 0
    def get(s, n):
        v = 0
        for i in range(n):
            v |= ((s.b[s.p >> 3] >> (s.p & 7)) & 1) << i; s.p += 1
        return v
def build(lens):
    codes = {}; code = 0; bl = [0] * 16
    for l in lens:
        if l: bl[l] += 1
    nxt = [0] * 16
    for b in range(1, 16):
        code = (code + bl[b - 1]) << 1; nxt[b] = code
    for sym, l in enumerate(lens):
        if l: codes[(l, nxt[l])] = sym; nxt[l] += 1
    return codes
def dec(bs, t):
    c = 0; l = 0
    while True:
        c = (c << 1) | bs.get(1); l += 1
        if (l, c) in t: return t[(l, c)]
LB = [3,4,5,6,7,8,9,10,11,13,15,17,19,23,27,31,35,43,51,59,67,83,99,115,131,163,195,227,258]
LE = [0,0,0,0,0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,4,4,5,5,5,5,0]
DB = [1,2,3,4,5,7,9,13,17,25,33,49,65,97,129,193,257,385,513,769,1025,1537,2049,3073,4097,6145,8193,12289,16385,24577]
DE = [0,0,0,0,1,1,2,2,3,3,4,4,5,5,6,6,7,7,8,8,9,9,10,10,11,11,12,12,13,13]
def tokens(b):
    bs = Bits(b); out = []; pos = 0
    while True:
        fin = bs.get(1); typ = bs.get(2)
        out.append(("B", typ, pos, bs.p))
        if typ == 0:
            bs.p = (bs.p + 7) & ~7
            n = bs.get(16); bs.get(16)
            for i in range(n): out.append(("L", bs.get(8)))
            pos += n
        else:
            if typ == 1:
                lt = build([8]*144 + [9]*112 + [7]*24 + [8]*8); dt = build([5]*30)
            else:
                hl = bs.get(5) + 257; hd = bs.get(5) + 1; hc = bs.get(4) + 4
                order = [16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15]
                cl = [0]*19
                for i in range(hc): cl[order[i]] = bs.get(3)
                ct = build(cl); ls = []
                while len(ls) < hl + hd:
                    sy = dec(bs, ct)
                    if sy < 16: ls.append(sy)
                    elif sy == 16: ls += [ls[-1]] * (3 + bs.get(2))
                    elif sy == 17: ls += [0] * (3 + bs.get(3))
                    else: ls += [0] * (11 + bs.get(7))
                lt = build(ls[:hl]); dt = build(ls[hl:])
            while True:
                sy = dec(bs, lt)
                if sy < 256: out.append(("L", sy)); pos += 1
                elif sy == 256: break
                else:
                    k = sy - 257; ln = LB[k] + bs.get(LE[k]); d = dec(bs, dt); dist = DB[d] + bs.get(DE[d])
                    out.append(("M", ln, dist)); pos += ln
        if fin: break
        if bs.p >= len(b) * 8 - 2: break
    return out
