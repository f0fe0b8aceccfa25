"""Table sizes needed by the dynamic trees of block-mode streams (root R,
two-level tables with subtables sized by the longest code under a prefix)."""
import sys, os, numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jdeflate_amd.engine as E
from oracle import jdoracle as O

class Bits:
    def __init__(s, b): s.b = b; s.p = 0
    def get(s, n):
        v = 0
        for i in range(n):
            v |= ((s.b[s.p >> 3] >> (s.p & 7)) & 1) << i; s.p += 1
        return v

ORDER = [16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15]

def canon(lens):
    cnt = [0]*16
    for l in lens: cnt[l] += 1
    cnt[0] = 0; code = 0; nxt = [0]*16
    for i in range(1,16): code = (code + cnt[i-1]) << 1; nxt[i] = code
    codes = []
    for l in lens:
        if l: c = nxt[l]; nxt[l] += 1; codes.append((int(format(c, '0%db' % l)[::-1], 2), l))
    return codes

def tsize(lens, R):
    m = {}
    for c, l in canon(lens):
        if l > R:
            p = c & ((1 << R) - 1); m[p] = max(m.get(p, 0), l - R)
    return (1 << R) + sum(1 << v for v in m.values())

def headers(blk):
    """yield (litlens, distlens) of each dynamic deflate block; decodes symbols
    only to skip over them"""
    bs = Bits(blk)
    import zlib
    out = []
    # use a simple decoder walk
    while bs.p < len(blk) * 8 - 7:
        fin = bs.get(1); t = bs.get(2)
        if t == 0:
            bs.p = (bs.p + 7) & ~7; ln = bs.get(16); bs.get(16); bs.p += 8 * ln
        elif t == 2:
            hl = bs.get(5) + 257; hd = bs.get(5) + 1; hc = bs.get(4) + 4
            pl = [0]*19
            for i in range(hc): pl[ORDER[i]] = bs.get(3)
            ptab = {(c, l): s for s, (c, l) in zip([i for i in range(19) if pl[i]], canon(pl))}
            def sym(tab):
                c = 0
                for l in range(1, 16):
                    c |= bs.get(1) << (l - 1)
                    if (c, l) in tab: return tab[(c, l)]
                raise ValueError
            lens = []
            while len(lens) < hl + hd:
                s = sym(ptab)
                if s < 16: lens.append(s)
                elif s == 16: lens += [lens[-1]] * (3 + bs.get(2))
                elif s == 17: lens += [0] * (3 + bs.get(3))
                else: lens += [0] * (11 + bs.get(7))
            ll, dl = lens[:hl], lens[hl:hl + hd]
            out.append((ll, dl))
            lt = {(c, l): s for s, (c, l) in zip([i for i in range(hl) if ll[i]], canon(ll))}
            dt = {(c, l): s for s, (c, l) in zip([i for i in range(hd) if dl[i]], canon(dl))}
            LB = [3,4,5,6,7,8,9,10,11,13,15,17,19,23,27,31,35,43,51,59,67,83,99,115,131,163,195,227,258]
            LE = [0,0,0,0,0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,4,4,5,5,5,5,0]
            DE = [0,0,0,0,1,1,2,2,3,3,4,4,5,5,6,6,7,7,8,8,9,9,10,10,11,11,12,12,13,13]
            while True:
                s = sym(lt)
                if s == 256: break
                if s > 256:
                    bs.get(LE[s - 257]); d = sym(dt); bs.get(DE[d])
        else:
            # static: skip by decoding with fixed tables
            fl = [8]*144 + [9]*112 + [7]*24 + [8]*8
            lt = {(c, l): s for s, (c, l) in zip(range(288), canon(fl))}
            dt = {(c, l): s for s, (c, l) in zip(range(32), canon([5]*32))}
            LE = [0,0,0,0,0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,4,4,5,5,5,5,0]
            DE = [0,0,0,0,1,1,2,2,3,3,4,4,5,5,6,6,7,7,8,8,9,9,10,10,11,11,12,12,13,13]
            def sym(tab):
                c = 0
                for l in range(1, 16):
                    c |= bs.get(1) << (l - 1)
                    if (c, l) in tab: return tab[(c, l)]
            while True:
                s = sym(lt)
                if s == 256: break
                if s > 256:
                    bs.get(LE[s - 257] if s < 285 else 0); d = sym(dt); bs.get(DE[d])
        if fin: break
    return out

if __name__ == "__main__":
    for name, gen in (("text", lambda n: E.corpus_text(n, seed=1000)), ("mixed", lambda n: E.corpus_mixed(n, seed=7))):
      d = gen(64 * 65536).tobytes()
      for lv in (6, 9):
          g, gs = O.deflate_blocks(d, level=lv)
          offs = np.concatenate([[0], np.cumsum(gs)])
          need = {}
          for i in range(len(gs)):
              for ll, dl in headers(g[offs[i]:offs[i+1]]):
                  for R in (8, 9, 10):
                      need.setdefault(('L', R), []).append(tsize(ll, R))
                  for R in (6, 7, 8):
                      need.setdefault(('D', R), []).append(tsize(dl, R))
                  need.setdefault('maxl', []).append(max(ll)); need.setdefault('maxd', []).append(max(dl))
          print(name, lv, {k: (max(v), int(np.percentile(v, 99))) for k, v in need.items()})
