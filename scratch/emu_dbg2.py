import sys
sys.path.insert(0, '/root/repo')
exec(open('scratch/emu_cmp.py').read().split("m = J.corpus_mixed")[0])
m = J.corpus_mixed(16 * 65536, seed=4).tobytes()
d = m[11 * 65536:12 * 65536]
a, ab = emu(d, 6); o, obd = ora(d, 6)
f = lambda t: ("M", (t >> 16) & 0x7fff, t & 0xffff) if t & 0x80000000 else ("L", t)
def positions(toks):
    pos = 0; out = []
    for x in toks:
        out.append(pos); pos += ((x >> 16) & 0x7fff) if x & 0x80000000 else 1
    return out
pa, po = positions(a), positions(o)
for i in range(305, 316):
    print(i, pa[i], f(a[i]), "|", po[i], f(o[i]))
