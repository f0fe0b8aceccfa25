import sys, ctypes
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/scratch')
exec(open('scratch/emu_cmp.py').read().split("m = J.corpus_mixed")[0])
m = J.corpus_mixed(16 * 65536, seed=4).tobytes()
d = m[11 * 65536:12 * 65536]
a, ab = emu(d, 6); o, obd = ora(d, 6)
f = lambda t: ("M", (t >> 16) & 0x7fff, t & 0xffff) if t & 0x80000000 else ("L", t)
pos = 0
for i, (x, y) in enumerate(zip(a, o)):
    if x != y:
        print("diff at tok", i, "pos", pos, "emu", f(x), "ora", f(y))
        print("ctx emu", [f(z) for z in a[i-6:i+4]])
        print("ctx ora", [f(z) for z in o[i-6:i+4]])
        print("bytes", d[pos-40:pos+20])
        break
    pos += ((x >> 16) & 0x7fff) if x & 0x80000000 else 1
