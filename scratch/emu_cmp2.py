import sys, ctypes, numpy as np
sys.path.insert(0, '/root/repo')
exec(open('scratch/emu_cmp.py').read().split("m = J.corpus_mixed")[0])
sc = ctypes.c_ulong.in_dll(E, "slowcalls")
sets = {"mixed": J.corpus_mixed(64 * 65536, seed=4).tobytes(), "text": J.corpus_text(32 * 65536, seed=3).tobytes(),
        "rand": np.random.default_rng(1).integers(0, 256, 4 * 65536, dtype=np.uint8).tobytes(),
        "src": open('/usr/lib/python3.10/typing.py','rb').read() + open('/usr/lib/python3.10/os.py','rb').read()}
for lvl in (6, 7, 8, 9):
    for name, data in sets.items():
        bad = 0; sc.value = 0; nb = -(-len(data) // 65536)
        for blk in range(nb):
            d = data[blk * 65536:(blk + 1) * 65536]
            a, ab = emu(d, lvl); o, obd = ora(d, lvl)
            if a != o or ab != obd: bad += 1
        print(f"L{lvl} {name}: {nb} blocks, mismatched {bad}, slow-path calls {sc.value}")
