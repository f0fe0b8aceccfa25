"""GPU debug aid: the stream decoder with and without the parallel resume,
call by call (status, produced, consumed) and the first differing output
byte, on a few streams and call patterns."""
import os
import sys
import zlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jdeflate_amd as J
from jdeflate_amd import engine as E


def run(comp, piece, tgt, rpar):
    s = E.IStream()
    s.rpar(1 if rpar else 0)
    out, tr, pos = bytearray(), [], 0
    for _ in range(200000):
        st, err, prod, cons, _ = s.inflate(comp[pos:pos + piece], tgt)
        out += s.out.raw[:prod]
        tr.append((st, err, prod, cons, len(out)))
        pos += cons
        if st == E.IS_FULL:
            continue
        if st != E.IS_NEEDINPUT or pos >= len(comp):
            break
    n = s.rpar()
    s.close()
    return tr, bytes(out), n


text = J.corpus_text(197840, seed=197840 & 0xffff).tobytes()
blk, _ = J.deflate_blocks(text, level=6)
z = zlib.compressobj(6, zlib.DEFLATED, -15)
zl = z.compress(text) + z.flush()
bad = 0
for name, comp in (("blocks", blk), ("zlib", zl)):
    for piece, tgt in ((5000, 70000), (5000, 1 << 20), (32768, 65536), (100000, 1 << 20)):
        a, oa, na = run(comp, piece, tgt, True)
        b, ob, nb = run(comp, piece, tgt, False)
        ok = oa == ob == text and a == b
        msg = f"{name} piece {piece} tgt {tgt}: rpar launches {na}, calls {len(a)}/{len(b)}, ok {ok}"
        if not ok:
            bad += 1
            i = next((k for k, (x, y) in enumerate(zip(a, b)) if x != y), None)
            j = next((k for k in range(min(len(oa), len(text))) if oa[k] != text[k]), None)
            msg += f"; first differing call {i}: {a[i] if i is not None else None} vs {b[i] if i is not None else None}"
            msg += f"; first wrong byte {j} (len {len(oa)} vs {len(text)})"
        print(msg, flush=True)
        if not ok and bad <= 2:
            # again with one stderr line per launch (JD_IS_TRACE), and the
            # bytes around the first wrong one
            os.environ["JD_IS_TRACE"] = "1"
            sys.stderr.flush()
            a, oa, na = run(comp, piece, tgt, True)
            os.environ["JD_IS_TRACE"] = "0"
            j = next((k for k in range(min(len(oa), len(text))) if oa[k] != text[k]), None)
            if j is not None:
                nw = sum(1 for k in range(j, min(len(oa), len(text))) if oa[k] != text[k])
                print(f"  wrong byte {j}: {nw} wrong bytes after it; got {oa[j:j + 24]!r}",
                      f"want {text[j:j + 24]!r}; want before {text[j - 24:j]!r}", flush=True)
                # where the wrong bytes appear earlier in the text (source of a copy?)
                w = oa[j:j + 12]
                print("  got bytes found in text at", [m for m in range(len(text)) if text.startswith(w, m)][:8],
                      flush=True)
print("rpar_debug", "FAIL" if bad else "ok", bad)
sys.exit(1 if bad else 0)
