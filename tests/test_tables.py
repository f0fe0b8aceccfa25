"""Decode tables from unusual code-length sets, built by a small RFC 1951
bit writer: codes up to 15 bits (subtables under the 10-bit and 8-bit
roots), a single one-bit distance code (the one incomplete code the
reference accepts, buildtable :381-568 mode 1), and the trees it rejects
(over-subscribed, incomplete literal/length codes, a missing end-of-block
code).  The CPU tests pin the writer against the oracle; the GPU tests
compare every decoder path -- block mode (P1 walks, the multi-phase and
wave-per-block fallbacks), the one-shot stream decoder and the drop-in
stream decoder with its parallel resume -- with the oracle's output and
error codes."""
import pytest

from oracle import jdoracle as O

LB = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115,
      131, 163, 195, 227, 258]
LE = [0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0]
CL_ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


class Bits:
    def __init__(self):
        self.acc, self.n, self.out = 0, 0, bytearray()

    def put(self, v, nb):
        self.acc |= v << self.n
        self.n += nb
        while self.n >= 8:
            self.out.append(self.acc & 0xff)
            self.acc >>= 8
            self.n -= 8

    def huff(self, code, ln):              # Huffman codes go MSB first
        self.put(int(format(code, f"0{ln}b")[::-1], 2), ln)

    def done(self):
        if self.n:
            self.out.append(self.acc & 0xff)
            self.acc, self.n = 0, 0
        return bytes(self.out)


def canonical(lens):
    """RFC 1951 3.2.2 codes for the lengths (0 = unused)"""
    mx = max(lens)
    cnt = [0] * (mx + 1)
    for ln in lens:
        if ln:
            cnt[ln] += 1
    code, nxt = 0, [0] * (mx + 2)
    for b in range(1, mx + 1):
        code = (code + cnt[b - 1]) << 1 if b > 1 else 0
        nxt[b] = code
    out = []
    for ln in lens:
        if ln:
            out.append(nxt[ln])
            nxt[ln] += 1
        else:
            out.append(None)
    return out


def dynamic_block(litlens, distlens, tokens, final=True):
    """one dynamic block: the lengths sent plainly (code-length symbols 0-15,
    every code-length code 4 bits), then the tokens: ints = literals,
    (length, distance) = matches; the end of block is appended"""
    hlit, hdist = len(litlens), len(distlens)
    w = Bits()
    w.put(1 if final else 0, 1)
    w.put(2, 2)
    w.put(hlit - 257, 5)
    w.put(hdist - 1, 5)
    w.put(19 - 4, 4)
    clens = [4 if s < 16 else 0 for s in range(19)]
    for s in CL_ORDER:
        w.put(clens[s], 3)
    ccode = canonical(clens)
    for ln in list(litlens) + list(distlens):
        w.huff(ccode[ln], 4)
    lc, dc = canonical(litlens), canonical(distlens) if any(distlens) else [None] * hdist
    for t in tokens + [256]:
        if isinstance(t, tuple):
            ln, d = t
            ls = max(i for i in range(29) if LB[i] <= ln)
            w.huff(lc[257 + ls], litlens[257 + ls])
            w.put(ln - LB[ls], LE[ls])
            ds, base = 0, 1
            while True:                                  # distance symbol
                extra = max(0, ds // 2 - 1)
                if d < base + (1 << extra):
                    break
                base += 1 << extra
                ds += 1
            w.huff(dc[ds], distlens[ds])
            w.put(d - base, extra)
        else:
            w.huff(lc[t], litlens[t])
    return w.done()


def deep_litlens():
    """literals 0-14 and the end of block at lengths 1..15, 15: complete, and
    the long ones need subtables under a 10-bit root"""
    lens = [0] * 286
    for b in range(15):
        lens[b] = b + 1
    lens[256] = 15
    return lens


def _params():
    deep = deep_litlens()
    toks = [b % 15 for b in range(3000)]
    # literal/length code with length codes too (Kraft sum 1): 12 literals
    # at 4 bits, the end of block and 7 length codes at 5 bits
    mix = [0] * 286
    for b in range(12):
        mix[b] = 4
    mix[256] = 5
    for s in range(257, 264):
        mix[s] = 5
    mtoks = []
    for i in range(400):
        mtoks += [i % 12, (i * 7) % 12, (i * 5) % 12]
        if i > 2:
            mtoks.append((3 + i % 7, 1 + i % 3))
    mtoks1 = [t if not isinstance(t, tuple) else (t[0], 1) for t in mtoks]
    mtoks2 = [t if not isinstance(t, tuple) else (t[0], 1 + t[1] % 2) for t in mtoks]
    return deep, toks, mix, mtoks1, mtoks2


def good_streams():
    """name -> (stream, the tokens it spells)"""
    deep, toks, mix, mtoks1, mtoks2 = _params()
    one_dist = [1] + [0] * 29
    two_dist = [1, 1] + [0] * 28
    return {
        "deep_literals": (dynamic_block(deep, one_dist, toks), toks),
        "deep_literals_two_dist": (dynamic_block(deep, two_dist, toks), toks),
        "lengths_one_distance": (dynamic_block(mix, one_dist, mtoks1), mtoks1),
        "lengths_two_distances": (dynamic_block(mix, two_dist, mtoks2), mtoks2),
    }


def header_only(litlens, distlens):
    """a dynamic header with these lengths (the tree check rejects it before
    any symbol), followed by a few bytes of padding"""
    w = Bits()
    w.put(1, 1)
    w.put(2, 2)
    w.put(len(litlens) - 257, 5)
    w.put(len(distlens) - 1, 5)
    w.put(19 - 4, 4)
    clens = [4 if s < 16 else 0 for s in range(19)]
    for s in CL_ORDER:
        w.put(clens[s], 3)
    ccode = canonical(clens)
    for ln in list(litlens) + list(distlens):
        w.huff(ccode[ln], 4)
    return w.done() + bytes(8)


def bad_streams():
    deep, toks, mix, mtoks1, mtoks2 = _params()
    one_dist = [1] + [0] * 29
    over = list(deep)
    over[20] = 1                                           # over-subscribed
    incomplete = list(mix)
    incomplete[263] = 0                                    # Kraft sum < 1
    no_eob = [0] * 286
    for b in range(16):
        no_eob[b] = 4
    return {
        "over_subscribed": header_only(over, one_dist),
        "incomplete_litlen": header_only(incomplete, one_dist),
        "no_end_of_block": header_only(no_eob, one_dist),
    }


def spell(tokens):
    out = bytearray()
    for t in tokens:
        if isinstance(t, tuple):
            ln, d = t
            for _ in range(ln):
                out.append(out[-d])
        else:
            out.append(t)
    return bytes(out)


def test_writer_pinned_by_oracle():
    """the crafted streams decode with the oracle to the bytes their tokens
    spell, and the bad trees are rejected by it"""
    for name, (s, toks) in good_streams().items():
        r, err, out, cons = O.inflate(s, 1 << 20)
        assert r == 0 and err == 0 and out == spell(toks) and cons == len(s), (name, r, err)
    for name, s in bad_streams().items():
        r, err, out, cons = O.inflate(s, 1 << 20)
        assert r != 0 and err != 0, (name, r, err)


@pytest.mark.gpu
def test_tables_block_mode(engine):
    """block mode (P1 and its fallbacks) against the oracle, good and bad trees"""
    streams = [v[0] for v in good_streams().values()] + list(bad_streams().values())
    sizes = [len(s) for s in streams]
    g = b"".join(streams)
    assert engine.inflate_blocks(g, sizes) == O.inflate_blocks(g, sizes)


@pytest.mark.gpu
def test_tables_stream_decoders(engine):
    """the one-shot stream decoder and the drop-in stream decoder (32-byte
    and whole-stream pieces, parallel resume on and off) against the oracle"""
    from jdeflate_amd import engine as E
    allst = [(k, v[0]) for k, v in good_streams().items()] + list(bad_streams().items())
    for name, s in allst:
        r, err, out, cons = O.inflate(s, 1 << 20)
        gout, gerr, gused = engine.inflate_stream(s, 1 << 20)
        assert (gout, gerr) == (out, err), name
        for rp in (1, 0):
            for piece in (32, len(s)):
                st = E.IStream()
                st.rpar(rp)
                got, pos, res = bytearray(), 0, None
                for _ in range(100000):
                    res = st.inflate(s[pos:pos + piece], 1 << 20)
                    got += st.out.raw[:res[2]]
                    pos += res[3]
                    if res[0] != E.IS_NEEDINPUT or pos >= len(s):
                        break
                st.close()
                assert bytes(got) == out[:len(got)], (name, rp, piece)
                if r == 0:
                    assert res[0] == E.IS_ENDED and bytes(got) == out, (name, rp, piece)
                else:
                    assert res[0] == E.IS_ERROR and res[1] == err, (name, rp, piece, res)
