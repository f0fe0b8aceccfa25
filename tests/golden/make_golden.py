"""Generate the golden fixtures under tests/golden/ (committed with this script).

Source of truth: the oracle (oracle/jdoracle.c), a restatement of the
reference codec.  The reference itself cannot be built in this image (it
needs the un-vendored ctoolbox library and a meson-generated config.h), so
these vectors pin the restatement against regressions and serve as the
GPU's parity target; the restatement itself is pinned to the reference by the
known answers in known_answers.json (taken from SURVEY.md's probes of the
reference).  Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import jdoracle as O  # noqa: E402


def inputs():
    rng = np.random.default_rng(20261015)
    words = b"the of and to in is was he for it with as his on be at by had".split()
    text = b" ".join(words[i] for i in rng.integers(0, len(words), 4000))[:16384]
    code = b"".join(b"    if (x%d < %d) { y = f(x%d, %d); }\n" % (i % 7, i % 13, i % 5, i)
                    for i in range(600))[:16384]
    ints = np.cumsum(rng.integers(0, 9, 4096)).astype("<u4").tobytes()
    runs = b"".join(bytes([v]) * int(n) for v, n in zip(rng.choice([0, 1, 255], 400),
                                                          rng.integers(1, 90, 400)))[:16384]
    return {
        "text16k": text,
        "code16k": code,
        "random16k": rng.integers(0, 256, 16384, dtype=np.uint8).tobytes(),
        "ints16k": ints,
        "runs16k": runs,
        "zeros16k": bytes(16384),
        "tail262": text[:262],
        "size0": b"",
        "size1": b"Q",
        "size3": b"abc",
        "size4": b"abca",
        "size258": (b"ab" * 200)[:258],
        "size259": (b"xyz" * 100)[:259],
        "abcdefghij": b"ABCDEFGHIJABCDEFGHIJ",
    }


def main():
    manifest = {"generator": "tests/golden/make_golden.py", "source": "oracle (restatement)",
                "cases": []}
    for name, data in inputs().items():
        with open(os.path.join(HERE, f"in_{name}.bin"), "wb") as f:
            f.write(data)
        for level in (0, 1, 6, 9):
            for flush, fname in ((1, "end"), (2, "flush")):
                out = O.deflate(data, level=level, flush=flush)
                fn = f"out_{name}_L{level}_{fname}.bin"
                with open(os.path.join(HERE, fn), "wb") as f:
                    f.write(out)
                manifest["cases"].append({
                    "input": f"in_{name}.bin", "level": level, "flush": fname, "output": fn,
                    "in_sha256": hashlib.sha256(data).hexdigest(),
                    "out_sha256": hashlib.sha256(out).hexdigest(), "out_size": len(out)})
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(f"{len(manifest['cases'])} cases written")


if __name__ == "__main__":
    main()
