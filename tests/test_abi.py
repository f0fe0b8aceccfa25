"""The C-ABI library: builds for gfx950, exports every symbol the public
headers declare, keeps the reference's struct layout, compiles against the
drop-in headers, and has no CPU fallback.  No GPU needed."""
import ctypes
import glob
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")


def declared_symbols():
    names = set()
    for h in glob.glob(os.path.join(INC, "jdeflate", "**", "*.h"), recursive=True):
        src = open(h).read()
        for m in re.finditer(r"^\s*JDEFLATE_API\s+[^;(#]*?\b(\w+)\s*\(", src, re.M):
            names.add(m.group(1))
    return names


def test_headers_declare_the_reference_api():
    d = declared_symbols()
    ref = {"deflator_create", "deflator_destroy", "deflator_reset", "deflator_deflate",
           "deflator_setdctnr", "inflator_create", "inflator_destroy", "inflator_reset",
           "inflator_inflate", "inflator_setdctnr"}
    assert ref <= d, ref - d


def test_library_exports_every_declared_symbol(built_lib):
    out = subprocess.run(["nm", "-D", "--defined-only", built_lib], capture_output=True,
                         text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    missing = declared_symbols() - exported
    assert not missing, missing
    import jdeflate_amd as J
    L = J.load_library()
    for s in J.EXPORTS:
        assert hasattr(L, s), s


def test_only_api_symbols_exported(built_lib):
    out = subprocess.run(["nm", "-D", "--defined-only", built_lib], capture_output=True,
                         text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert exported <= declared_symbols(), exported - declared_symbols()


def test_gfx950_code_object(built_lib):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list",
                          "--type=o", f"--input={built_lib}"], capture_output=True, text=True)
    data = open(built_lib, "rb").read()
    assert b"gfx950" in data


def test_struct_layout_is_abi():
    import jdeflate_amd.engine as E
    assert ctypes.sizeof(E._Public) == 72    # deflator.h:81-99 on LP64


def test_dropin_program_compiles_and_links(built_lib, tmp_path):
    prog = tmp_path / "dropin.c"
    prog.write_text(r'''
#include <jdeflate/deflator.h>
#include <jdeflate/inflator.h>
#include <jdeflate/jdgpu.h>
#include <stdio.h>
int main(void) {
    struct JDEFLATEVersion v = jdeflate_getversion();
    TDeflator* d = deflator_create(0, 6, NULL);
    TInflator* i = inflator_create(0, NULL);
    printf("%d %d %d %s %d %d\n", (int) sizeof(TDeflator), (int) sizeof(TInflator),
           jdgpu_available(), v.versionstring, d != NULL, i != NULL);
    deflator_destroy(d);
    inflator_destroy(i);
    return 0;
}
''')
    exe = tmp_path / "dropin"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", INC, str(prog), "-o", str(exe),
                    "-L", os.path.dirname(built_lib), "-ljdeflate_amd",
                    "-Wl,-rpath," + os.path.dirname(built_lib)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, check=True)
    f = r.stdout.split()
    assert f[0] == "72" and f[1] == "72" and f[3].startswith("0.4.0")
    import jdeflate_amd as J
    if not J.available():
        # no GPU: the product refuses to run rather than fall back to a CPU codec
        assert f[2] == "0" and f[4] == "0" and f[5] == "0"


def test_no_cpu_fallback_without_gpu(built_lib):
    import jdeflate_amd as J
    if J.available():
        pytest.skip("GPU present")
    with pytest.raises(J.EngineUnavailable):
        J.deflate_blocks(b"hello")
    with pytest.raises(J.EngineUnavailable):
        J.Deflator(6)
    L = J.load_library()
    assert L.jdgpu_deflate(b"abc", 3, 65536, 6, 0, 1, ctypes.create_string_buffer(64), 64,
                           None) == J.engine.JDGPU_ENODEV
    # the multi-device entry points refuse too (no device list to drive)
    assert L.jdgpu_deflate_multi(b"abc", 3, 65536, 6, 0, 1, ctypes.create_string_buffer(64), 64,
                                 None, 0, None) == J.engine.JDGPU_ENODEV
    us = (ctypes.c_uint32 * 1)()
    er = (ctypes.c_int32 * 1)()
    assert L.jdgpu_inflate_multi(b"abc", 3, (ctypes.c_uint32 * 1)(3), 1, 65536,
                                 ctypes.create_string_buffer(65536), us, er, 0,
                                 None) == J.engine.JDGPU_ENODEV


def test_bound(built_lib):
    import jdeflate_amd as J
    assert J.bound(0) >= 5
    assert J.bound(65536) >= 65536 * 2
    assert J.bound(65537) == 2 * J.bound(65536)
    assert J.bound(100, 17) == 0            # block size must be a multiple of 16


def test_bench_finds_committed_pmc_traffic():
    """the bench line's roofline.traffic comes from the committed PMC summary
    of the default workload (C2+C3: 1 GiB text, level 6); the dominant
    kernel's entry must be found under its templated name"""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    t, src = bench.pmc_traffic("k_match", 6, 1 << 30)
    assert t and t > 0 and src.startswith("profiles/pmc_summary"), (t, src)
