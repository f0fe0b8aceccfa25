"""k_chains files positions with ds_mskor_rtn_b32 (the block-mode slices:
ds_add_rtn_u32 on the bucket counts) through inline asm and
waits for all 16 results with one explicit `s_waitcnt lgkmcnt(0)`
(jd_deflate.hip, stage B).  The compiler does not know those results arrive
late, so nothing between an exchange and that wait may read or copy its
result register; a copy would pass on garbage and corrupt the chains.  This
checks the shipped gfx950 code object of the built library (CPU only:
llvm-objcopy / clang-offload-bundler / llvm-objdump, no GPU)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "jdeflate_amd", "lib", "libjdeflate_amd.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
XCHG = ("ds_mskor_rtn_b32", "ds_add_rtn_u32")


def tool(name):
    p = os.path.join(LLVM, name)
    return p if os.path.exists(p) else shutil.which(name)


def disassemble(tmp_path):
    objcopy, bundler, objdump = tool("llvm-objcopy"), tool("clang-offload-bundler"), tool("llvm-objdump")
    if not (objcopy and bundler and objdump) or not os.path.exists(LIB):
        pytest.skip("llvm tools or the built library missing")
    fat = tmp_path / "fat.bin"
    subprocess.run([objcopy, "--dump-section", f".hip_fatbin={fat}", LIB], check=True)
    data = fat.read_bytes()
    starts = []
    i = data.find(MAGIC)
    while i >= 0:
        starts.append(i)
        i = data.find(MAGIC, i + 1)
    text = []
    for k, s in enumerate(starts):
        part = tmp_path / f"b{k}.bin"
        part.write_bytes(data[s:starts[k + 1] if k + 1 < len(starts) else len(data)])
        co = tmp_path / f"b{k}.o"
        r = subprocess.run([bundler, "--unbundle", "--type=o",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                            f"--input={part}", f"--output={co}"], capture_output=True)
        if r.returncode or not co.exists() or co.stat().st_size == 0:
            continue
        text.append(subprocess.run([objdump, "-d", "--no-show-raw-insn", str(co)],
                                   capture_output=True, text=True, check=True).stdout)
    return "\n".join(text)


def functions(dis):
    cur, out = None, {}
    for line in dis.split("\n"):
        if line.endswith(">:") and "<" in line:
            cur = line[line.index("<") + 1:-2]
            out[cur] = []
        elif cur is not None:
            ins = line.split("//")[0].strip()
            if ins:
                out[cur].append(ins)
    return out


def hazards(ins):
    """(sequences, violations): each run of exchanges up to the next
    lgkmcnt(0) wait, and any instruction there naming a pending result"""
    seqs, bad, i = 0, [], 0
    while i < len(ins):
        if not ins[i].startswith(XCHG):
            i += 1
            continue
        seqs += 1
        pending = set()
        while i < len(ins) and not (ins[i].startswith("s_waitcnt") and "lgkmcnt(0)" in ins[i]):
            ops = ins[i].replace(",", " ").split()
            if ops[0] in XCHG:
                pending.add(ops[1])
            elif any(r in pending for r in ops[1:]):
                bad.append(ins[i])
            i += 1
    return seqs, bad


def test_chains_exchange_results_untouched_before_wait(tmp_path):
    fns = functions(disassemble(tmp_path))
    chains = {k: v for k, v in fns.items() if "k_chains" in k}
    assert len(chains) >= 2, sorted(fns)[:20]
    for name, ins in chains.items():
        seqs, bad = hazards(ins)
        assert seqs >= 1, name
        assert not bad, (name, bad[:5])


def test_hazard_checker_flags_a_copy():
    ins = ["ds_mskor_rtn_b32 v4, v1, v2, v3", "ds_mskor_rtn_b32 v5, v1, v2, v3",
           "v_mov_b32_e32 v9, v4", "s_waitcnt lgkmcnt(0)", "v_mov_b32_e32 v8, v5"]
    assert hazards(ins) == (1, ["v_mov_b32_e32 v9, v4"])


def test_hazard_checker_flags_a_count_copy():
    ins = ["ds_add_rtn_u32 v4, v1, v2", "v_add_u32_e32 v9, v4, v1", "s_waitcnt lgkmcnt(0)"]
    assert hazards(ins) == (1, ["v_add_u32_e32 v9, v4, v1"])
