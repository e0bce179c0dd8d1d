"""Checks on the product library's gfx950 code object (no GPU needed).

The scans take work with an inline-asm returning atomic (grab_async,
syncr_amd/csrc/cdc_kernels.hip) whose result register is read only after a
later `s_waitcnt vmcnt(0)`.  hipcc's waitcnt insertion cannot see memory
operations inside inline asm, so the code is correct only while the register
allocator leaves that register alone until the wait: a copy, spill or
rematerialisation of it in between would read the register before the atomic
returned, and the scan would silently skip or repeat work.  These tests
disassemble the shipped code object and follow every control-flow path from
each such atomic to its wait, and check that no product kernel
spills VGPRs to scratch.
"""
import os
import re
import shutil
import subprocess

import pytest

LLVM = "/opt/rocm/lib/llvm/bin"
# the kernels that carry grab_async, by mangled-name prefix
GRAB_KERNELS = ("_ZN3cdc18cdc_scan_st_kernel", "_ZN3cdc15cdc_scan_kernelILi144ELi28ELi1E")
CTR_OFFSET = "offset:12"          # CTR_CANDS_HI * 4: the grab's counter word


def _tools():
    for t in ("clang-offload-bundler", "llvm-objdump", "llvm-readelf"):
        if not os.path.exists(os.path.join(LLVM, t)):
            pytest.skip(f"{t} not available")
    if not shutil.which("objcopy"):
        pytest.skip("objcopy not available")


@pytest.fixture(scope="module")
def code_objects(tmp_path_factory):
    """The gfx950 code object of every translation unit of the product library
    (the .hip_fatbin section holds one offload bundle per .hip source)."""
    _tools()
    from syncr_amd import build as B
    lib = B.build()
    d = tmp_path_factory.mktemp("co")
    fat = str(d / "fatbin.bin")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fat], check=True)
    blob = open(fat, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), blob)]
    cos = []
    for k, a in enumerate(starts):
        part, co = str(d / f"part{k}.bin"), str(d / f"dev{k}.co")
        open(part, "wb").write(blob[a: starts[k + 1] if k + 1 < len(starts) else len(blob)])
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={part}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        cos.append(co)
    assert len(cos) >= 2                       # cdc_kernels.hip, b3_kernels.hip
    return cos


@pytest.fixture(scope="module")
def code_object(code_objects):
    """The code object holding the scans."""
    for co in code_objects:
        if any("cdc_scan_st_kernel" in n for n in _kernels(co)):
            return co
    pytest.fail("no code object holds cdc_scan_st_kernel")


def _kernels(co):
    """{mangled name: [(address, text)]} from llvm-objdump -d."""
    out = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", co], capture_output=True, text=True,
                         check=True).stdout
    ks, cur = {}, None
    for line in out.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = ks.setdefault(m.group(1), [])
            continue
        m = re.match(r"^\s+(\S.*?)\s*// ([0-9A-F]{12}):", line)
        if cur is not None and m:
            cur.append((int(m.group(2), 16), m.group(1)))
    return ks


def _vregs(text):
    """VGPR numbers an instruction names (v7, v[4:7])."""
    regs = set()
    for a, b in re.findall(r"\bv\[(\d+):(\d+)\]", text):
        regs.update(range(int(a), int(b) + 1))
    regs.update(int(x) for x in re.findall(r"\bv(\d+)\b", text))
    return regs


def _branch_target(addr, text):
    m = re.match(r"s_(?:c)?branch\w*\s+(-?\d+)", text)
    return addr + 4 + 4 * int(m.group(1)) if m else None


def _grab_paths_ok(insns, k):
    """Follow every path from the atomic at insns[k] to a `s_waitcnt vmcnt(0)`:
    returns (ok, what) -- ok False if an instruction on a path names the
    atomic's result register first."""
    vdst = int(re.match(r"global_atomic_add v(\d+),", insns[k][1]).group(1))
    index = {a: i for i, (a, _) in enumerate(insns)}
    todo, seen = [k + 1], set()
    while todo:
        i = todo.pop()
        while i < len(insns) and i not in seen:
            seen.add(i)
            addr, text = insns[i]
            op = text.split()[0]
            if op == "s_waitcnt" and "vmcnt(0)" in text:
                break
            if vdst in _vregs(text):
                return False, f"{addr:#x}: {text} reads/writes v{vdst} before the wait"
            if op in ("s_endpgm", "s_setpc_b64"):
                break
            tgt = _branch_target(addr, text)
            if op == "s_branch":
                i = index.get(tgt, len(insns))
                continue
            if tgt is not None:                      # conditional: both ways
                todo.append(index.get(tgt, len(insns)))
            i += 1
    return True, ""


def test_grab_result_untouched_until_wait(code_object):
    ks = _kernels(code_object)
    checked = 0
    for prefix in GRAB_KERNELS:
        names = [n for n in ks if n.startswith(prefix)]
        assert names, f"kernel {prefix}* not in the product code object"
        for n in names:
            insns = ks[n]
            grabs = [i for i, (_, t) in enumerate(insns)
                     if t.startswith("global_atomic_add") and CTR_OFFSET in t and " sc0" in t]
            assert grabs, f"{n}: no returning grab atomic found"
            for g in grabs:
                ok, what = _grab_paths_ok(insns, g)
                assert ok, f"{n}: {what}"
                checked += 1
    assert checked >= 2


def test_kernels_spill_no_vgprs(code_objects):
    """No product kernel spills VGPRs to scratch (the scans: the grab invariant
    above; the hash leaf: it runs at its 128-VGPR cap)."""
    spills = {}
    for co in code_objects:
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], capture_output=True,
                               text=True, check=True).stdout
        name = None
        for line in notes.splitlines():
            m = re.match(r"\s+\.name:\s+(\S+)", line)
            if m:
                name = m.group(1)
            m = re.match(r"\s+\.vgpr_spill_count:\s+(\d+)", line)
            if m and name:
                spills[name] = int(m.group(1))
    assert any("cdc_scan" in n for n in spills) and any("b3_leaf" in n for n in spills), sorted(spills)
    assert all(c == 0 for c in spills.values()), {n: c for n, c in spills.items() if c}


def test_checker_catches_an_early_read():
    """The path walk itself: a copy of the result before the wait, on the
    taken side of a branch, is reported; the same copy after the wait is not."""
    insns = [(0x0, "global_atomic_add v9, v1, v2, s[4:5] offset:12 sc0"),
             (0x8, "s_cbranch_scc1 2"),
             (0xC, "s_waitcnt vmcnt(0)"),
             (0x10, "s_endpgm"),
             (0x14, "v_mov_b32_e32 v3, v9"),
             (0x18, "s_waitcnt vmcnt(0)")]
    ok, what = _grab_paths_ok(insns, 0)
    assert not ok and "0x14" in what
    insns[4], insns[5] = (0x14, "s_waitcnt vmcnt(0)"), (0x18, "v_mov_b32_e32 v3, v9")
    assert _grab_paths_ok(insns, 0)[0]
