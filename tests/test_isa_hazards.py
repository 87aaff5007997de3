"""
Static check of the shipped gfx950 code (CPU only): no vector-memory store of more than 8 bytes is followed
at once by a VALU instruction that overwrites one of its data VGPRs.

Why: a buffer store of > 8 bytes reads its data VGPRs after it issues.  LLVM's hazard recognizer inserts the
wait state before a VALU write of those registers for FLAT / global stores and for MUBUF stores whose soffset
is a constant, but not for MUBUF stores with an SGPR soffset (GCNHazardRecognizer::createsVALUHazard).  On
the MI355X that exemption does not hold: the fp64 in-LDS FFT's fast store (`buffer_store_dwordx4 v[0:3], ...,
s2 offen` followed by `v_add_u32 v0, ...`) wrote, now and then, the next LDS address into the low dword of an
fp64 result -- the intermittent 4e-10 / 5e-10 failures of
test_fft_vs_numpy[(2048, 2048)-(0, 1)-float64-True] in rounds 4 and 5 (16 values of one row, low dwords
0xd940..0xdc30, high dwords exact).  csrc/fft.hip now gives those stores a constant soffset;
this test pins that no kernel of the library ships the pattern again.
"""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

LLVM = "/opt/rocm/lib/llvm/bin/llvm-objdump"
LIB = os.path.join(ROOT, "pyxu_amd", "libpyxu_amd.so")


def _code_objects(tmp_path):
    lib = tmp_path / "lib.so"
    shutil.copy(LIB, lib)  # llvm-objdump --offloading writes the bundles next to its input
    subprocess.run([LLVM, "--offloading", str(lib)], check=True, capture_output=True, cwd=tmp_path)
    return sorted(p for p in tmp_path.iterdir() if "amdgcn-amd-amdhsa--gfx950" in p.name)


def _vgprs(op):
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"v(\d+)", op)
    return {int(m.group(1))} if m else set()


def store_data_hazards(lines):
    """(store, next) pairs where a > 8-byte buffer / global / flat store's data VGPRs are written by the very next
    VALU instruction (disassembly lines of one code object)."""
    ins = []
    for ln in lines:
        t = ln.split("//")[0].strip()
        if t and not t.endswith(":") and not t.startswith((".", ";", "<")) and re.match(r"[a-z_0-9]+\s", t + " "):
            ins.append(t)
    out = []
    for i, t in enumerate(ins[:-1]):
        op, _, rest = t.partition(" ")
        if not re.fullmatch(r"(buffer|global|flat)_store_dwordx[34]|(buffer|global|flat)_store_b(96|128)", op):
            continue
        args = [a.strip() for a in rest.split(",")]
        data = _vgprs(args[1] if op.startswith(("global", "flat")) else args[0])
        nxt = ins[i + 1]
        nop, _, nrest = nxt.partition(" ")
        if nop.startswith("v_") and not nop.startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
            dst = nrest.split(",")[0].strip()
            if _vgprs(dst) & data:
                out.append((t, nxt))
    return out


def test_hazard_checker_flags_the_round4_pattern():
    bad = ["buffer_store_dwordx4 v[0:3], v12, s[4:7], s2 offen", "v_add_u32_e32 v0, s8, v13"]
    ok = ["buffer_store_dwordx4 v[0:3], v12, s[4:7], 0 offen", "s_nop 0", "v_add_u32_e32 v0, s8, v13"]
    addr = ["global_store_dwordx4 v[4:5], v[8:11], off", "v_lshrrev_b32_e32 v4, 3, v1"]  # address, not data
    assert len(store_data_hazards(bad)) == 1
    assert store_data_hazards(ok) == [] and store_data_hazards(addr) == []


@pytest.mark.skipif(not (os.path.exists(LLVM) and os.path.exists(LIB)), reason="needs the ROCm toolchain and the built library")
def test_no_store_data_hazard_in_shipped_kernels(tmp_path):
    objs = _code_objects(tmp_path)
    assert objs, "no gfx950 code object found in libpyxu_amd.so"
    found = []
    for co in objs:
        dis = subprocess.run([LLVM, "-d", "--mcpu=gfx950", str(co)], check=True, capture_output=True, text=True).stdout
        found += [(co.name, s, n) for s, n in store_data_hazards(dis.splitlines())]
    assert not found, found[:8]


def _kernel_notes(tmp_path):
    """(name, metadata text) of every kernel in the library's gfx950 code objects."""
    out = []
    for co in _code_objects(tmp_path):
        notes = subprocess.run([LLVM.replace("llvm-objdump", "llvm-readelf"), "--notes", str(co)], check=True,
                               capture_output=True, text=True).stdout
        for ent in re.split(r"\n\s+- \.agpr_count:", notes):
            m = re.search(r"\.name:\s+(\S+)", ent)
            if m:
                out.append((m.group(1), ent))
    return out


@pytest.mark.skipif(not (os.path.exists(LLVM) and os.path.exists(LIB)), reason="needs the ROCm toolchain and the built library")
def test_hot_kernels_do_not_spill(tmp_path):
    """The PGD tile kernel (fp32, radius 6: the headline), the fp32 radius-6 look-ahead PDS kernels and the dense normal
    operator keep their registers: a scratch spill there costs more than any of their round-5 A/B variants won
    (a shared helper once pulled 64 extra VGPRs into the tile kernel's tail and spilled 14).  SGPR spills, which
    land in VGPR lanes, not in memory, are allowed (kernel D has 10-14)."""
    hot = ("pgd_tv2d_kernelIfLi6", "pds_march_kernelIfLi6", "pds_plane_kernelIfLi6", "normal_group_kernel")
    seen = {}
    for name, ent in _kernel_notes(tmp_path):
        for h in hot:
            if h in name:
                v = re.search(r"\.vgpr_spill_count:\s+(\d+)", ent)
                sg = re.search(r"\.sgpr_spill_count:\s+(\d+)", ent)
                seen[name] = (int(v.group(1)) if v else 0, int(sg.group(1)) if sg else 0)
    assert any("pgd_tv2d_kernelIfLi6" in n for n in seen), "tile kernel not found"
    spilled = {n[:80]: v for n, v in seen.items() if v[0] != 0}  # VGPR spills go to scratch memory
    assert not spilled, spilled
