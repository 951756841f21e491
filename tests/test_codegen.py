"""Code-generation guard (CPU): the libraries' gfx950 code objects never narrow exec without saving the mask.

LLVM's removal of "redundant" end-of-if exec restores lowers a divergent if that ends where an enclosing one ends to
`s_and_b64 exec, exec, s[..]` with no saved mask; register copies the allocator then places at the join run under the
inner mask, and the lanes outside it keep stale values.  That corrupted the LM solve once (DESIGN.md §4,
profiles/r05m); floam_amd/csrc/Makefile compiles with -mllvm -amdgpu-remove-redundant-endcf=false so the pattern
cannot appear.  This test disassembles the built product and diagnostic libraries (the GPU tests load both) and
fails if it does (e.g. a build without the flag).
"""
import glob
import os
import shutil
import subprocess

import pytest

from floam_amd import _ffi

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


import re

NARROW = re.compile(r"s_and_b64 exec, exec, (vcc|s\[)")   # exec narrowed without saving the mask
HIPCC = "/opt/rocm/bin/hipcc"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("lib", [_ffi.PRODUCT_LIB_PATH, _ffi.DIAG_LIB_PATH], ids=["product", "diag"])
def test_no_unsaved_exec_narrowing(tmp_path, lib):
    # no skip: a library that cannot be checked (not built, no ROCm disassembler) fails the suite (VERDICT r05 Weak 9)
    assert os.path.exists(OBJDUMP), "llvm-objdump (ROCm) is needed to check the code objects"
    assert os.path.exists(lib), f"{os.path.basename(lib)} not built (floam_amd/csrc: make)"
    name = os.path.basename(lib)
    local = tmp_path / name
    shutil.copy(lib, local)
    # --offloading writes every embedded code object beside its input (here: the temporary copy)
    subprocess.run([OBJDUMP, "--offloading", str(local)], check=True, capture_output=True, cwd=tmp_path)
    objs = sorted(glob.glob(str(tmp_path / f"{name}.*gfx950")))
    assert len(objs) >= 10, objs   # one per HIP source
    bad = []
    for o in objs:
        dis = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", o], check=True, capture_output=True, text=True).stdout
        assert "s_and_saveexec_b64" in dis or "v_" in dis   # (a real disassembly)
        bad += [ln.strip() for ln in dis.splitlines() if NARROW.search(ln)]
    assert not bad, f"{len(bad)} exec narrowings without a saved mask, e.g. {bad[:3]}"


def test_endcf_reproducer(tmp_path):
    """tools/micro/endcf_repro.hip: the nested-if shape of lm_solve's write-back.  The default LLVM pipeline narrows
    exec without saving the mask there (the compiler's transformation: the source has no divergence hazard); the
    Makefile's -amdgpu-remove-redundant-endcf=false keeps the inner if's own save / restore."""
    assert os.path.exists(HIPCC)
    src = os.path.join(ROOT, "tools", "micro", "endcf_repro.hip")
    counts = {}
    for name, extra in (("default", []), ("flag", ["-mllvm", "-amdgpu-remove-redundant-endcf=false"])):
        out = tmp_path / f"{name}.s"
        subprocess.run([HIPCC, "-O3", "--offload-arch=gfx950", "--offload-device-only", "-S", *extra, src, "-o",
                        str(out)], check=True, capture_output=True)
        asm = out.read_text()
        counts[name] = (len(NARROW.findall(asm)), asm.count("s_and_saveexec_b64"))
    assert counts["default"][0] >= 1, counts   # the unsaved narrowing appears without the flag
    assert counts["flag"][0] == 0 and counts["flag"][1] >= 2, counts   # both ifs save and restore with it
