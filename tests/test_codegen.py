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


@pytest.mark.skipif(not os.path.exists(OBJDUMP), reason="llvm-objdump (ROCm) not installed")
@pytest.mark.parametrize("lib", [_ffi.PRODUCT_LIB_PATH, _ffi.DIAG_LIB_PATH], ids=["product", "diag"])
def test_no_unsaved_exec_narrowing(tmp_path, lib):
    if not os.path.exists(lib):
        pytest.skip(f"{os.path.basename(lib)} not built")
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
        bad += [ln.strip() for ln in dis.splitlines() if "s_and_b64 exec, exec, s[" in ln]
    assert not bad, f"{len(bad)} exec narrowings without a saved mask, e.g. {bad[:3]}"
