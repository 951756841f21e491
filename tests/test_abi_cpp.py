"""The C ABI from C++ (VERDICT r01 "a C++ test that calls the ABI directly, with static_asserts on floam_point
offsets"): tests/abi_check.cpp is compiled with the host g++ against include/floam_c.h and linked with
libfloam_amd.so, as a reference node / adapter would be, then run."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "floam_amd", "libfloam_amd.so")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_abi_from_cpp(tmp_path):
    if not os.path.exists(LIB):
        pytest.fail("libfloam_amd.so is not built (python -c 'import __graft_entry__ as g; g.build()')")
    exe = tmp_path / "abi_check"
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "abi_check.cpp"), "-o", str(exe), "-L", os.path.dirname(LIB),
                    "-lfloam_amd", "-Wl,-rpath," + os.path.dirname(LIB)], check=True)
    import torch
    mode = "device" if torch.cuda.is_available() else "nodevice"
    out = tmp_path / "out"
    out.mkdir()
    r = subprocess.run([str(exe), str(out), mode], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "abi_check ok" in r.stdout
