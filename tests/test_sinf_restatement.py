"""lo::sincosf_ref (lo_math.h), the device's sin / cos of SO3::Exp's rotation angle (MathUtils.cpp:23-39 calls
std::sin / std::cos on a float: glibc's sinf / cosf) against the host's glibc sinf / cosf, bit for bit.  Compiled on the
host from the same header the kernels include (scripts/check_sinf_ref.cpp); the full sweep (every float in (1e-7, 120)
and its negative, 5.1e8 arguments, ~20 s) matched with zero mismatches -- this test runs every 13th float."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_sincosf_ref_equals_glibc(tmp_path):
    exe = str(tmp_path / "check_sinf_ref")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17",
                    os.path.join(ROOT, "scripts", "check_sinf_ref.cpp"), "-o", exe], check=True)
    p = subprocess.run([exe, "13"], capture_output=True, text=True)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "sinf_mismatch=0 cosf_mismatch=0" in p.stdout, p.stdout
