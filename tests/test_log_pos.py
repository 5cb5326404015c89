"""lo::log_pos (lo_math.h), the log of the PKO JS terms (AdaptiveMEstimator.cpp calculate_js_divergence): <= 1 ulp
from glibc log over log-uniform and near-1 samples, and log's special values (0, inf, NaN, negative, denormals).
Compiled on the host from the same header the kernels include (scripts/check_log_pos.cpp)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_log_pos_within_one_ulp(tmp_path):
    exe = str(tmp_path / "check_log_pos")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17",
                    os.path.join(ROOT, "scripts", "check_log_pos.cpp"), "-o", exe], check=True)
    p = subprocess.run([exe, "3000000"], capture_output=True, text=True)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "worst=0" in p.stdout or "worst=1" in p.stdout, p.stdout
