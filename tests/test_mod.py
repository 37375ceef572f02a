"""The snapshot builders' Floyd draws take hash % (j + 1) through an exact fp64-reciprocal remainder
(oversim_amd/csrc/kad_dev.hpp mod_u64_u32, two steps); the tables stay bit-identical only if it
equals the integer %.  Built for the host with hipcc (the __host__ __device__ function itself) and
checked on edge cases and 3e7 seeded random (dividend, divisor) pairs."""
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
HIPCC = Path("/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not HIPCC.exists(), reason="hipcc not installed")
def test_mod_u64_u32_equals_integer_remainder(tmp_path):
    exe = tmp_path / "mod_check"
    subprocess.run([str(HIPCC), "-O2", "-std=c++17", "-ffp-contract=off", f"-I{ROOT / 'oversim_amd' / 'csrc'}",
                    f"-I{ROOT / 'include'}", str(ROOT / "tests" / "host" / "mod_check.hip"), "-o", str(exe)],
                   check=True, capture_output=True)
    r = subprocess.run([str(exe), "10000000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout
