"""ASan + UBSan build of the CPU restatement (oracle/ovs_oracle.c) and the host-side .ini binder
(oversim_amd/csrc/ovs_ini.cpp), compiled with -Wall -Wextra -Werror and run on small networks
through every oracle entry point (tests/sanitize_driver.cpp).  SURVEY.md §5: sanitizers run on the
host code; GPU code is checked by the parity tests.  CPU only."""
from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-g", "-O1"]
WARN = ["-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter"]


@pytest.mark.skipif(shutil.which("gcc") is None or shutil.which("g++") is None, reason="needs gcc/g++")
def test_oracle_and_ini_binder_clean_under_asan_ubsan(tmp_path):
    objs = []
    cmds = [
        ["gcc", "-std=gnu11", "-fopenmp", "-ffp-contract=off", *SAN, *WARN, "-c", str(ROOT / "oracle" / "ovs_oracle.c"),
         "-o", str(tmp_path / "oracle.o")],
        ["g++", "-std=c++17", *SAN, *WARN, "-c", str(ROOT / "oversim_amd" / "csrc" / "ovs_ini.cpp"),
         "-o", str(tmp_path / "ini.o")],
        ["g++", "-std=c++17", *SAN, *WARN, "-c", str(ROOT / "tests" / "sanitize_driver.cpp"),
         "-o", str(tmp_path / "driver.o")],
    ]
    for c in cmds:
        r = subprocess.run(c, capture_output=True, text=True)
        assert r.returncode == 0, f"{' '.join(c)}\n{r.stdout}{r.stderr}"
        objs.append(c[-1])
    exe = tmp_path / "sanitize_driver"
    r = subprocess.run(["g++", "-fopenmp", *SAN, *objs, "-o", str(exe), "-lm"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    # the environment is passed through unchanged (a preloaded library may precede the ASan runtime)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1",
               OMP_NUM_THREADS="2")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and "clean" in r.stdout, r.stdout[-3000:] + r.stderr[-6000:]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_table_bookkeeping_clean_under_asan_ubsan(tmp_path):
    """The C ABI's host-side table code (oversim_amd/csrc/host_tables.cpp: explicit Chord tables, the
    fixfingers and stabilize rounds' updates, EpiChord snapshot validation and ordering) built with
    plain g++ under ASan/UBSan -Werror and driven through a converging ring and broken inputs
    (tests/host_tables_driver.cpp)."""
    inc = ["-I", str(ROOT / "oversim_amd" / "csrc")]
    objs = []
    for src, o in ((ROOT / "oversim_amd" / "csrc" / "host_tables.cpp", "ht.o"),
                   (ROOT / "tests" / "host_tables_driver.cpp", "drv.o")):
        c = ["g++", "-std=c++17", *SAN, *WARN, *inc, "-c", str(src), "-o", str(tmp_path / o)]
        r = subprocess.run(c, capture_output=True, text=True)
        assert r.returncode == 0, f"{' '.join(c)}\n{r.stdout}{r.stderr}"
        objs.append(str(tmp_path / o))
    exe = tmp_path / "host_tables_driver"
    r = subprocess.run(["g++", *SAN, *objs, "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and "clean" in r.stdout, r.stdout[-3000:] + r.stderr[-6000:]
