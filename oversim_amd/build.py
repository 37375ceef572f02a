"""Build the MI355X engine (libovs_kbr.so) and the CPU oracle in-tree.

Product: every HIP translation unit under oversim_amd/csrc is compiled for
gfx950 with hipcc and linked into oversim_amd/libovs_kbr.so (a C-ABI shared
library, include/ovs_kbr.h).  -ffp-contract=off keeps the fp64 delay
arithmetic bit-identical to the reference's x86-64 build.

Checker: oracle/ is compiled with gcc into oracle/_build/libovs_oracle.so
(test infrastructure only).
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "oversim_amd" / "csrc"
OBJ = ROOT / "build" / "obj"
LIB = ROOT / "oversim_amd" / "libovs_kbr.so"
ORACLE = ROOT / "oracle"

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("OVS_OFFLOAD_ARCH", "gfx950")
CFLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off",
    "-Wall", "-Wno-unused-function", "-Wno-unused-result", "-Wno-unused-value", "-Wno-bitwise-instead-of-logical",
]
SOURCES = ["chord.hip", "kad.hip", "kad_shard.hip", "stats.hip", "ovs_kbr.cpp", "ovs_ini.cpp"]


def _newer(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build_engine(verbose: bool = False) -> Path:
    OBJ.mkdir(parents=True, exist_ok=True)
    headers = sorted(CSRC.glob("*.hpp")) + [ROOT / "include" / "ovs_kbr.h"]
    procs = []
    objs = []
    for src in SOURCES:
        s = CSRC / src
        o = OBJ / (src.rsplit(".", 1)[0] + ".o")
        objs.append(o)
        if not _newer(o, [s] + headers):
            continue
        cmd = [HIPCC, *CFLAGS, "-x", "hip", "-c", str(s), "-o", str(o)]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    failed = []
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            failed.append((cmd, out.decode(errors="replace")))
        elif verbose and out:
            print(out.decode(errors="replace"))
    if failed:
        msg = "\n".join(f"$ {' '.join(c)}\n{o}" for c, o in failed)
        raise RuntimeError(f"hipcc failed:\n{msg}")
    if _newer(LIB, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-o", str(LIB), *map(str, objs)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return LIB


def build_oracle(verbose: bool = False) -> Path:
    cmd = ["make", "-s", "-C", str(ORACLE)]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return ORACLE / "_build" / "libovs_oracle.so"


def main() -> int:
    v = "-v" in sys.argv
    print(build_engine(v))
    print(build_oracle(v))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
