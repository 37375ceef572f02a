"""Build the MI355X engine (libovs_kbr.so) and the CPU oracle in-tree.

Product: every HIP translation unit under oversim_amd/csrc is compiled for
gfx950 with hipcc and linked into oversim_amd/libovs_kbr.so (a C-ABI shared
library, include/ovs_kbr.h).  -ffp-contract=off keeps the fp64 delay
arithmetic bit-identical to the reference's x86-64 build.

Rebuilds are decided by content, not mtime: each object carries a stamp with
the hash of its source, every header and the flags, and the library embeds
`ovs_build_id()` = the hash of all engine sources + flags (source_hash()).
kbr.lib() refuses to load a library whose id differs from the sources next to
it, so a tested binary is always the one built from the tree it ships with.

Checker: oracle/ is compiled with gcc into oracle/_build/libovs_oracle.so
(test infrastructure only).
"""
from __future__ import annotations

import hashlib
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
SOURCES = ["chord.hip", "compact.hip", "epichord.hip", "ksort.hip", "kad.hip", "kad_general.hip", "kad_refresh.hip", "kad_route.hip", "kad_shard.hip", "koorde.hip", "stats.hip", "ovs_kbr.cpp", "shard_route.cpp",
           "ovs_ini.cpp", "host_tables.cpp"]
# translation units compiled more than once: (source, object stem, extra flags).  K2 is built per
# (alpha, exact) pair so its instantiations compile in parallel; A = 8 serves alpha 5..8 (A is the
# pending-call capacity, the lookup's alpha is a runtime parameter).
VARIANTS = {
    "kad_route.hip": [(f"kad_route_a{a}{'x' if x else ''}", [f"-DOVS_KAD_A={a}", f"-DOVS_KAD_EX={x}"])
                      for a in (1, 2, 3, 4, 8) for x in (0, 1)],
}


def _engine_files() -> list[Path]:
    return sorted([CSRC / s for s in SOURCES] + list(CSRC.glob("*.hpp")) + [ROOT / "include" / "ovs_kbr.h"])


def _digest(files: list[Path], extra: str) -> str:
    h = hashlib.sha256(extra.encode())
    for f in files:
        h.update(f.relative_to(ROOT).as_posix().encode() + b"\0")
        h.update(f.read_bytes())
        h.update(b"\0")
    return h.hexdigest()[:32]


def source_hash() -> str:
    """Hash of every engine source and header plus the compile flags (= the library's ovs_build_id())."""
    return _digest(_engine_files(), " ".join(CFLAGS))


def _stamp_ok(target: Path, digest: str) -> bool:
    stamp = target.with_name(target.name + ".stamp")
    return target.exists() and stamp.exists() and stamp.read_text() == digest


def _write_stamp(target: Path, digest: str):
    target.with_name(target.name + ".stamp").write_text(digest)


def build_engine(verbose: bool = False) -> Path:
    OBJ.mkdir(parents=True, exist_ok=True)
    headers = sorted(CSRC.glob("*.hpp")) + [ROOT / "include" / "ovs_kbr.h"]
    flags = " ".join(CFLAGS)
    procs = []
    objs = []
    units = [(src, stem, extra) for src in SOURCES
             for stem, extra in VARIANTS.get(src, [(src.rsplit(".", 1)[0], [])])]
    for src, stem, extra in units:
        s = CSRC / src
        o = OBJ / (stem + ".o")
        objs.append(o)
        d = _digest([s] + headers, flags + " " + " ".join(extra))
        if _stamp_ok(o, d):
            continue
        cmd = [HIPCC, *CFLAGS, *extra, "-x", "hip", "-c", str(s), "-o", str(o)]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((cmd, o, d, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    failed = []
    for cmd, o, d, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            failed.append((cmd, out.decode(errors="replace")))
        else:
            _write_stamp(o, d)
            if verbose and out:
                print(out.decode(errors="replace"))
    if failed:
        msg = "\n".join(f"$ {' '.join(c)}\n{o}" for c, o in failed)
        raise RuntimeError(f"hipcc failed:\n{msg}")
    bid = source_hash()
    if not _stamp_ok(LIB, bid):
        # the build id: a one-function translation unit linked into the library
        idsrc = OBJ / "buildid.cpp"
        idsrc.write_text(f'extern "C" const char* ovs_build_id(void) {{ return "{bid}"; }}\n')
        idobj = OBJ / "buildid.o"
        subprocess.run(["g++", "-O2", "-fPIC", "-c", str(idsrc), "-o", str(idobj)], check=True)
        tmp = LIB.with_name(LIB.name + ".tmp")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-o", str(tmp), *map(str, objs), str(idobj)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(tmp, LIB)          # never rewrite a library a running process may have mapped
        _write_stamp(LIB, bid)
    return LIB


C_CONSUMER = ROOT / "tests" / "c_consumer"


def build_c_consumer(verbose: bool = False) -> Path:
    """tests/c_consumer/route_batch: a gcc-built C program against include/ovs_kbr.h, linked to the
    engine library (RUNPATH next to it) -- the ABI as an OverSim-side C/C++ adapter calls it."""
    src, exe = C_CONSUMER / "route_batch.c", C_CONSUMER / "route_batch"
    cmd = ["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-Werror", "-I", str(ROOT / "include"), str(src),
           "-L", str(LIB.parent), "-lovs_kbr", "-Wl,-rpath,$ORIGIN/../../oversim_amd",
           "-Wl,-rpath-link,/opt/rocm/lib", "-o", str(exe)]
    d = _digest([src, ROOT / "include" / "ovs_kbr.h"], " ".join(cmd))
    if not _stamp_ok(exe, d):
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        _write_stamp(exe, d)
    # the sharded route from C: W ranks as pthreads over the library's in-process exchange (device
    # buffers through the HIP runtime API, which is C)
    src2, exe2 = C_CONSUMER / "sharded_route.c", C_CONSUMER / "sharded_route"
    cmd2 = ["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__", "-I", str(ROOT / "include"),
            "-I", "/opt/rocm/include", str(src2), "-L", str(LIB.parent), "-lovs_kbr", "-L", "/opt/rocm/lib", "-lamdhip64",
            "-lpthread", "-Wl,-rpath,$ORIGIN/../../oversim_amd", "-Wl,-rpath,/opt/rocm/lib",
            "-Wl,-rpath-link,/opt/rocm/lib", "-o", str(exe2)]
    d2 = _digest([src2, ROOT / "include" / "ovs_kbr.h"], " ".join(cmd2))
    if not _stamp_ok(exe2, d2):
        if verbose:
            print(" ".join(cmd2), flush=True)
        subprocess.run(cmd2, check=True)
        _write_stamp(exe2, d2)
    return exe


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
    print(build_c_consumer(v))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
