"""The C ABI as a C compiler sees it: tests/abi_layout.c is built with gcc -std=c99 against
include/ovs_kbr.h alone and prints sizeof/offsetof of every ABI struct; each must match the
Python mirrors the bindings read and write through (ctypes structures in oversim_amd/kbr.py,
numpy record dtypes in oversim_amd/kbr.py and oversim_amd/shard.py).  A field-order drift
between the header and a binding fails here instead of silently corrupting parameters."""
from __future__ import annotations

import ctypes as C
import json
import subprocess
from pathlib import Path

import numpy as np
import pytest

from oversim_amd import kbr, shard

ROOT = Path(__file__).resolve().parent.parent


@pytest.fixture(scope="module")
def layout(tmp_path_factory):
    exe = tmp_path_factory.mktemp("abi") / "abi_layout"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-I", str(ROOT / "include"),
                    str(ROOT / "tests" / "abi_layout.c"), "-o", str(exe)], check=True)
    return json.loads(subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout)


CTYPES = {
    "ovs_params": kbr.Params,
    "ovs_stddev": kbr.StdDev,
    "ovs_kbrtest_stats": kbr.KbrTestStats,
    "ovs_kbrtest_lookup_stats": kbr.KbrTestLookupStats,
    "ovs_fixfingers_stats": kbr.FixFingersStats,
    "ovs_stabilize_stats": kbr.StabilizeStats,
}

DTYPES = {
    "ovs_route_out": kbr.ROUTE_OUT_DTYPE,
    "ovs_lookup_out": kbr.LOOKUP_OUT_DTYPE,
    "ovs_lookup_rec": shard.REC_DTYPE,
    "ovs_kad_req": shard.KAD_REQ_DTYPE,
    "ovs_kad_resp": shard.KAD_RESP_DTYPE,
    "ovs_kad_resp16": shard.KAD_RESP16_DTYPE,
    "ovs_koorde_ext": kbr.KOORDE_EXT_DTYPE,
}


@pytest.mark.parametrize("name", sorted(CTYPES))
def test_ctypes_mirror(layout, name):
    cls = CTYPES[name]
    want = layout[name]
    assert C.sizeof(cls) == want["size"], name
    assert [f for f, _ in cls._fields_] == list(want["fields"]), name
    for f, off in want["fields"].items():
        assert getattr(cls, f).offset == off, (name, f)


@pytest.mark.parametrize("name", sorted(DTYPES))
def test_dtype_mirror(layout, name):
    dt = DTYPES[name]
    want = layout[name]
    assert dt.itemsize == want["size"], name
    assert list(dt.names) == list(want["fields"]), name
    for f, off in want["fields"].items():
        assert dt.fields[f][1] == off, (name, f)


def test_done_rec_embeds_route_out(layout):
    d = layout["ovs_done_rec"]
    assert d["size"] == shard.DONE_DTYPE.itemsize == shard.DONE_BYTES
    assert d["fields"]["qid"] == shard.DONE_DTYPE.fields["qid"][1]
    base = d["fields"]["out"]
    for f, off in layout["ovs_route_out"]["fields"].items():
        assert shard.DONE_DTYPE.fields[f][1] == base + off, f
    assert layout["ovs_key160"]["size"] == 20
    assert kbr.keys_array(np.zeros((1, 5), np.uint32)).itemsize * 5 == 20
