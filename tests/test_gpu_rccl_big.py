"""RCCL record loss above 1 GiB: one ncclSend/ncclRecv pair of more than 2^30 bytes
delivers only its first half on this image's RCCL (2.26.6, torch's librccl), whatever the datatype
(tools/diag/rccl_big.py, profiles/r05_rccl/).  The library's RCCL exchange (shard_route.cpp,
rccl_alltoallv) cuts every transfer into messages of at most 256 MiB; this checks, through the same
librccl calls on a one-rank communicator (a rank sending to itself), that a 1.5 GiB transfer cut that
way arrives whole, and that the uncut one still loses its second half (so the test would notice a
fixed RCCL and the guard could be revisited)."""
from __future__ import annotations

import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu
MB = 1 << 20
CHUNK = 256 * MB          # shard_route.cpp RCCL_CHUNK


def _rccl():
    for name in ("librccl.so.1", "librccl.so"):
        try:
            return C.CDLL(name)
        except OSError:
            pass
    pytest.skip("librccl not loadable")


def _transfer(lib, comm, send, recv, chunk):
    lib.ncclSend.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    lib.ncclRecv.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    nb = send.numel()
    assert lib.ncclGroupStart() == 0
    for o in range(0, nb, chunk):
        assert lib.ncclSend(C.c_void_p(send.data_ptr() + o), min(chunk, nb - o), 1, 0, comm, s) == 0
    for o in range(0, nb, chunk):
        assert lib.ncclRecv(C.c_void_p(recv.data_ptr() + o), min(chunk, nb - o), 1, 0, comm, s) == 0
    assert lib.ncclGroupEnd() == 0
    torch.cuda.synchronize()


def test_chunked_rccl_transfer_above_1gib_is_complete():
    import torch  # noqa: F811  (one HIP runtime: torch first)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = _rccl()
    class UID(C.Structure):                     # ncclUniqueId: 128 bytes, passed by value
        _fields_ = [("internal", C.c_char * 128)]
    uid = UID()
    assert lib.ncclGetUniqueId(C.byref(uid)) == 0
    comm = C.c_void_p()
    assert lib.ncclCommInitRank(C.byref(comm), 1, uid, 0) == 0
    try:
        nb = 1536 * MB
        send = (torch.arange(nb // 8, dtype=torch.int64, device=dev) * 0x9E3779B97F4A7C15 + 7).view(torch.uint8)
        recv = torch.full_like(send, 0xFF)
        _transfer(lib, comm, send, recv, CHUNK)
        for o in range(0, nb, CHUNK):
            assert torch.equal(send[o:o + CHUNK], recv[o:o + CHUNK]), f"chunked transfer lost bytes at {o}"
        # the uncut message: the RCCL behaviour the chunking avoids
        recv.fill_(0xFF)
        _transfer(lib, comm, send, recv, 1 << 62)
        head_ok = torch.equal(send[:nb // 2], recv[:nb // 2])
        tail_lost = bool((recv[nb // 2:nb // 2 + MB] == 0xFF).all())
        assert head_ok
        if not tail_lost:
            pytest.xfail("this RCCL delivers > 1 GiB messages whole: RCCL_CHUNK is no longer needed")
    finally:
        lib.ncclCommDestroy(comm)
