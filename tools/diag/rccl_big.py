"""Pin the cause of the record loss seen when an RCCL all-to-all moved more than ~1 GB at world size
1, and time the 0xFF sentinel fill of an exchange receive buffer.

Three probes, each transfer checked byte for byte against a position-dependent pattern:
  torch  -- torch.distributed.all_to_all_single (backend nccl = RCCL) at world size 1, for several
            byte sizes around 1 GB and 2 GB and for uint8 / int32 / int64 elements (does the limit
            follow the byte count or the element count?);
  p2p    -- one ncclSend + ncclRecv to self in one group, straight through librccl (the transport
            all_to_all_single uses), one message of the whole size;
  chunk  -- the same split into 256 MB messages, as the library's RCCL exchange sends
            (shard_route.cpp RCCL_CHUNK).
Prints one JSON line per transfer and one per fill timing.  world size 1 only; 127.0.0.1 rendezvous.

usage: python tools/diag/rccl_big.py [--sizes-mb 512,1023,1024,1025,1536,2047,2048,2049,3072]"""
import argparse
import ctypes as C
import json
import os
import sys

import torch
import torch.distributed as dist

ap = argparse.ArgumentParser()
ap.add_argument("--sizes-mb", default="512,1000,1023,1024,1025,1100,1536,2047,2048,2049,3072")
ap.add_argument("--probes", default="torch,p2p,chunk,fill")
a = ap.parse_args()
sizes = [int(x) for x in a.sizes_mb.split(",")]
probes = set(a.probes.split(","))

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
MB = 1 << 20


def pattern(nbytes: int) -> torch.Tensor:
    # byte i = (i * 2654435761 >> 7) & 0xFF: position-dependent, so a shifted or missing piece shows
    i = torch.arange(nbytes // 8, dtype=torch.int64, device=dev)
    return (i * 0x9E3779B97F4A7C15 + 0x1234567).view(torch.uint8)[:nbytes].contiguous()


def check(tag: str, send: torch.Tensor, recv: torch.Tensor, **kw):
    # compared in 256 MiB pieces (boolean indexing / nonzero of > 2^31 elements is not safe here)
    torch.cuda.synchronize()
    nbad = untouched = 0
    first = last = -1
    piece = 256 * MB
    for o in range(0, send.numel(), piece):
        a, b = send[o:o + piece], recv[o:o + piece]
        bad = a != b
        k = int(bad.sum())
        if k:
            nbad += k
            untouched += int((bad & (b == 0xFF)).sum())
            if first < 0:
                first = o + int(bad.to(torch.uint8).argmax())
            last = o + int(bad.numel() - 1 - bad.flip(0).to(torch.uint8).argmax())
    print(json.dumps(dict(probe=tag, bytes=int(send.numel()), mismatched=nbad, first_bad=first, last_bad=last,
                          bad_still_sentinel=untouched, **kw)), flush=True)


if "torch" in probes:
    for mb in sizes:
        for dt, es in ((torch.uint8, 1), (torch.int32, 4), (torch.int64, 8)):
            s = pattern(mb * MB)
            r = torch.full_like(s, 0xFF)
            dist.all_to_all_single(r.view(dt), s.view(dt))
            check("torch", s, r, dtype=str(dt).split(".")[-1], elements=mb * MB // es)
            del s, r
            torch.cuda.empty_cache()

if "p2p" in probes or "chunk" in probes:
    rccl = None
    for name in ("librccl.so.1", "librccl.so"):
        try:
            rccl = C.CDLL(name)
            break
        except OSError:
            pass
    if rccl is None:
        print(json.dumps(dict(probe="p2p", error="librccl not loadable")), flush=True)
    else:
        class UID(C.Structure):
            _fields_ = [("internal", C.c_char * 128)]
        uid = UID()
        assert rccl.ncclGetUniqueId(C.byref(uid)) == 0
        comm = C.c_void_p()
        assert rccl.ncclCommInitRank(C.byref(comm), 1, uid, 0) == 0
        rccl.ncclSend.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        rccl.ncclRecv.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        NCCL_UINT8 = 1
        stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)

        def p2p(send, recv, chunk):
            nb = send.numel()
            assert rccl.ncclGroupStart() == 0
            for o in range(0, nb, chunk):
                c = min(chunk, nb - o)
                assert rccl.ncclSend(C.c_void_p(send.data_ptr() + o), c, NCCL_UINT8, 0, comm, stream) == 0
            for o in range(0, nb, chunk):
                c = min(chunk, nb - o)
                assert rccl.ncclRecv(C.c_void_p(recv.data_ptr() + o), c, NCCL_UINT8, 0, comm, stream) == 0
            assert rccl.ncclGroupEnd() == 0

        for mb in sizes:
            for tag, chunk in (("p2p", 1 << 62), ("chunk", 256 * MB)):
                if tag not in probes:
                    continue
                s = pattern(mb * MB)
                r = torch.full_like(s, 0xFF)
                p2p(s, r, chunk)
                check(tag, s, r, messages=(mb * MB + chunk - 1) // chunk)
                del s, r
                torch.cuda.empty_cache()
        rccl.ncclCommDestroy(comm)

if "fill" in probes:
    # the sentinel fill of a receive buffer: config C round 2 at W = 8 (9.4M x 48 B) and config E
    # round 1 (10.5M x 136 B) per arc
    for label, nbytes in (("C_w8_round2", 9_400_000 * 48), ("E_w8_round1", 10_500_000 * 136)):
        buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        buf.fill_(0xFF)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(10):
            buf.fill_(0xFF)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(json.dumps(dict(probe="fill", what=label, bytes=nbytes, ms=round(ms, 4),
                              GBps=round(nbytes / ms / 1e6, 1))), flush=True)
        del buf

dist.destroy_process_group()
