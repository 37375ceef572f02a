"""Seeded synthetic populations and lookup batches.

The reference draws node IDs with OverlayKey::random() (OverlayKey.cc:673-682),
lookup keys with KBRTestApp::createDestKey (KBRTestApp.cc:447-456: the ID of a
random live node when lookupNodeIds = true, else a random key) and coordinates
from nodes_2d_15000.xml (SimpleUnderlayConfigurator.cc:161-184) or
uniform(0, fieldSize) - fieldSize/2 (SimpleNodeEntry.cc:86-87).  OMNeT++'s
Mersenne-Twister streams are not reproduced; IDs, keys, sources and
coordinates are *inputs* generated here from numpy PCG64 seeds and recorded
in every fixture.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np

_COORDS = Path(__file__).resolve().parent / "data" / "nodes_2d_15000.f64"


def file_coords() -> np.ndarray:
    """The 15 000 records of the reference's nodes_2d_15000.xml, (15000, 2) float64."""
    return np.fromfile(_COORDS, dtype="<f8").reshape(-1, 2)


def random_keys(n: int, rng: np.random.Generator) -> np.ndarray:
    """Uniform 160-bit keys as (n,5) uint32 words (w[0] least significant)."""
    return rng.integers(0, 1 << 32, size=(n, 5), dtype=np.uint64).astype(np.uint32)


def sorted_unique_ids(n: int, seed: int) -> np.ndarray:
    """n distinct uniform 160-bit IDs in ascending order."""
    rng = np.random.default_rng(seed)
    out = np.empty((0, 5), dtype=np.uint32)
    need = n
    while need > 0:
        k = random_keys(need + need // 1000 + 8, rng)
        out = np.concatenate([out, k])
        # sort by the top 64 bits, ties by the rest (lexsort: last key is primary)
        top = (out[:, 4].astype(np.uint64) << np.uint64(32)) | out[:, 3].astype(np.uint64)
        low = (out[:, 2].astype(np.uint64) << np.uint64(32)) | out[:, 1].astype(np.uint64)
        order = np.lexsort((out[:, 0], low, top))
        out = out[order]
        dup = np.zeros(len(out), dtype=bool)
        dup[1:] = np.all(out[1:] == out[:-1], axis=1)
        out = out[~dup]
        if len(out) > n:
            # drop surplus uniformly at random (keeps the distribution uniform)
            keep = np.sort(rng.choice(len(out), size=n, replace=False))
            out = out[keep]
        need = n - len(out)
    return np.ascontiguousarray(out)


def coordinates(n: int, seed: int, field_size: int = 150, use_file: bool | None = None) -> np.ndarray:
    """SimpleUnderlay coordinates: file records (n <= 15000) or uniform(-fs/2, fs/2)."""
    rng = np.random.default_rng(seed ^ 0xC0FFEE)
    recs = file_coords()
    if use_file is None:
        use_file = n <= len(recs)
    if use_file:
        if n > len(recs):
            raise ValueError("No unused coordinates left (SimpleUnderlayConfigurator.cc:165-176)")
        return np.ascontiguousarray(recs[rng.permutation(len(recs))[:n]])
    # uniform(0, fieldSize) - fieldSize / 2  (integer division of the uint32 fieldSize)
    return rng.random((n, 2)) * float(field_size) - float(field_size // 2)


def lookups(ids: np.ndarray, m: int, seed: int, node_ids: bool = True) -> tuple[np.ndarray, np.ndarray]:
    """m (key, source) pairs: key = ID of a uniform random node (lookupNodeIds) or a uniform key."""
    rng = np.random.default_rng(seed)
    n = len(ids)
    src = rng.integers(0, n, size=m, dtype=np.int64).astype(np.uint32)
    if node_ids:
        keys = ids[rng.integers(0, n, size=m, dtype=np.int64)]
    else:
        keys = random_keys(m, rng)
    return np.ascontiguousarray(keys), src


def population(n: int, seed: int, use_file: bool | None = None):
    from .kbr import Network
    return Network(ids=sorted_unique_ids(n, seed), xy=coordinates(n, seed, use_file=use_file))


def device_population(n: int, seed: int, device, field_size: int = 150):
    """Large rings generated on the GPU (configs D/E): sorted unique uniform 160-bit IDs
    and uniform(-fs/2, fs/2) coordinates as device tensors ((n,5) int32 view of u32, (n,2) f64).
    Sorting is on the top 64 bits (torch int64 sort, sign bit flipped); the rare groups of
    equal top 64 bits are ordered by the low 96 bits on the host."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    w = torch.randint(-(1 << 31), 1 << 31, (n, 5), dtype=torch.int64, device=device, generator=g)
    w = w.to(torch.int32)
    top = (w[:, 4].to(torch.int64) << 32) | (w[:, 3].to(torch.int64) & 0xFFFFFFFF)
    top = top ^ (-(1 << 63))                    # unsigned order as signed
    order = torch.argsort(top)
    w = w[order].contiguous()
    top = top[order]
    eq = (top[1:] == top[:-1]).nonzero().flatten()
    if eq.numel():
        wc = w.cpu().numpy().view(np.uint32)
        idx = sorted(set(eq.tolist()) | set((eq + 1).tolist()))
        # sort each run of equal top words by the remaining words (exact 160-bit order)
        runs, cur = [], [idx[0]]
        for i in idx[1:]:
            if i == cur[-1] + 1 and top[i] == top[cur[0]]:
                cur.append(i)
            else:
                runs.append(cur); cur = [i]
        runs.append(cur)
        for r in runs:
            sub = wc[r]
            o = np.lexsort((sub[:, 0], sub[:, 1], sub[:, 2]))
            wc[r] = sub[o]
        w = torch.from_numpy(wc.view(np.int32)).to(device)
        full = [tuple(x) for x in wc[idx]]
        assert len(set(full)) == len(full), "duplicate 160-bit id (re-seed)"
    xy = torch.rand((n, 2), dtype=torch.float64, device=device, generator=g) * float(field_size) - float(field_size // 2)
    return w, xy


def device_lookups(n_nodes: int, m: int, seed: int, device, src_lo: int = 0, src_hi: int | None = None):
    """m uniform random 160-bit keys and uniform sources in [src_lo, src_hi) as device tensors."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    keys = torch.randint(-(1 << 31), 1 << 31, (m, 5), dtype=torch.int64, device=device, generator=g).to(torch.int32)
    hi = n_nodes if src_hi is None else src_hi
    src = torch.randint(src_lo, hi, (m,), dtype=torch.int64, device=device, generator=g).to(torch.int32)
    return keys.contiguous(), src.contiguous()


# ---------------------------------------------------------------------------
# The bench workloads (BASELINE.json configs A-E), shared by bench.py and the parity tests that
# check the exact timed path on the exact timed inputs (tests/test_gpu_timed.py).

WORKLOADS = {
    "A": dict(overlay="chord", nodes=1000, per_gpu_nodes=False, lookups=100_000, node_ids=True, file_coords=True,
              seed=0x4213,
              desc="A: Chord 1000 nodes (nodes_2d_15000.xml), successorListSize 8, 100k node-ID iterative one-way "
                   "lookups per GPU, seed 0x4213 (replicas)"),
    "C": dict(overlay="chord", nodes=1 << 20, per_gpu_nodes=True, lookups=10_000_000, node_ids=False,
              desc="C: Chord 2^20 nodes per GPU (ring sharded over GPUs), 10M random-key iterative one-way lookups per GPU"),
    "D": dict(overlay="chord", nodes=1 << 26, per_gpu_nodes=False, lookups=8_000_000, node_ids=False,
              desc="D: Chord 2^26-node ring sharded over the GPUs, 8M random-key iterative one-way lookups per GPU"),
    "B": dict(overlay="kademlia", nodes=15000, per_gpu_nodes=False, lookups=1_000_000, node_ids=True, alpha=1,
              desc="B: Kademlia 15000 nodes (nodes_2d_15000.xml), k=8, alpha=1, 1M node-ID lookups per GPU"),
    "E": dict(overlay="kademlia", nodes=1 << 24, per_gpu_nodes=False, lookups=4_000_000, node_ids=False, alpha=3,
              desc="E: Kademlia 2^24 nodes, k=8, alpha=3, 4M random-key lookups per GPU (ID arcs sharded over GPUs)"),
    "R": dict(overlay="kademlia", nodes=1 << 20, per_gpu_nodes=False, lookups=0, node_ids=False, alpha=3,
              refresh_nodes=1 << 16,
              desc="R: Kademlia 2^20 nodes, k=8, alpha=3, the bucket refresh of 2^16 nodes per GPU "
                   "(exhaustive-iterative lookups of self ^ 2^i, bucketRefreshNodes = 8; replicas)"),
    "K": dict(overlay="koorde", nodes=1 << 20, per_gpu_nodes=False, lookups=4_000_000, node_ids=False,
              desc="K: Koorde 2^20 nodes (successorListSize = deBruijnListSize = 16, shiftingBits = 4), "
                   "4M random-key iterative one-way lookups per GPU (replicas)"),
}

SMALL_HOST_LIMIT = 1 << 22     # populations up to this size are generated on the host (numpy)


def bench_inputs(workload: str, device, world: int = 1, rank: int = 0, seed: int | None = None, nodes: int | None = None,
                 n_lookups: int | None = None, sharded: bool | None = None) -> dict:
    """The population and this rank's lookups of a bench workload, resident on `device`.

    Returns ids_t (n,5) int32 view of the u32 words, xy_t (n,2) f64, keys_t (m,5) int32, src_t (m,)
    int32 device tensors; ids / xy / keys / src as numpy arrays when the population is generated
    on the host (n <= SMALL_HOST_LIMIT), else None; n_total, m, lo, hi (this rank's source arc)."""
    import torch
    wl = WORKLOADS[workload]
    if seed is None:
        seed = wl.get("seed", 0xC)
    n_node = nodes or wl["nodes"]
    n_total = n_node * world if wl["per_gpu_nodes"] else n_node
    m = n_lookups or wl["lookups"]
    kind = wl["overlay"]
    if sharded is None:
        sharded = world > 1
    if sharded:
        lo, hi = rank * n_total // world, (rank + 1) * n_total // world
    else:
        lo, hi = 0, n_total
    small = n_total <= SMALL_HOST_LIMIT
    if small:
        ids = sorted_unique_ids(n_total, seed)
        xy = coordinates(n_total, seed, use_file=wl.get("file_coords", kind == "kademlia" and n_total <= 15000))
        ids_t = torch.from_numpy(ids.view(np.int32)).to(device)
        xy_t = torch.from_numpy(xy).to(device)
        keys, src = lookups(ids, m, seed + 1000 + rank, node_ids=wl["node_ids"])
        src = (lo + (src.astype(np.int64) % (hi - lo))).astype(np.uint32)
        keys_t = torch.from_numpy(keys.view(np.int32)).to(device)
        src_t = torch.from_numpy(src.view(np.int32)).to(device)
    else:
        ids_t, xy_t = device_population(n_total, seed, device)
        keys_t, src_t = device_lookups(n_total, m, seed + 1000 + rank, device, lo, hi)
        ids = xy = keys = src = None
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    return dict(ids_t=ids_t, xy_t=xy_t, keys_t=keys_t, src_t=src_t, ids=ids, xy=xy, keys=keys, src=src,
                n_total=n_total, m=m, lo=lo, hi=hi, kind=kind, seed=seed, alpha=wl.get("alpha", 1), desc=wl["desc"],
                per_gpu_nodes=wl["per_gpu_nodes"])

