"""Kademlia maintenance rounds from a partially joined network to their fixed point:
per round the counters of ovs_kad_maintenance_round and its wall time, then how the converged
tables differ from the snapshot rule.  usage: python tools/diag/kad_maint_rounds.py [n] [join_frac]"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
from kad_maint import partial_join  # noqa: E402
from oracle_lib import OracleNet, kad_params  # noqa: E402
from oversim_amd import KbrEngine, Params, workload as W  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 15000
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.1
net = W.population(n, 0x4b41)
tabs, join = partial_join(net.ids, net.xy, frac, 13)
rows = []
with KbrEngine(0) as eng:
    eng.set_params(Params.kademlia())
    eng.kad_load_tables(net.ids, net.xy, tabs["siblings"], tabs["bucket_count"], tabs["bucket_nodes"])
    for r in range(10):
        t0 = time.perf_counter()
        st = eng.kad_maintenance_round(join, 1) if r == 0 else eng.kad_maintenance_round()
        st["wall_s"] = round(time.perf_counter() - t0, 3)
        st["round"] = r
        rows.append(st)
        print(json.dumps(st), flush=True)
        if r > 0 and st["changes"] == 0:
            break
    sib, cnt, nodes = eng.kad_tables()
snap_s, snap_c, snap_n = OracleNet("kademlia", net.ids, net.xy, kad_params()).kad_tables()
same_sib = np.mean([set(a[a != 0xFFFFFFFF]) == set(b[b != 0xFFFFFFFF]) for a, b in zip(sib, snap_s)])
full = cnt == 8
same_members = np.mean([set(nodes[v, m, :cnt[v, m]]) == set(snap_n[v, m, :snap_c[v, m]])
                        for v in range(0, n, 97) for m in range(160) if cnt[v, m]])
print(json.dumps({"n": n, "joined": len(join), "rounds": len(rows), "sibling_tables_equal_snapshot": float(same_sib),
                  "bucket_fill_equal_snapshot": float(np.mean(cnt == snap_c)), "full_buckets": int(full.sum()),
                  "bucket_members_equal_snapshot_sample": float(same_members)}), flush=True)
