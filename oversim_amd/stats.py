"""KBRTestApp statistics in OverSim's own output format.

The engine reduces a batch of one-way test lookups to the statistics a KBRTestApp
run hands to GlobalStatistics (`KbrEngine.kbrtest_stats`, C ABI
`ovs_kbrtest_stats_batch`).  This module writes them the way
`GlobalStatistics::finalizeStatistics` records them (GlobalStatistics.cc:103-140)
into an OMNeT++ 4 scalar file (`.sca`, result-file format version 2), so a
results pipeline built for OverSim reads the engine's output unchanged:

  scalar <network>.globalObserver.globalStatistics "GlobalStatistics: Simulation Time" <t>
  scalar ... "KBRTestApp: One-way Delivered Messages/s.mean" <v>     (stdDevMap, name order)
  scalar ... "Vector: KBRTestApp: One-way Hop Count.mean" <v>        (outVectorMap, name order)

`.stddev` / `.min` / `.max` lines follow the outputStdDev / outputMinMax
parameters (default.ini:522-523 sets both false).
"""
from __future__ import annotations

import datetime as _dt
from pathlib import Path

from .kbr import KbrTestLookupStats, KbrTestStats

GLOBAL_STATS_MODULE = "SimpleUnderlayNetwork.globalObserver.globalStatistics"


def scalars(st: KbrTestStats | None, sim_time_s: float, output_stddev: bool = False,
            output_min_max: bool = False, lookup: KbrTestLookupStats | None = None) -> list[tuple[str, float]]:
    """(name, value) pairs in finalizeStatistics order: the one-way test (st) and/or the lookup
    test (lookup) of the same run."""
    out: list[tuple[str, float]] = [("GlobalStatistics: Simulation Time", float(sim_time_s))]
    sd = []
    for obj, names in ((st, KbrTestStats.STDDEV_NAMES), (lookup, KbrTestLookupStats.STDDEV_NAMES)):
        if obj is not None:
            sd += [(name, getattr(obj, field)) for field, name in names.items()
                   if getattr(obj, field).count > 0]       # addStdDev only called when collected
    sd.sort(key=lambda t: t[0])
    for name, s in sd:                                    # std::map<std::string, cStdDev*> order
        out.append((name + ".mean", s.mean))
        if output_stddev:
            out.append((name + ".stddev", s.stddev))
        if output_min_max:
            out.append((name + ".min", s.min))
            out.append((name + ".max", s.max))
    vec = []
    if st is not None and st.num_delivered > 0:           # recordOutVector only on evaluateData
        vec += [("KBRTestApp: One-way Hop Count", st.hop_count_mean),
                ("KBRTestApp: One-way Latency", st.latency_mean_s)]
    if lookup is not None:                                # handleLookupResponse (KBRTestApp.cc:341-369)
        if lookup.num_success > 0:
            vec += [("KBRTestApp: Lookup Success Latency", lookup.success_latency_mean_s),
                    ("KBRTestApp: Lookup Hop Count", lookup.hop_count_mean)]
        if lookup.num_failed > 0:
            vec += [("KBRTestApp: Failed Lookup Hop Count", lookup.failed_hop_count_mean)]
        if lookup.num_sent > 0:
            vec += [("KBRTestApp: Lookup Total Latency", lookup.total_latency_mean_s)]
    vec.sort(key=lambda t: t[0])
    out.extend(("Vector: " + n + ".mean", v) for n, v in vec)
    return out


def _q(s: str) -> str:
    return '"' + s.replace("\\", "\\\\").replace('"', '\\"') + '"' if (" " in s or '"' in s) else s


def write_sca(path: str | Path, st: KbrTestStats | None, sim_time_s: float, config: str = "General",
              run_number: int = 0, network: str = "SimpleUnderlayNetwork", output_stddev: bool = False,
              output_min_max: bool = False, module: str = GLOBAL_STATS_MODULE,
              lookup: KbrTestLookupStats | None = None) -> Path:
    """Write an OMNeT++ 4 scalar file with the batch's KBRTestApp statistics."""
    path = Path(path)
    now = _dt.datetime.now(_dt.timezone.utc).strftime("%Y%m%d-%H:%M:%S")
    run_id = f"{config}-{run_number}-{now}-0"
    lines = ["version 2", f"run {run_id}", f"attr configname {config}", f"attr datetime {now}",
             f"attr experiment {config}", "attr measurement \"\"", f"attr network {network}",
             "attr replication #0", f"attr runnumber {run_number}", ""]
    for name, v in scalars(st, sim_time_s, output_stddev, output_min_max, lookup):
        lines.append(f"scalar {module} \t{_q(name)} \t{v!r}")
    path.write_text("\n".join(lines) + "\n")
    return path


def read_sca(path: str | Path) -> dict[str, float]:
    """Scalars of a .sca file by name (module ignored) -- for tests and tooling."""
    res: dict[str, float] = {}
    for line in Path(path).read_text().splitlines():
        if not line.startswith("scalar "):
            continue
        rest = line[len("scalar "):].strip()
        _, rest = rest.split(None, 1)
        rest = rest.strip()
        if rest.startswith('"'):
            end = rest.index('"', 1)
            name, val = rest[1:end], rest[end + 1:]
        else:
            name, val = rest.split(None, 1)
        res[name] = float(val)
    return res


def summary(st: KbrTestStats) -> dict:
    """Plain-dict view (JSON friendly)."""
    d = {f: getattr(st, f) for f, _ in KbrTestStats._fields_
         if f not in ("status_count", "hop_hist") and f not in KbrTestStats.STDDEV_NAMES}
    d["status_count"] = list(st.status_count)
    d["hop_hist"] = list(st.hop_hist)
    for f, name in KbrTestStats.STDDEV_NAMES.items():
        s = getattr(st, f)
        d[name] = {"count": s.count, "mean": s.mean, "stddev": s.stddev, "min": s.min, "max": s.max}
    return d
