"""Write the PMC traffic summary bench.py reports as roofline.traffic.

usage: python tools/pmc_json.py <prof summary txt (tools/prof_summary.py)> <kernel substring> <workload> [out dir]
Takes the mean FETCH_SIZE / WRITE_SIZE (KB) per dispatch of the kernel from the summary of the
rocprofv3 --pmc passes of `bench.py --workload <workload>` and writes <out dir>/<workload>.json.
"""
import json
import sys
from pathlib import Path


def main():
    src, ksub, wl = sys.argv[1], sys.argv[2], sys.argv[3]
    out = Path(sys.argv[4] if len(sys.argv) > 4 else Path(__file__).resolve().parent.parent / "profiles" / "pmc")
    vals, kname, avg_ns = {}, None, None
    for line in Path(src).read_text().splitlines():
        if line.startswith("#") or ksub not in line:
            continue
        parts = line.rsplit(",", 3)
        if len(parts) == 4 and parts[1] in ("FETCH_SIZE", "WRITE_SIZE"):
            vals[parts[1]] = float(parts[2])
            kname = parts[0]
    if "FETCH_SIZE" not in vals:
        raise SystemExit(f"no FETCH_SIZE for {ksub} in {src}")
    out.mkdir(parents=True, exist_ok=True)
    d = {"workload": wl, "kernel": kname, "fetch_kb": vals["FETCH_SIZE"], "write_kb": vals.get("WRITE_SIZE", 0.0),
         "unit": "KB per dispatch (x1024 = bytes); FETCH_SIZE calibrated at 64 B per random 64 B line",
         "source": str(src)}
    (out / f"{wl}.json").write_text(json.dumps(d, indent=1) + "\n")
    print(json.dumps(d))


if __name__ == "__main__":
    main()
