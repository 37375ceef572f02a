"""Convert the reference's SimpleUnderlay coordinate file to raw float64 pairs.

Input : /root/reference/simulations/nodes_2d_15000.xml (data file of the reference,
        parsed like SimpleUnderlayConfigurator::parseCoordFile, SimpleUnderlayConfigurator.cc:254-310:
        one <node> per record, its <coord> children read with atof).
Output: oversim_amd/data/nodes_2d_15000.f64 -- little-endian float64, shape (records, 2).
Python's float() and glibc atof() are both correctly rounded, so the doubles are identical.
"""
import re
import sys
from pathlib import Path

import numpy as np

src = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/simulations/nodes_2d_15000.xml")
dst = Path(__file__).resolve().parent.parent / "oversim_amd" / "data" / "nodes_2d_15000.f64"
text = src.read_text()
assert 'dimensions="2"' in text
recs = []
for node in re.finditer(r"<node[^>]*>(.*?)</node>", text, re.S):
    coords = [float(c.strip()) for c in re.findall(r"<coord>(.*?)</coord>", node.group(1), re.S)]
    assert len(coords) == 2
    recs.append(coords)
arr = np.asarray(recs, dtype="<f8")
arr.tofile(dst)
print(dst, arr.shape, arr.min(axis=0), arr.max(axis=0))
