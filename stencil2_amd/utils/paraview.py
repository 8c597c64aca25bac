"""Reader for the ParaView CSV dumps written by DistributedDomain.write_paraview (reference src/stencil.cu:866-939,
README.md:172-183: columns Z,Y,X,<quantity names>, one row per interior cell)."""
from __future__ import annotations

import csv
import glob


def read_paraview(prefix: str):
    """Return {column: list} merged over every `prefix_<n>.txt` file."""
    cols: dict[str, list] = {}
    for path in sorted(glob.glob(prefix + "_*.txt")):
        with open(path) as f:
            r = csv.reader(f)
            header = next(r)
            for h in header:
                cols.setdefault(h, [])
            for row in r:
                for h, v in zip(header, row):
                    cols[h].append(int(v) if h in ("X", "Y", "Z") else float(v))
    return cols
