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


def paraview_grid(prefix: str, name: str, size_xyz):
    """Assemble quantity `name` of the dumps `prefix_*.txt` into a dense (z, y, x) float64 tensor of the global grid
    (every cell must be present exactly once: the dumps of all sub-domains tile the grid)."""
    import torch

    cols = read_paraview(prefix)
    X, Y, Z = size_xyz
    z = torch.tensor(cols["Z"], dtype=torch.long)
    y = torch.tensor(cols["Y"], dtype=torch.long)
    x = torch.tensor(cols["X"], dtype=torch.long)
    if len(z) != X * Y * Z:
        raise ValueError(f"{len(z)} cells in the dumps, {X * Y * Z} in the grid")
    g = torch.full((Z, Y, X), float("nan"), dtype=torch.float64)
    g[z, y, x] = torch.tensor(cols[name], dtype=torch.float64)
    return g
