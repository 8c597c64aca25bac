"""Sample statistics with the reference's definitions (bin/statistics.cpp)."""
from __future__ import annotations

from .. import _C


def summarize(samples):
    s = _C.Statistics()
    for v in samples:
        s.insert(float(v))
    return {"count": s.count(), "min": s.min(), "max": s.max(), "avg": s.avg(), "trimean": s.trimean(),
            "med": s.med(), "stddev": s.stddev()}
