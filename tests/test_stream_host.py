"""CPU: the host side of the streaming rows -- timespan labels of rollup
periods (build_timespan_label, heatmap.py:38-52) and the per-span row
assembly (Cells with several labels) on hand-made counts."""
import datetime

import numpy as np

from heatmap_amd import heatmap
from heatmap_amd.stream import span_label


def test_span_labels():
    d = (datetime.date(2025, 1, 1) - datetime.date(1970, 1, 1)).days
    assert span_label("day", d) == "2025-01-01"
    assert span_label("day", d - 1) == "2024-12-31"
    assert span_label("month", 2024 * 12 + 1) == "2024-02"
    assert span_label("year", 2024) == "2024"
    assert span_label("alltime", 0) == "alltime"


def test_cells_with_several_spans():
    """Two periods' cells concatenated keep their own labels in rows and table."""
    d, zmax = 1, 3
    parts = []
    for lab, n in (("2024", 1), ("2025", 2)):
        allc = (np.array([3]), np.array([5]), np.array([6]), np.array([n]))
        grp = (np.array([1]), np.array([3]), np.array([5]), np.array([6]), np.array([n]))
        parts.append(heatmap.combine_cells(["all", "u"], allc, grp, zmax, d, lab))
    cells = heatmap.concat_cells(parts, ["all", "u"], d)
    rows = heatmap.cells_to_rows(cells)
    assert rows == {"all|2024|2_2_3": {"3_5_6": 1.0}, "u|2024|2_2_3": {"3_5_6": 1.0},
                    "all|2025|2_2_3": {"3_5_6": 2.0}, "u|2025|2_2_3": {"3_5_6": 2.0}}
    t = heatmap.cells_to_table(cells)
    assert sorted(t.column("id").to_pylist()) == sorted(rows)
