"""Writes tests/golden/reference_pi_cells.json: the 131 PublicInputGate-row
cells (wires 4..134 of row 7039) and the PoW witness of each of the
reference's current-circuit proofs, read out of their own openings
(tests/test_reference_layout.py: every wire column of a fixture equals the
native witness of test_inputs() except at that row, so the one-row residual is
the cell).  Derived data: no reference file is read beyond the two fixtures.

    python tests/golden/make_pi_cells.py
"""
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(os.path.dirname(HERE)), "qp-zk-circuits-rm_amd")]


def cells():
    from oracle_lib import golden
    from qp_wormhole import Circuit
    from test_reference_layout import PROOFS, fixture_points, reference_pi_cells
    pts = fixture_points()
    circ = Circuit.wormhole(zero_knowledge=False)
    out = {"source": "tests/golden/make_pi_cells.py (one-row residuals of the fixtures' wire openings)",
           "pi_row": 7039}
    for name in PROOFS:
        pf = golden(name)
        out[name] = {"pi_row_cells": [int(v) for v in reference_pi_cells(pts, circ, name)],
                     "pow_witness": struct.unpack_from("<Q", pf, len(pf) - 8 * 18)[0]}
    return out


if __name__ == "__main__":
    with open(os.path.join(HERE, "reference_pi_cells.json"), "w") as f:
        json.dump(cells(), f, indent=1)
