"""A missing device table is an error, not a fault (the class of the round-3
null-table fault on the first GPU aggregation run, commit 0d3293f): every prove
entry point checks the tables its kernels read before launching them and
returns QP_ERR_STATE naming the table (qp_prover_debug_drop_table releases one,
test-only)."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("table,path", [("wg_wslot_cm", "witnesses"), ("wg_wslot_cm", "inputs"),
                                        ("wg_gens", "inputs"), ("qtab", "wires")])
def test_missing_table_is_reported(table, path):
    import qp_wormhole
    from qp_wormhole._native import lib
    from qp_wormhole.synthetic import synthetic_inputs
    circ = qp_wormhole.Circuit.wormhole()
    p = qp_wormhole.Prover(qp_wormhole.Context(0), circ, max_batch=1)
    inp = synthetic_inputs(7, 1)
    w = circ.commit(inp)
    assert lib().qp_prover_debug_drop_table(p.h, table.encode()) == 0
    with pytest.raises(qp_wormhole.QpError) as e:
        if path == "witnesses":
            p.prove_witnesses([w])
        elif path == "inputs":
            p.prove_inputs([inp])
        else:
            p.prove_wires(w.wires()[None], w.public_inputs()[None])
    assert e.value.code == 4 and table in str(e.value)
    p.free()
