"""CPU stand-in for the aggregator's GPU level prover (tests only): the same
aggregation circuit and host witness, proven by the oracle's CPU prover.
Lets the multi-process (gloo) and CPU tests run aggregate_level /
aggregate_to_tree / aggregate_subtrees without a GPU."""
from qp_wormhole import Circuit
from qp_wormhole.aggregator import AggregatedProof, CircuitData
from qp_wormhole.prover import ProofWithPublicInputs
from test_gpu_prover import oracle_prove

_cache = {}


class OracleLevel:
    def __init__(self, inner_common, branching):
        self.circuit = Circuit.aggregation(inner_common, branching)
        self.data = None

    def prove_chunks(self, chunks, inner_vo):
        out = []
        for ch in chunks:
            w = self.circuit.commit_proofs(inner_vo, [p.to_bytes() for p in ch])
            pb, vd = oracle_prove(self.circuit, w.wires(), w.public_inputs())
            common = self.circuit.common_data()
            self.data = CircuitData(common, vd[:len(vd) - len(common)])
            out.append(AggregatedProof(ProofWithPublicInputs(pb, w.public_inputs()), self.data))
        return out


def oracle_backend(inner_common, branching, device, max_batch):
    key = (bytes(inner_common), branching)
    if key not in _cache:
        _cache[key] = OracleLevel(inner_common, branching)
    return _cache[key]
