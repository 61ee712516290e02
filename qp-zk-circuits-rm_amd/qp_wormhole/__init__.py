"""qp_wormhole — host-side mirror of the reference's prover API over the
MI355X-native C ABI (include/qpgpu.h, libqpgpu.so).

Mirrors qp-wormhole-prover's WormholeProver (wormhole/prover/src/lib.rs:74-237)
and plonky2's PolynomialBatch for the parity tests.  The HIP library is the
only backend: importing the native pieces raises if it is not built.
"""
from ._native import (GATE_KINDS, Context, FriLayer, GateDesc, PolynomialBatch, QpError, fri_fold, gate_desc,  # noqa: F401
                      header_symbols, ifft, lde, lib, poseidon_permute, pow_grind, quotient)

from .circuits import (Circuit, CircuitInputs, PrivateCircuitInputs, ProcessedStorageProof,  # noqa: F401,E402
                       PublicCircuitInputs, VoteCircuitData, VotePrivateInputs, VotePublicInputs, Witness)
from .prover import (Prover, ProofWithPublicInputs, WormholeProver, generate_circuit_binaries,  # noqa: F401,E402
                     prover_only_bytes)
from .aggregator import (AggregatedProof, CircuitData, TreeAggregationConfig, WormholeProofAggregator,  # noqa: F401,E402
                         aggregate_chunk, aggregate_level, aggregate_to_tree)

__all__ = ["Circuit", "CircuitInputs", "PrivateCircuitInputs", "ProcessedStorageProof", "PublicCircuitInputs",
           "Witness", "VoteCircuitData", "VotePrivateInputs", "VotePublicInputs", "Prover", "ProofWithPublicInputs", "WormholeProver", "Context", "PolynomialBatch", "QpError", "ifft", "lde", "poseidon_permute", "lib", "header_symbols",
           "generate_circuit_binaries", "prover_only_bytes", "AggregatedProof", "CircuitData", "TreeAggregationConfig",
           "WormholeProofAggregator", "aggregate_chunk", "aggregate_level", "aggregate_to_tree", "GateDesc", "gate_desc", "quotient", "FriLayer", "fri_fold", "pow_grind"]
