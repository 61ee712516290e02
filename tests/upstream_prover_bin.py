"""Test helper: a ProverOnlyCircuitData::to_bytes-framed file of a circuit
(the framing qp_wormhole.prover.upstream_prover_layout restates from upstream
plonky2's write_prover_only_circuit_data; parity unpinned -- the reference
commits no prover.bin).  Generator bodies, the watch map, the Merkle leaves and
digests and the public-input targets are opaque filler here: the reader checks
only their presence by search, and the preprocessing content around them."""
import struct

import numpy as np

P = 0xFFFFFFFF00000001


def q(x):
    return struct.pack("<Q", x)


def upstream_prover_bin(circuit, cap, digest, ngen=1500, gap=0):
    n = circuit.n
    co, vals = circuit.constants_sigmas_coeffs(), circuit.constants_sigmas()
    out = [q(ngen), b"\x11" * (12 * ngen), q(0)]                 # generators, generator_indices_by_watches
    out.append(q(co.shape[0]))                                   # PolynomialBatch.polynomials
    for c in co:
        out.append((q(n) if gap else b"") + q(n) + c.tobytes())
    out += [q(0), q(0)]                                          # MerkleTree leaves, digests (filler)
    out.append(q(len(cap) // 4) + np.ascontiguousarray(cap, dtype=np.uint64).tobytes())
    out += [q(circuit.degree_bits), q(3), b"\0"]                 # degree_log, rate_bits, blinding
    nsig = co.shape[0] - circuit.num_constants
    out.append(q(nsig))
    for j in range(nsig):
        out.append(q(n) + vals[circuit.num_constants + j].tobytes())
    w = pow(7277203076849721926, 1 << (32 - circuit.degree_bits), P)  # plonky2 POWER_OF_TWO_GENERATOR
    sub, x = [], 1
    for _ in range(n):
        sub.append(x)
        x = x * w % P
    out.append(q(n) + np.array(sub, np.uint64).tobytes())        # subgroup
    out.append(q(circuit.num_public_inputs) +                    # PI targets (virtual)
               b"".join(b"\0" + q(i) for i in range(circuit.num_public_inputs)))
    m = n * circuit.num_wires + 1000
    out.append(q(m) + np.arange(m, dtype=np.uint64).tobytes())   # representative_map
    out.append(b"\0")                                            # fft_root_table: None
    out.append(struct.pack("<4Q", *[int(d) for d in digest]) + q(0) + q(0))
    return b"".join(out)
