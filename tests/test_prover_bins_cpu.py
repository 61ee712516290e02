"""prover.bin on the host (no GPU): upstream plonky2 ProverOnlyCircuitData::to_bytes
written by the native writer (csrc/prover_bin.cpp) and walked section by section
by the reader (qp_wormhole.prover.read_upstream_prover_only), this backend's own
format, and clear errors for anything else or a header that disagrees with the
common data (wormhole/circuit-builder/src/lib.rs:53-59,
wormhole/prover/src/lib.rs:105-187)."""
import hashlib
import struct

import numpy as np
import pytest

from qp_wormhole import prover as P


def _file(common, zk=0, degree_bits=13, kind=0):
    head = P.PROVER_MAGIC + struct.pack("<IBBI", P.PROVER_VERSION, kind, zk, degree_bits)
    return head + hashlib.sha256(common).digest() + b"\0" * 40


def test_common_degree_bits_and_config():
    nz = P._common_of("standard_recursion_config")
    zk = P._common_of("standard_recursion_zk_config")
    assert P._common_degree_bits(nz) == 13 and P._common_degree_bits(zk) == 13
    assert P._config_of_common(nz) == "standard_recursion_config"
    assert P._config_of_common(zk) == "standard_recursion_zk_config"
    assert P._config_of_common(nz[:-1]) is None


def test_unrecognised_prover_bin_is_rejected_clearly():
    nz = P._common_of("standard_recursion_config")
    with pytest.raises(ValueError, match="neither this backend's prover.bin"):
        P._parse_prover_only(b"\x05\x00\x00\x00" + b"\x11" * 200, nz)


def _reference_vd():
    from current_circuit_vd import current_circuit_verifier_data
    from test_oracle_golden import current_common_bytes
    vd, cap, dig = current_circuit_verifier_data(current_common_bytes())
    return vd[:len(vd) - len(current_common_bytes())], [int(x) for x in dig]


@pytest.fixture(scope="module")
def circ():
    import qp_wormhole
    return qp_wormhole.Circuit.wormhole()


def test_host_coefficients_are_the_constants_sigmas_polynomials(circ):
    """qp_circuit_constants_sigmas_coeffs (host ifft) interpolates the columns:
    evaluated at w_n^i (Horner) they give back the values."""
    Pm = 0xFFFFFFFF00000001
    co, vals = circ.constants_sigmas_coeffs(), circ.constants_sigmas()
    w = pow(7277203076849721926, 1 << (32 - circ.degree_bits), Pm)
    for col in (0, 3, 4, 50, 83):
        for i in (0, 1, 777, circ.n - 1):
            x, acc = pow(w, i, Pm), 0
            for c in reversed([int(v) for v in co[col]]):
                acc = (acc * x + c) % Pm
            assert acc == int(vals[col][i])


@pytest.fixture(scope="module")
def upstream(circ):
    """The native writer's upstream prover.bin (qp_circuit_prover_only_bytes)."""
    return circ.prover_only_bytes()


def test_upstream_prover_bin_round_trip(circ, upstream):
    """writer -> structural reader -> checks: every section parses in
    write_prover_only_circuit_data order and ends exactly; the commitment inside
    (constants||sigmas cap, computed on the host from the LDE rows, and the
    circuit digest) equals the reference's own verifier data -- reconstructed
    from the reference's proofs, so this part is pinned; the rest (generator
    order and bodies, watch index, representative map) is restated from
    upstream plonky2, parity unpinned."""
    vo, dig = _reference_vd()
    cap = np.frombuffer(vo, np.uint64, 64, 8)
    f = P.read_upstream_prover_only(upstream)
    assert np.array_equal(f["cap"], cap) and list(f["circuit_digest"]) == dig
    assert f["degree_log"] == 13 and f["rate_bits"] == 3 and not f["blinding"]
    assert f["leaves"].shape == (1 << 16, 84) and f["digests"].shape == (2 * ((1 << 16) - 16), 4)
    assert f["sigmas"].shape == (circ.n, 80)
    # write_merkle_cap: the cap is prefixed by its HEIGHT (log2 of 16 hashes), as
    # in VerifierOnlyCircuitData (verifier.bin, a reference fixture)
    k = upstream.find(cap.tobytes())
    assert k > 0 and struct.unpack_from("<Q", upstream, k - 8)[0] == 4 == struct.unpack_from("<Q", vo, 0)[0]
    names = {}
    for name, _ in f["generators"]:
        names[name] = names.get(name, 0) + 1
    gens, rows = circ.census()
    assert names["PoseidonGenerator"] == rows["poseidon"] and names["RandomValueGenerator"] == 131
    assert names["EqualityGenerator"] == gens["equality"]
    assert names["ArithmeticBaseGenerator"] == 20 * rows["arithmetic"]
    # every generator's watched targets are indexed under their representatives
    rep = f["representative_map"]
    assert all(rep[key] == key for key in f["watches"])
    # build() connects each ConstantGate's output wire to its constant's target as
    # connect(Target::wire(row, wire), t): Forest::merge puts t's root under the
    # fresh wire, which stays its set's representative
    W = circ.num_wires
    consts = [b for name, b in f["generators"] if name == "ConstantGenerator"]
    assert consts
    assert all(rep[int(b[0]) * W + int(b[2])] == int(b[0]) * W + int(b[2]) for b in consts)
    assert P.upstream_prover_layout(upstream, circ, cap, check_subtrees=2) == tuple(dig)
    nz = P._common_of("standard_recursion_config")
    parsed = P._parse_prover_only(upstream, nz, circ, vo)
    assert parsed[:2] == (None, None) and P._same_preprocessing(vo, parsed[2])


def _gen_tag_offsets(data, count=3):
    """Byte offsets of the first generators' u32 tags (walk of their bodies)."""
    w = P._Walk(data)
    w.u64()
    offs = []
    for _ in range(count):
        offs.append(w.p)
        _, body = P.UPSTREAM_GENERATORS[w.u32()]
        for k in body:
            if k in "uf":
                w.u64()
            elif k == "t":
                w.target()
            else:
                w.vec("gates")
    return offs


def test_truncated_or_foreign_upstream_blobs_are_rejected(circ, upstream):
    """The walk refuses truncations in every section, a foreign generator tag,
    bytes past the end, a flipped coefficient, sigma, Merkle leaf or digest, a
    different cap, and a blob that only ends like a prover.bin."""
    nz = P._common_of("standard_recursion_config")
    vo, dig = _reference_vd()
    cap = np.frombuffer(vo, np.uint64, 64, 8)
    good = upstream
    tail = good[-48:]
    foreign = struct.pack("<Q", 1500) + b"\x11" * 40000 + tail
    with pytest.raises(ValueError, match="foreign generator|truncated"):
        P._parse_prover_only(foreign, nz, circ, vo)
    for cut in (9, len(good) // 10, len(good) // 3, len(good) // 2, len(good) - 8 * circ.n - 100, len(good) - 60):
        with pytest.raises(ValueError):
            P._parse_prover_only(good[:cut] + tail, nz, circ, vo)
    with pytest.raises(ValueError, match="past"):
        P.read_upstream_prover_only(good + bytes(8))
    # a generator kind the leaf circuits do not have (ArithmeticExtensionGenerator, tag 1)
    t = _gen_tag_offsets(good)[1]
    bad = bytearray(good)
    bad[t:t + 4] = struct.pack("<I", 1)
    with pytest.raises(ValueError, match="foreign generator"):
        P.read_upstream_prover_only(bytes(bad))
    # one coefficient of column 40, one sigma value, one leaf of cap subtree 0, one digest
    co = circ.constants_sigmas_coeffs()
    sig_row = np.ascontiguousarray(circ.constants_sigmas()[circ.num_constants:, 7])
    f = P.read_upstream_prover_only(good)
    leaf = good.find(struct.pack("<Q", 84) + f["leaves"][3].tobytes())
    digk = good.find(f["digests"][5].tobytes())
    for pos, what in ((good.find(co[40].tobytes()) + 8 * 5, "coefficient column 40"),
                      (good.find(struct.pack("<Q", 80) + sig_row.tobytes()) + 8 + 16, "sigma"),
                      (leaf + 8 + 8 * 2, "merkle"), (digk + 3, "merkle")):
        bad = bytearray(good)
        bad[pos] ^= 1
        with pytest.raises(ValueError, match=what):
            P._parse_prover_only(bytes(bad), nz, circ, vo)
    cap2 = cap.copy()
    cap2[5] ^= 1
    with pytest.raises(ValueError, match="Merkle cap"):
        P._parse_prover_only(good, nz, circ, vo[:8] + cap2.tobytes() + vo[8 + 512:])
    # without the circuit an upstream file cannot be checked
    with pytest.raises(ValueError, match="needs the circuit"):
        P._parse_prover_only(good, nz)


def test_upstream_prover_bin_of_the_voting_circuit():
    """The second leaf circuit (configs[4]) through the same writer and walk."""
    import qp_wormhole
    v = qp_wormhole.Circuit.voting()
    data = v.prover_only_bytes()
    d = P.upstream_prover_layout(data, v, check_subtrees=16)
    f = P.read_upstream_prover_only(data)
    assert f["degree_log"] == v.degree_bits and d == f["circuit_digest"]
    assert len(f["public_inputs"]) == v.num_public_inputs == 13


def test_aggregation_circuits_have_no_upstream_writer():
    """Only the leaf circuits' generator kinds are restated (QP_ERR_ARG)."""
    import qp_wormhole
    from test_oracle_golden import current_common_bytes
    with pytest.raises(qp_wormhole.QpError):
        qp_wormhole.Circuit.aggregation(current_common_bytes(), 2).prover_only_bytes()


def test_header_must_agree_with_common_data():
    nz = P._common_of("standard_recursion_config")
    zk, db, vd = P._parse_prover_only(_file(nz), nz)
    assert (zk, db, len(vd)) == (False, 13, 40)
    with pytest.raises(ValueError, match="zk flag"):
        P._parse_prover_only(_file(nz, zk=1), nz)
    with pytest.raises(ValueError, match="degree_bits"):
        P._parse_prover_only(_file(nz, degree_bits=14), nz)
    with pytest.raises(ValueError, match="different common data"):
        P._parse_prover_only(_file(nz), P._common_of("standard_recursion_zk_config"))
