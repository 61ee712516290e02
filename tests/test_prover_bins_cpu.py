"""prover.bin parsing on the host (no GPU): this backend's format, an upstream
plonky2 ProverOnlyCircuitData file recognised by its circuit digest (the native
circuit is the reference's, so the reference's digest matches), and clear errors
for anything else or a header that disagrees with the common data
(wormhole/prover/src/lib.rs:105-187)."""
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


def test_upstream_prover_bin_walked_against_the_circuit(circ):
    """A file framed as upstream ProverOnlyCircuitData::to_bytes carrying this
    circuit's preprocessing (the reference's cap and digest, reconstructed from
    its own proofs; the native circuit's columns) is accepted, with either
    length-prefix gap; its digest is the reference's."""
    from upstream_prover_bin import upstream_prover_bin
    nz = P._common_of("standard_recursion_config")
    vo, dig = _reference_vd()
    cap = np.frombuffer(vo, np.uint64, 64, 8)
    for gap in (0, 8):
        data = upstream_prover_bin(circ, cap, dig, gap=gap)
        parsed = P._parse_prover_only(data, nz, circ, vo)
        assert parsed[:2] == (None, None) and P._same_preprocessing(vo, parsed[2])
    other = [dig[0] ^ 1] + dig[1:]
    assert not P._same_preprocessing(vo, P._parse_prover_only(upstream_prover_bin(circ, cap, other), nz, circ, vo)[2])


def test_truncated_or_foreign_upstream_blobs_are_rejected(circ):
    """The old tail check accepted anything ending in digest || 0 || 0; the walk
    refuses truncations (at every section), a flipped coefficient or sigma, a
    different cap, and a foreign blob with the right tail."""
    from upstream_prover_bin import upstream_prover_bin
    nz = P._common_of("standard_recursion_config")
    vo, dig = _reference_vd()
    cap = np.frombuffer(vo, np.uint64, 64, 8)
    good = upstream_prover_bin(circ, cap, dig)
    tail = good[-48:]
    foreign = struct.pack("<Q", 1500) + b"\x11" * 40000 + tail
    assert P.upstream_prover_digest(foreign) is not None  # what the tail check used to accept
    with pytest.raises(ValueError, match="coefficients of this circuit not found"):
        P._parse_prover_only(foreign, nz, circ, vo)
    n = circ.n
    for cut in (len(good) // 10, len(good) // 3, len(good) // 2, len(good) - 8 * n - 100, len(good) - 60):
        with pytest.raises(ValueError):
            P._parse_prover_only(good[:cut] + tail, nz, circ, vo)
    # one coefficient of column 40, one sigma value, one cap element
    k = good.find(circ.constants_sigmas_coeffs()[40].tobytes())
    for pos, what in ((k + 8 * 5, "coefficient column 40"), (good.find(circ.constants_sigmas()[10].tobytes()) + 16,
                                                             "sigma")):
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
