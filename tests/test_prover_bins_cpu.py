"""prover.bin parsing on the host (no GPU): this backend's format, an upstream
plonky2 ProverOnlyCircuitData file recognised by its circuit digest (the native
circuit is the reference's, so the reference's digest matches), and clear errors
for anything else or a header that disagrees with the common data
(wormhole/prover/src/lib.rs:105-187)."""
import hashlib
import struct

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


def _upstream_shaped(digest, ngen=1500, body=4096):
    """generators.len() || (opaque body) || circuit digest || 0u64 || 0u64 -- the
    frame of ProverOnlyCircuitData::to_bytes for a lookup-free circuit."""
    return struct.pack("<Q", ngen) + b"\x11" * body + struct.pack("<4Q", *digest) + bytes(16)


def test_upstream_prover_bin_recognised_by_the_reference_circuit_digest():
    """The reference's circuit digest (reconstructed from its own proofs) is the
    native circuit's, so an upstream prover.bin of the Wormhole circuit matches."""
    from current_circuit_vd import current_circuit_verifier_data
    from test_oracle_golden import current_common_bytes
    nz = P._common_of("standard_recursion_config")
    vd, cap, dig = current_circuit_verifier_data(current_common_bytes())
    vo = vd[:len(vd) - len(current_common_bytes())]
    parsed = P._parse_prover_only(_upstream_shaped([int(x) for x in dig]), nz)
    assert parsed[:2] == (None, None)
    assert P._same_preprocessing(vo, parsed[2])
    other = [int(dig[0]) ^ 1] + [int(x) for x in dig[1:]]
    assert not P._same_preprocessing(vo, P._parse_prover_only(_upstream_shaped(other), nz)[2])
    # a file with lookup tables (non-empty tail) or no generators is not taken for one
    assert P.upstream_prover_digest(_upstream_shaped(dig)[:-8] + struct.pack("<Q", 1)) is None
    assert P.upstream_prover_digest(_upstream_shaped(dig, ngen=0)) is None


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
