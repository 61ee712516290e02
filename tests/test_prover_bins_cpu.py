"""prover.bin parsing on the host (no GPU): this backend's format only, with
clear errors for an upstream plonky2 ProverOnlyCircuitData file and for a
header that disagrees with the common data (wormhole/prover/src/lib.rs:105-187)."""
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


def test_upstream_prover_bin_is_rejected_clearly():
    nz = P._common_of("standard_recursion_config")
    with pytest.raises(ValueError, match="upstream plonky2 ProverOnlyCircuitData"):
        P._parse_prover_only(b"\x05\x00\x00\x00" + b"\x11" * 200, nz)


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
