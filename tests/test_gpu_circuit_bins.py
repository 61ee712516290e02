"""Circuit binaries: generate_circuit_binaries writes
common.bin / verifier.bin / prover.bin (wormhole/circuit-builder/src/lib.rs:11-66);
WormholeProver.new_from_bytes / new_from_files / default load them
(wormhole/prover/src/lib.rs:81-187) with the reference's error messages, and
the loaded prover's proofs verify under the written verifier.bin."""
import os

import pytest

import wormhole_inputs as WI
from oracle_lib import lib as olib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bins(tmp_path_factory):
    import qp_wormhole
    d = tmp_path_factory.mktemp("generated-bins")
    qp_wormhole.generate_circuit_binaries(str(d), include_prover=True)
    return d


def test_binaries_written(bins):
    import qp_wormhole
    common = open(bins / "common.bin", "rb").read()
    assert common == qp_wormhole.Circuit.wormhole().common_data()
    assert len(open(bins / "verifier.bin", "rb").read()) == 8 + 16 * 32 + 32  # as bench-data/verifier.bin
    assert open(bins / "prover.bin", "rb").read().startswith(b"QPGPU-PROVER-ONLY")


def test_new_from_files_proves_and_verifies(bins):
    from qp_wormhole import WormholeProver
    p = WormholeProver.new_from_files(bins / "prover.bin", bins / "common.bin")
    proof = p.commit(WI.test_inputs()).prove()
    vd = open(bins / "verifier.bin", "rb").read()
    common = open(bins / "common.bin", "rb").read()
    pb = proof.to_bytes()
    assert olib().ora_verify(vd + common, len(vd) + len(common), pb, len(pb)) == 0


def test_new_from_bytes_errors(bins):
    from qp_wormhole import WormholeProver
    common = open(bins / "common.bin", "rb").read()
    prover = open(bins / "prover.bin", "rb").read()
    assert WormholeProver.new_from_bytes(prover, common).config == "standard_recursion_config"
    with pytest.raises(ValueError, match="Failed to deserialize common circuit data"):
        WormholeProver.new_from_bytes(prover, common[:-1])
    with pytest.raises(ValueError, match="Failed to deserialize prover only data"):
        WormholeProver.new_from_bytes(b"junk" + prover, common)
    bad = bytearray(prover)
    bad[-1] ^= 1  # the stored commitment
    with pytest.raises(ValueError, match="commitment differs"):
        WormholeProver.new_from_bytes(bytes(bad), common)


def test_new_from_bytes_takes_an_upstream_prover_bin(bins):
    """A ProverOnlyCircuitData::to_bytes-framed file carrying the Wormhole circuit
    digest (the reference's generate_circuit_binaries output) loads, proves and
    verifies; one with another digest is refused."""
    import struct
    import numpy as np
    import qp_wormhole
    from qp_wormhole import WormholeProver
    from upstream_prover_bin import upstream_prover_bin
    common = open(bins / "common.bin", "rb").read()
    vo = open(bins / "verifier.bin", "rb").read()
    dig = struct.unpack_from("<4Q", vo, len(vo) - 32)
    circ = qp_wormhole.Circuit.wormhole()
    up = upstream_prover_bin(circ, np.frombuffer(vo, np.uint64, 64, 8), dig)
    wp = WormholeProver.new_from_bytes(up, common)
    proof = wp.commit(WI.test_inputs()).prove()
    vd = vo + common
    from oracle_lib import lib as olib
    pb = proof.to_bytes()
    assert olib().ora_verify(vd, len(vd), pb, len(pb)) == 0
    bad = upstream_prover_bin(circ, np.frombuffer(vo, np.uint64, 64, 8), [dig[0] ^ 1] + list(dig[1:]))
    with pytest.raises(ValueError, match="commitment differs"):
        WormholeProver.new_from_bytes(bad, common)
    foreign = struct.pack("<Q", 1500) + b"\x11" * 40000 + struct.pack("<4Q", *dig) + bytes(16)
    with pytest.raises(ValueError, match="not found"):
        WormholeProver.new_from_bytes(foreign, common)


def test_zk_binaries_and_default(bins, tmp_path, monkeypatch):
    import qp_wormhole
    from qp_wormhole import WormholeProver
    qp_wormhole.generate_circuit_binaries(str(tmp_path / "zk"), config="standard_recursion_zk_config")
    p = WormholeProver.new_from_files(tmp_path / "zk" / "prover.bin", tmp_path / "zk" / "common.bin")
    assert p.config == "standard_recursion_zk_config"
    # prover.bin of one config does not load with the other's common data
    with pytest.raises(ValueError, match="different common data"):
        WormholeProver.new_from_files(tmp_path / "zk" / "prover.bin", bins / "common.bin")
    # default(): generated-bins/ in the working directory, else a fresh build
    monkeypatch.chdir(tmp_path)
    assert WormholeProver.default().config == "standard_recursion_config"
    os.makedirs("generated-bins")
    for f in ("prover.bin", "common.bin"):
        open(os.path.join("generated-bins", f), "wb").write(open(tmp_path / "zk" / f, "rb").read())
    assert WormholeProver.default().config == "standard_recursion_zk_config"
