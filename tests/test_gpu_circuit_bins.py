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


def test_binaries_written(bins, tmp_path):
    """prover.bin is upstream ProverOnlyCircuitData::to_bytes by default (its
    commitment equal to the written verifier.bin's, i.e. the device prover's);
    prover_format="backend" writes this backend's identity + commitment blob."""
    import struct
    import qp_wormhole
    from qp_wormhole.prover import read_upstream_prover_only
    common = open(bins / "common.bin", "rb").read()
    assert common == qp_wormhole.Circuit.wormhole().common_data()
    vo = open(bins / "verifier.bin", "rb").read()
    assert len(vo) == 8 + 16 * 32 + 32  # as bench-data/verifier.bin
    f = read_upstream_prover_only(open(bins / "prover.bin", "rb").read())
    assert f["cap"].tobytes() == vo[8:8 + 512] and f["circuit_digest"] == struct.unpack_from("<4Q", vo, 8 + 512)
    qp_wormhole.generate_circuit_binaries(str(tmp_path), prover_format="backend")
    assert open(tmp_path / "prover.bin", "rb").read().startswith(b"QPGPU-PROVER-ONLY")


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
    bad[-17] ^= 1  # the stored circuit digest
    with pytest.raises(ValueError, match="Failed to deserialize prover only data"):
        WormholeProver.new_from_bytes(bytes(bad), common)


def test_new_from_bytes_backend_blob_and_commitment(bins, tmp_path):
    """This backend's prover.bin loads too; one whose stored commitment differs
    from the circuit's is refused."""
    import qp_wormhole
    from qp_wormhole import WormholeProver
    common = open(bins / "common.bin", "rb").read()
    qp_wormhole.generate_circuit_binaries(str(tmp_path), prover_format="backend")
    blob = open(tmp_path / "prover.bin", "rb").read()
    wp = WormholeProver.new_from_bytes(blob, common)
    pb = wp.commit(WI.test_inputs()).prove().to_bytes()
    vd = open(bins / "verifier.bin", "rb").read() + common
    assert olib().ora_verify(vd, len(vd), pb, len(pb)) == 0
    bad = bytearray(blob)
    bad[-1] ^= 1  # the stored commitment
    with pytest.raises(ValueError, match="commitment differs"):
        WormholeProver.new_from_bytes(bytes(bad), common)


def test_zk_binaries_and_default(bins, tmp_path, monkeypatch):
    import qp_wormhole
    from qp_wormhole import WormholeProver
    qp_wormhole.generate_circuit_binaries(str(tmp_path / "zk"), config="standard_recursion_zk_config")
    p = WormholeProver.new_from_files(tmp_path / "zk" / "prover.bin", tmp_path / "zk" / "common.bin")
    assert p.config == "standard_recursion_zk_config"
    # the two configs share their preprocessing (no salt, no blinding rows under
    # no_random), so their upstream prover.bin is the same file; the common data
    # decides the config.  This backend's blob names its common data and refuses
    # the other config's
    assert open(tmp_path / "zk" / "prover.bin", "rb").read() == open(bins / "prover.bin", "rb").read()
    assert WormholeProver.new_from_files(tmp_path / "zk" / "prover.bin", bins / "common.bin").config == \
        "standard_recursion_config"
    qp_wormhole.generate_circuit_binaries(str(tmp_path / "zkb"), config="standard_recursion_zk_config",
                                          prover_format="backend")
    with pytest.raises(ValueError, match="different common data"):
        WormholeProver.new_from_files(tmp_path / "zkb" / "prover.bin", bins / "common.bin")
    # default(): generated-bins/ in the working directory, else a fresh build
    monkeypatch.chdir(tmp_path)
    assert WormholeProver.default().config == "standard_recursion_config"
    os.makedirs("generated-bins")
    for f in ("prover.bin", "common.bin"):
        open(os.path.join("generated-bins", f), "wb").write(open(tmp_path / "zk" / f, "rb").read())
    assert WormholeProver.default().config == "standard_recursion_zk_config"
