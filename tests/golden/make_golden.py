"""Regenerates the small golden fixtures in tests/golden/ from the reference.

Run in the build container only (the GPU box has no /root/reference):
    python tests/golden/make_golden.py
Outputs (data only, no reference source):
  * common.bin, verifier.bin, proof.bin      <- wormhole/bench-data/*.bin
  * dummy_proof.bin, dummy_proof_zk.bin      <- wormhole/aggregator/data/*.bin
    (also into qp-zk-circuits-rm_amd/qp_wormhole/data/: the aggregator's padding
    proofs, as util.rs:6-9 include_bytes! them)
  * storage_proof.json <- the DEFAULT_STORAGE_PROOF node hex strings and indices of
    wormhole/tests/test-helpers/src/lib.rs:64-80 (test input data)
"""
import json
import os
import re
import shutil

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
PKG_DATA = os.path.join(HERE, "..", "..", "qp-zk-circuits-rm_amd", "qp_wormhole", "data")


def main():
    for sub, names in (("wormhole/bench-data", ["common.bin", "verifier.bin", "proof.bin"]),
                       ("wormhole/aggregator/data", ["dummy_proof.bin", "dummy_proof_zk.bin"])):
        for n in names:
            shutil.copyfile(os.path.join(REF, sub, n), os.path.join(HERE, n))
            if n.startswith("dummy_proof"):
                shutil.copyfile(os.path.join(REF, sub, n), os.path.join(PKG_DATA, n))
    src = open(os.path.join(REF, "wormhole/tests/test-helpers/src/lib.rs")).read()
    block = src[src.index("DEFAULT_STORAGE_PROOF: [&str; 7]"):]
    block = block[:block.index("];")]
    nodes = re.findall(r'"([0-9a-f]+)"', block)
    idx_src = src[src.index("DEFAULT_STORAGE_PROOF_INDICIES"):]
    idx = [int(x) for x in re.findall(r"\[([0-9, ]+)\]", idx_src)[0].split(",")]
    assert len(nodes) == 7 and len(idx) == 7
    with open(os.path.join(HERE, "storage_proof.json"), "w") as f:
        json.dump({"nodes": nodes, "indices": idx,
                   "source": "wormhole/tests/test-helpers/src/lib.rs:64-80"}, f, indent=1)


if __name__ == "__main__":
    main()
