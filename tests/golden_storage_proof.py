"""Loads tests/golden/storage_proof.json (made by tests/golden/make_golden.py)."""
import json
import os

_d = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "storage_proof.json")))
DEFAULT_STORAGE_PROOF = _d["nodes"]
DEFAULT_STORAGE_PROOF_INDICES = _d["indices"]
