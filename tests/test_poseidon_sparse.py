"""The sparse partial-round form of Poseidon used by the GPU hashing kernels
(tools/gen_poseidon_partial.py -> csrc/poseidon_partial_consts.h) is the same
permutation as the plain rounds (poseidon.h / the oracle), and the committed
header is what the generator produces."""
import importlib.util
import os
import random

import numpy as np

from oracle_lib import permute as ora_permute

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gen():
    spec = importlib.util.spec_from_file_location("gen_poseidon_partial",
                                                  os.path.join(ROOT, "tools", "gen_poseidon_partial.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_sparse_rounds_equal_plain_and_oracle():
    g = _gen()
    A, init_rows, init_k, kscalar, c26 = g.derive()
    rnd = random.Random(1)
    states = [[0] * 12, [g.P - 1] * 12] + [[rnd.randrange(g.P) for _ in range(12)] for _ in range(8)]
    for s in states:
        fast = g.permute_fast(s, A, init_rows, init_k, kscalar, c26)
        assert fast == g.permute_plain(s)
        assert fast == [int(x) for x in ora_permute(np.array(s, np.uint64))]
        # grouped form (lane 1..11 updates deferred over G rounds, gamma terms)
        for G in (2, 3, 4, 5):
            assert g.permute_fast_grouped(s, A, init_rows, init_k, kscalar, c26, G) == fast


def test_committed_header_is_generated(tmp_path, monkeypatch):
    g = _gen()
    out = tmp_path / "h.h"
    monkeypatch.setattr(g, "HDR", str(out))
    g.emit(*g.derive())
    with open(os.path.join(ROOT, "qp-zk-circuits-rm_amd", "csrc", "poseidon_partial_consts.h")) as f:
        assert f.read() == out.read_text()


def test_dot_pieces_bounds():
    """AH2 pieces are 22/22/20 bits, so 22 products with 32-bit halves stay
    below 2^59 in each accumulator (the device combine relies on it)."""
    g = _gen()
    A = g.derive()[0]
    for r in range(4, 26):
        for j in range(11):
            for h in range(2):
                c = A[r][0][j] * (1 << (32 * h)) % g.P
                assert (c & 0x3FFFFF) < 1 << 22 and ((c >> 22) & 0x3FFFFF) < 1 << 22 and (c >> 44) < 1 << 20
    assert 22 * (2**32 - 1) * (2**22 - 1) + 25 * 2**32 + 2**32 < 2**59
