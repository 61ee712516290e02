"""CPU-side checks of the C ABI boundary: the library loads, exports every
symbol include/qpgpu.h declares, and the product's Poseidon constants are the
pinned plonky2 table."""
import hashlib
import os
import re
import struct

import qp_wormhole
from qp_wormhole import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RC_SHA = "d2fcbb5be293c50ab4b1ddcd9c81005b12d689816a54c91a054f97f6588a20a8"


def test_library_exports_header_symbols():
    L = qp_wormhole.lib()
    syms = qp_wormhole.header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), s
    assert b"gfx950" in L.qp_version()


def test_product_round_constants_pinned():
    src = open(os.path.join(ROOT, "qp-zk-circuits-rm_amd", "csrc", "poseidon.h")).read()
    block = src[src.index("#define QP_POSEIDON_RC_LIST"):src.index("static const uint64_t RC_HOST")]
    vals = [int(x, 16) for x in re.findall(r"0x([0-9a-f]{16})ULL", block)]
    assert len(vals) == 360
    assert hashlib.sha256(b"".join(struct.pack("<Q", v) for v in vals)).hexdigest() == RC_SHA


def test_oracle_round_constants_pinned():
    src = open(os.path.join(ROOT, "oracle", "poseidon.c")).read()
    vals = [int(x, 16) for x in re.findall(r"0x([0-9a-f]{16})ULL", src)]
    assert len(vals) == 360
    assert hashlib.sha256(b"".join(struct.pack("<Q", v) for v in vals)).hexdigest() == RC_SHA


def test_no_device_fails_loudly():
    # in the CPU container there is no HIP device: context creation must fail with a status
    import ctypes
    h = ctypes.c_void_p()
    rc = _native.lib().qp_ctx_create(0, ctypes.byref(h))
    if rc == 0:  # running on a GPU box
        _native.lib().qp_ctx_destroy(h)
    else:
        assert rc == 2
