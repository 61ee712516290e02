"""sha256[:16] of the in-tree libqpgpu.so: stamped into every profile summary
(tools/kernel_summary.py, pmc_summary.py, pmc_sq_summary.py, issue_ceiling.py)
so bench.py reports a profile-derived field as this build's only when the
stamp matches the library it loaded."""
import hashlib
import os

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qp-zk-circuits-rm_amd",
                   "qp_wormhole", "libqpgpu.so")


def lib_sha16(path=None):
    p = path or os.environ.get("QPGPU_LIB") or LIB
    try:
        return hashlib.sha256(open(p, "rb").read()).hexdigest()[:16]
    except OSError:
        return None
