"""Recursive tree aggregation of leaf proofs on the MI355X prover — the host
mirror of qp-wormhole-aggregator (wormhole/aggregator/src):

* TreeAggregationConfig, AggregatedProof   circuits/tree.rs:17-53
* aggregate_to_tree / aggregate_level /
  aggregate_chunk                           circuits/tree.rs:55-143
* WormholeProofAggregator                  aggregator.rs:13-92
* pad_with_dummy_proofs                    util.rs:11-29
* PublicCircuitInputs.try_from_aggregated  wormhole/circuit/src/inputs.rs:57-131

aggregate_chunk's circuit (add_virtual_verifier_data + verify_proof per
proof + register_public_inputs) is the native recursive verifier
(csrc/recursion.cpp); its witness is generated on the host and every level's
chunks are proven in ONE batched GPU launch sequence (the reference proves
chunks one by one, with rayon across chunks).  The reference rebuilds the
circuit for every chunk (tree.rs:111-127); here a level's circuit and its
device preprocessing are built once per (inner circuit, branching) and cached.
The aggregation circuit is parity-unpinned: the reference commits no
aggregated proof.
"""
import os
import struct
import threading
from dataclasses import dataclass
from typing import List, Optional

from ._native import Context, QpError
from .circuits import Circuit, PublicCircuitInputs
from .prover import ProofWithPublicInputs, Prover

DEFAULT_TREE_BRANCHING_FACTOR = 2  # tree.rs:17
DEFAULT_TREE_DEPTH = 3             # tree.rs:20
LEAF_PI_LEN = 16                   # inputs.rs:91


@dataclass
class TreeAggregationConfig:
    """tree.rs:30-53: num_leaf_proofs = branching ** depth."""
    num_leaf_proofs: int
    tree_branching_factor: int
    tree_depth: int

    @classmethod
    def new(cls, tree_branching_factor: int, tree_depth: int):
        return cls(tree_branching_factor ** tree_depth, tree_branching_factor, tree_depth)

    @classmethod
    def default(cls):
        return cls.new(DEFAULT_TREE_BRANCHING_FACTOR, DEFAULT_TREE_DEPTH)


@dataclass
class CircuitData:
    """The parts of plonky2 CircuitData an aggregation level hands to the next:
    CommonCircuitData bytes and VerifierOnlyCircuitData bytes (cap height, cap,
    circuit digest)."""
    common: bytes
    verifier_only: bytes

    def verifier_data(self) -> bytes:
        """verifier.bin layout: VerifierOnlyCircuitData || CommonCircuitData."""
        return self.verifier_only + self.common


@dataclass
class AggregatedProof:
    """tree.rs:22-27."""
    proof: ProofWithPublicInputs
    circuit_data: CircuitData


class _LevelProver:
    """One aggregation circuit (inner common data, branching) with its device
    provers: QP_AGG_PROVERS (default 2; 3 raises a level's throughput but not the
    256-leaf subtree inside bench.py, profiles/r04_agg_provers_ab.log) contexts,
    each with its own HIP stream
    and workspace, so one prover's host phases (transcript, query assembly)
    overlap the other's kernels, as the leaf bench's provers do."""

    def __init__(self, inner_common: bytes, branching: int, device: int, max_batch: int, nprov: int = 0):
        self.circuit = aggregation_circuit(inner_common, branching)
        self.max_batch = max_batch
        if not nprov:
            nprov = _agg_provers() if max_batch > 1 else 1
        # (a high-priority stream for the level provers changed nothing next to
        # concurrent leaf provers: profiles/r05_configs3_pipelined_ab.log)
        ctxs = [Context(device) for _ in range(nprov)]
        self.provers = [Prover(c, self.circuit, max_batch=max_batch) for c in ctxs]
        # the provers split the process's host budget (qp_prover_set_host_threads:
        # each would otherwise take min(hardware threads, 16))
        for p in self.provers:
            p.set_host_threads(max(1, _host_budget() // nprov))
        self.prover = self.provers[0]
        vd = self.prover.verifier_data()
        common = self.circuit.common_data()
        assert vd.endswith(common)
        self.data = CircuitData(common, vd[:len(vd) - len(common)])
        self.lock = threading.Lock()  # the host-witness path's
        self.locks = [threading.Lock() for _ in self.provers]

    def prove_chunks(self, chunks, inner_vo: bytes, prover: Optional[int] = None) -> List[AggregatedProof]:
        """Every chunk aggregated: split evenly over the provers, or all on
        provers[prover] (a sub-tree's thread, see aggregate_to_tree)."""
        if os.environ.get("QP_AGG_WITNESS", "device") == "host":
            return self._prove_chunks_host(chunks, inner_vo)
        # device witness generation (qp_prover_prove_aggregation): the host only
        # deserializes the inner proofs into the circuit's input targets; the
        # chunks are split evenly over the provers, each proving its share in
        # batches of max_batch on its own stream
        npis = self.circuit.num_public_inputs
        if prover is not None:
            sel = [prover % len(self.provers)]
            per, first = [len(chunks)], [0]
        else:
            sel = list(range(min(len(self.provers), len(chunks))))
            per = [len(chunks) // len(sel) + (1 if i < len(chunks) % len(sel) else 0) for i in range(len(sel))]
            first = [sum(per[:i]) for i in range(len(sel))]
        outs = [None] * len(sel)
        errors = []

        def run(j):
            i = sel[j]
            try:
                res = []
                mine = chunks[first[j]:first[j] + per[j]]
                with self.locks[i]:
                    for k in range(0, len(mine), self.max_batch):
                        grp = mine[k:k + self.max_batch]
                        res += self.provers[i].prove_aggregation(inner_vo, [[p.to_bytes() for p in ch] for ch in grp])
                outs[j] = res
            except BaseException as e:  # re-raised on the calling thread
                errors.append(e)

        if len(sel) == 1:
            run(0)
        else:
            th = [threading.Thread(target=run, args=(j,)) for j in range(len(sel))]
            for t in th:
                t.start()
            for t in th:
                t.join()
        if errors:
            raise errors[0]
        out = []
        for data in (d for o in outs for d in o):
            pis = struct.unpack_from(f"<{npis}Q", data, len(data) - 8 * npis)
            out.append(AggregatedProof(ProofWithPublicInputs(data, pis), self.data))
        return out

    def _prove_chunks_host(self, chunks, inner_vo: bytes) -> List[AggregatedProof]:
        # aggregate_chunk's witnesses on host threads (the C call releases the GIL;
        # ~50 ms each for two leaves), each max_batch group proven on the GPU as
        # soon as its witnesses exist while the next group's are generated
        def commit(ch):
            return self.circuit.commit_proofs(inner_vo, [p.to_bytes() for p in ch])

        futs = [_witness_pool().submit(commit, ch) for ch in chunks]
        out = []
        try:
            with self.lock:
                for i in range(0, len(futs), self.max_batch):
                    ws = [f.result() for f in futs[i:i + self.max_batch]]
                    for w, data in zip(ws, self.prover.prove_witnesses(ws)):
                        out.append(AggregatedProof(ProofWithPublicInputs(data, w.public_inputs()), self.data))
        finally:
            for f in futs:
                if f.done() and f.exception() is None:
                    f.result().free()
        return out


# the GPU prover's largest circuit (prover.cpp setup): n <= 2^15, its LDE of
# 2^18 points within the twiddle tables (n > 2^14 runs the HBM-level NTTs)
GPU_MAX_DEGREE_BITS = 15

_circuits = {}
_circuits_lock = threading.Lock()


def aggregation_circuit(inner_common: bytes, branching: int) -> Circuit:
    """aggregate_chunk's circuit for (inner common data, branching), built once."""
    key = (bytes(inner_common), branching)
    with _circuits_lock:
        c = _circuits.get(key)
        if c is None:
            c = _circuits[key] = Circuit.aggregation(inner_common, branching)
        return c


_pool = None


def _cores_per_rank() -> int:
    """The cores this process may use (affinity mask, capped by a cgroup v2 cpu.max
    quota) divided among the node's local ranks (LOCAL_WORLD_SIZE)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 4
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return max(1, n // max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1"))))


def _host_budget() -> int:
    """Host threads aggregation may use: QP_AGG_THREADS, else the larger of
    OMP_NUM_THREADS (the GPU boxes' per-job share) and this rank's share of the
    usable cores (torchrun sets OMP_NUM_THREADS=1 for its workers when the
    environment has none), at most 16."""
    if os.environ.get("QP_AGG_THREADS"):
        return max(1, min(int(os.environ["QP_AGG_THREADS"]), 16))
    n = max(int(os.environ.get("OMP_NUM_THREADS") or 0), _cores_per_rank())
    return max(1, min(n, 16))


def _witness_pool():
    """Host threads for aggregation witnesses (the host-witness path)."""
    global _pool
    if _pool is None:
        import concurrent.futures
        _pool = concurrent.futures.ThreadPoolExecutor(max_workers=_host_budget())
    return _pool


_levels = {}
_levels_lock = threading.Lock()


def _agg_provers() -> int:
    """Device provers per aggregation level (QP_AGG_PROVERS, default 2)."""
    return max(1, int(os.environ.get("QP_AGG_PROVERS", "2")))


def _level_prover(inner_common: bytes, branching: int, device: int, max_batch: int,
                  nprov: int = 0) -> _LevelProver:
    """The cached level prover of (inner circuit, branching, device), rebuilt when
    a call needs a larger batch or more provers than it has (nprov 0: the
    default count)."""
    key = (bytes(inner_common), branching, device)
    with _levels_lock:
        lp = _levels.get(key)
        if lp is None or lp.max_batch < max_batch or len(lp.provers) < nprov:
            lp = _LevelProver(inner_common, branching, device, max(max_batch, lp.max_batch if lp else 0),
                              max(nprov, len(lp.provers) if lp else 0))
            _levels[key] = lp
        return lp


def _as_proof(p) -> ProofWithPublicInputs:
    return p if isinstance(p, ProofWithPublicInputs) else ProofWithPublicInputs(bytes(p), [])


def aggregate_chunk(chunk, common_data: bytes, verifier_only: bytes, device: int = 0,
                    backend=None) -> AggregatedProof:
    """tree.rs:106-143: verify every proof of the chunk in one circuit and prove it."""
    return aggregate_level(list(chunk), common_data, verifier_only, TreeAggregationConfig.new(len(chunk), 1),
                           device, backend)[0]


def aggregate_level(proofs, common_data: bytes, verifier_only: bytes, config: TreeAggregationConfig,
                    device: int = 0, backend=None, prover: Optional[int] = None,
                    nprov: int = 0) -> List[AggregatedProof]:
    """tree.rs:80-103: chunks of `tree_branching_factor` proofs, each aggregated
    (all chunks of the level proven as one GPU batch).  backend(inner_common,
    branching, device, max_batch) -> an object with .data and .prove_chunks()
    (default: the GPU level prover; tests inject a CPU one).  prover: the level
    prover's device prover that takes every chunk (a sub-tree's thread);
    nprov: the device provers the cached level prover must have (the sub-tree
    threads all pass the same count, so the first call builds it once)."""
    k = config.tree_branching_factor
    proofs = [_as_proof(p) for p in proofs]
    if not proofs or k < 1:
        raise ValueError("aggregate_level: no proofs / branching factor < 1")
    chunks = [proofs[i:i + k] for i in range(0, len(proofs), k)]
    # proofs.chunks(k) (tree.rs:86-89): a shorter last chunk is aggregated by a
    # circuit built for its own size (the next level can only take its proof
    # if it is alone, as in the reference, whose next level uses proofs[0]'s
    # circuit data for every proof)
    tail = chunks.pop() if len(chunks[-1]) != k else None
    out = []
    if backend is not None:
        if chunks:
            out = backend(common_data, k, device, max(1, min(len(chunks), 32))).prove_chunks(chunks, verifier_only)
        if tail is not None:
            out += backend(common_data, len(tail), device, 1).prove_chunks([tail], verifier_only)
        return out
    if prover is not None:
        nprov = max(nprov, prover + 1, _agg_provers())
    if chunks:
        # up to 32 aggregation proofs per GPU batch (2.7 vs 3.2 ms per proof at 16;
        # tools/agg_bench.py, profiles/r03_agg_bench.log)
        out = _level_prover(common_data, k, device, max(1, min(len(chunks), 32)), nprov).prove_chunks(
            chunks, verifier_only, prover)
    if tail is not None:
        out += _level_prover(common_data, len(tail), device, 1, nprov).prove_chunks([tail], verifier_only, prover)
    return out


class CircuitTooLarge(ValueError):
    """A tree level's aggregation circuit exceeds the GPU prover's size; .proofs
    holds the level below it (the highest level that could be proven)."""

    def __init__(self, msg, proofs):
        super().__init__(msg)
        self.proofs = proofs


def _too_large(config, backend, inner_common, proofs):
    """The degree of the first circuit a level over `proofs` would build that
    exceeds the GPU prover (full chunks of k and a shorter tail), else None."""
    if backend is not None:
        return None
    k = config.tree_branching_factor
    sizes = ([k] if len(proofs) >= k else []) + ([len(proofs) % k] if len(proofs) % k else [])
    for size in sizes:
        c = aggregation_circuit(inner_common, size)
        if c.degree_bits > GPU_MAX_DEGREE_BITS:
            return c.degree_bits
    return None


def _levels_down(proofs, config, device, backend, prover=None, nprov=0):
    """Levels down to one proof; returns (proofs, None) or (the last level
    proven, the message of the circuit that was too large)."""
    while len(proofs) > 1:
        cd = proofs[0].circuit_data
        db = _too_large(config, backend, cd.common, proofs)
        if db is not None:
            return proofs, (f"the next level's aggregation circuit is 2^{db} rows (its public inputs: every "
                            f"leaf's); the GPU prover proves up to 2^{GPU_MAX_DEGREE_BITS}")
        proofs = aggregate_level([p.proof for p in proofs], cd.common, cd.verifier_only, config, device,
                                 backend, prover, nprov)
    return proofs, None


def _sub_trees(part_leaves, parts, common_data, verifier_only, config, device, backend):
    """`parts` independent sub-trees, one thread and one device prover each,
    with no level barrier between them, so one sub-tree's host phases and
    latency-bound launches overlap the others' kernels; part_leaves(i) gives
    sub-tree i's leaf proofs (it may block until they exist).  Returns the
    sub-tree roots in order (CircuitTooLarge if a level is beyond the GPU)."""
    # one device prover per sub-tree, the same count for every thread (so no
    # thread rebuilds a level prover another thread has just built)
    nprov = max(parts, _agg_provers())
    res = [None] * parts
    errors = []

    def run(i):
        try:
            lv = aggregate_level(part_leaves(i), common_data, verifier_only, config, device, backend, i, nprov)
            res[i] = _levels_down(lv, config, device, backend, i, nprov)
        except BaseException as e:  # re-raised on the calling thread
            errors.append(e)

    th = [threading.Thread(target=run, args=(i,)) for i in range(parts)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errors:
        raise errors[0]
    msg = next((r[1] for r in res if r[1]), None)
    proofs = [p for r in res for p in r[0]]
    if msg:
        raise CircuitTooLarge(msg, proofs)
    return proofs


def aggregate_to_tree(leaf_proofs, common_data: bytes, verifier_only: bytes,
                      config: Optional[TreeAggregationConfig] = None, device: int = 0,
                      backend=None) -> AggregatedProof:
    """tree.rs:55-77: aggregate the first level, then each next level with the
    previous level's circuit data, down to one root proof.  Every leaf's public
    inputs are registered at every level, so circuits grow with the depth (the
    root of 2048 leaves registers 32,768 and needs 2^15 rows): a level whose
    circuit exceeds the GPU prover's 2^GPU_MAX_DEGREE_BITS raises
    CircuitTooLarge carrying the proofs of the level below (not with a CPU
    backend).  Large trees run as concurrent sub-trees (_subtree_parts: the
    same chunks as the level-by-level order, so the same proofs)."""
    config = config or TreeAggregationConfig.default()
    db = _too_large(config, backend, common_data, leaf_proofs)
    if db is not None:
        raise CircuitTooLarge(f"level-1 aggregation circuit is 2^{db} rows", [])
    parts = _subtree_parts(len(leaf_proofs), config.tree_branching_factor) if backend is None else 1
    if parts > 1:
        m = len(leaf_proofs) // parts
        proofs = _sub_trees(lambda i: leaf_proofs[i * m:(i + 1) * m], parts, common_data, verifier_only, config,
                            device, backend)
    else:
        proofs = aggregate_level(leaf_proofs, common_data, verifier_only, config, device, backend)
    proofs, msg = _levels_down(proofs, config, device, backend)
    if msg:
        raise CircuitTooLarge(msg, proofs)
    assert len(proofs) == 1
    return proofs[0]


def aggregate_to_tree_streamed(part_leaves, parts: int, common_data: bytes, verifier_only: bytes,
                               config: Optional[TreeAggregationConfig] = None, device: int = 0,
                               backend=None) -> AggregatedProof:
    """aggregate_to_tree over leaves that arrive one complete sub-tree at a
    time: part_leaves(i) blocks until sub-tree i's leaf proofs exist (a
    producer proving them in order), and each sub-tree is aggregated on its
    own thread as soon as they do, while the producer proves the next part's
    leaves -- so the sub-trees' latency-bound upper levels overlap the later
    leaves' kernels instead of idling the GPU at the end.  The parts are the
    consecutive leaf ranges of aggregate_to_tree's sub-trees, so the root is
    the same proof (same chunks, same order).  parts must be a power of the
    branching factor."""
    config = config or TreeAggregationConfig.default()
    k = config.tree_branching_factor
    p = parts
    while p % k == 0 and p > 1:
        p //= k
    if parts < 1 or p != 1:
        raise ValueError(f"{parts} parts are not a power of the branching factor {k}")
    proofs = _sub_trees(part_leaves, parts, common_data, verifier_only, config, device, backend)
    proofs, msg = _levels_down(proofs, config, device, backend)
    if msg:
        raise CircuitTooLarge(msg, proofs)
    assert len(proofs) == 1
    return proofs[0]


SUBTREE_MIN_LEAVES = 32


def _subtree_parts(n: int, k: int) -> int:
    """Sub-trees aggregate_to_tree proves concurrently: QP_AGG_SPLIT (default
    4) when n leaves split into that many complete k-ary sub-trees of at least
    SUBTREE_MIN_LEAVES leaves each, else 1.  256-leaf subtree: 0.376 s level
    by level, 0.378 s as 2 sub-trees, 0.343-0.359 s as 4, 0.37-0.38 s as 8; a
    tree of 8 leaves as 4 sub-trees of 2: 35 ms against 28 level by level
    (profiles/r05_ab_subtree_split.log)."""
    s = int(os.environ.get("QP_AGG_SPLIT") or 4)
    if s < 2 or k < 2 or n % s or n // s < max(k, SUBTREE_MIN_LEAVES):
        return 1
    m = n // s
    while m % k == 0:
        m //= k
    return s if m == 1 else 1


def pad_with_dummy_proofs(proofs, proof_len: int, dummy_proof) -> list:
    """util.rs:11-29 (the dummy is a proof of the leaf circuit on the default
    test inputs, as the reference's dummy_proof*.bin)."""
    if len(proofs) > proof_len:
        raise ValueError("proofs to aggregate was more than the maximum allowed")
    return list(proofs) + [dummy_proof] * (proof_len - len(proofs))


def _felts_to_digest(f) -> bytes:
    return b"".join(int(x).to_bytes(8, "little") for x in f)


def public_inputs_from_slice(pis) -> PublicCircuitInputs:
    """PublicCircuitInputs::try_from_slice (inputs.rs:91-131)."""
    if len(pis) != LEAF_PI_LEN:
        raise ValueError(f"public inputs should contain: {LEAF_PI_LEN} field elements, got: {len(pis)}")
    amount = 0
    for i, x in enumerate(pis[8:12]):
        if int(x) >> 32:
            raise ValueError("failed to deserialize funding amount")
        amount |= int(x) << (96 - 32 * i)
    return PublicCircuitInputs(funding_amount=amount, nullifier=_felts_to_digest(pis[0:4]),
                               root_hash=_felts_to_digest(pis[4:8]), exit_account=_felts_to_digest(pis[12:16]))


def public_inputs_from_aggregated(aggr: ProofWithPublicInputs, leaf_pi_len: int, num_leaves: int):
    """PublicCircuitInputs::try_from_aggregated (inputs.rs:57-89)."""
    pis = list(aggr.public_inputs)
    expected = leaf_pi_len * num_leaves
    if len(pis) != expected:
        raise ValueError(f"aggregated public inputs should contain: {expected} (= {num_leaves} leaves × "
                         f"{leaf_pi_len} fields), got: {len(pis)}")
    return [public_inputs_from_slice(pis[i:i + leaf_pi_len]) for i in range(0, len(pis), leaf_pi_len)]


class WormholeProofAggregator:
    """aggregator.rs:13-92 over this library's Wormhole leaf circuit."""

    def __init__(self, leaf_circuit_data: CircuitData, dummy_proof: Optional[ProofWithPublicInputs] = None,
                 device: int = 0):
        self.leaf_circuit_data = leaf_circuit_data
        self.config = TreeAggregationConfig.default()
        self.proofs_buffer = []
        self.device = device
        self._dummy = dummy_proof

    @classmethod
    def from_circuit_config(cls, config: str = "standard_recursion_zk_config", device: int = 0):
        """aggregator.rs:40-45 (the leaf verifier data of WormholeVerifier::new(config))."""
        from .prover import WormholeProver, _verifier_only
        wp = WormholeProver(config, device)
        with wp._prove_lock:
            vo = _verifier_only(wp.circuit, wp.prover)
        return cls(CircuitData(wp.circuit.common_data(), vo), device=device)

    @classmethod
    def default(cls, device: int = 0):
        """aggregator.rs:19-24: standard_recursion_zk_config."""
        return cls.from_circuit_config("standard_recursion_zk_config", device)

    def with_config(self, config: TreeAggregationConfig):
        self.config = config
        return self

    def push_proof(self, proof):
        if len(self.proofs_buffer) >= self.config.num_leaf_proofs:
            raise ValueError("tried to add proof when proof buffer is full")
        self.proofs_buffer.append(_as_proof(proof))

    def dummy_proof(self) -> ProofWithPublicInputs:
        """The padding proof: util.rs:6-9 embeds the reference's own proof of its
        test inputs (dummy_proof_zk.bin, or dummy_proof.bin under the `no_zk`
        feature).  This library's Wormhole leaf circuit IS the reference's
        (same constants||sigmas cap and circuit digest: tests/test_reference_layout.py),
        so the same bytes are embedded here (qp_wormhole/data/, copied by
        tests/golden/make_golden.py) and verify under the leaf verifier data."""
        if self._dummy is None:
            from .prover import CONFIGS, _config_of_common
            cfg = _config_of_common(self.leaf_circuit_data.common)
            if cfg not in CONFIGS:
                raise ValueError("no dummy proof for this leaf circuit: pass dummy_proof=")
            name = "dummy_proof_zk.bin" if cfg == "standard_recursion_zk_config" else "dummy_proof.bin"
            with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", name), "rb") as f:
                data = f.read()
            # the proof ends with num_public_inputs (u64) and the public inputs
            npis, = struct.unpack_from("<Q", data, len(data) - 8 * (LEAF_PI_LEN + 1))
            if npis != LEAF_PI_LEN:
                raise ValueError(f"dummy proof {name}: {npis} public inputs, expected {LEAF_PI_LEN}")
            self._dummy = ProofWithPublicInputs(data, struct.unpack_from(f"<{LEAF_PI_LEN}Q", data,
                                                                         len(data) - 8 * LEAF_PI_LEN))
        return self._dummy

    def extract_leaf_public_inputs(self, aggr) -> List[PublicCircuitInputs]:
        proof = aggr.proof if isinstance(aggr, AggregatedProof) else aggr
        return public_inputs_from_aggregated(proof, LEAF_PI_LEN, self.config.num_leaf_proofs)

    def aggregate(self) -> AggregatedProof:
        if not self.proofs_buffer:
            raise ValueError("there are no proofs to aggregate")
        proofs, self.proofs_buffer = self.proofs_buffer, []
        padded = pad_with_dummy_proofs(proofs, self.config.num_leaf_proofs, self.dummy_proof())
        return aggregate_to_tree(padded, self.leaf_circuit_data.common, self.leaf_circuit_data.verifier_only,
                                 self.config, self.device)


def verifier_only_of(verifier_data: bytes, common: bytes) -> bytes:
    """VerifierOnlyCircuitData bytes from a verifier.bin-layout blob."""
    if not verifier_data.endswith(common):
        raise ValueError("verifier data does not end with the common data")
    vo = verifier_data[:len(verifier_data) - len(common)]
    (h,) = struct.unpack_from("<Q", vo, 0)
    if len(vo) != 8 + 32 * (1 << h) + 32:
        raise QpError(1, "malformed VerifierOnlyCircuitData")
    return vo
