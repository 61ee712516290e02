"""Multi-GPU plumbing: one process per GPU, proofs sharded by rank, leaf proofs
gathered to the aggregator rank.

Proofs are independent, so there is no collective on the data path; the only
exchange is the gather of serialized leaf proofs (fixed size per circuit) to
the rank that feeds the recursive aggregator
(wormhole/aggregator/src/aggregator.rs:74-92).  torch.distributed backend
"nccl" is RCCL over xGMI on MI355X; "gloo" is used for CPU tests.
"""
import numpy as np


def shard(total: int, rank: int, world: int) -> range:
    """Contiguous shard of proof indices [0, total) for `rank` (sizes differ by <= 1)."""
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def pack_proofs(proofs, slot: int) -> np.ndarray:
    """[n][8 + slot] uint8: little-endian length prefix + proof bytes (zero padded)."""
    if proofs and all(len(p) == slot for p in proofs):
        # fixed-size proofs (the prover's case): one join + one strided copy
        out = np.empty((len(proofs), 8 + slot), np.uint8)
        out[:, :8] = np.frombuffer(slot.to_bytes(8, "little"), np.uint8)
        out[:, 8:] = np.frombuffer(b"".join(proofs), np.uint8).reshape(len(proofs), slot)
        return out
    out = np.zeros((len(proofs), 8 + slot), np.uint8)
    for i, p in enumerate(proofs):
        if len(p) > slot:
            raise ValueError(f"proof of {len(p)} bytes exceeds slot {slot}")
        out[i, :8] = np.frombuffer(len(p).to_bytes(8, "little"), np.uint8)
        out[i, 8:8 + len(p)] = np.frombuffer(p, np.uint8)
    return out


def unpack_proofs(arr: np.ndarray):
    res = []
    for row in arr:
        n = int.from_bytes(row[:8].tobytes(), "little")
        res.append(row[8:8 + n].tobytes())
    return res


def gather_proofs(proofs, slot: int, dist, device="cpu", dst: int = 0, raw: bool = False):
    """Gather every rank's proofs to `dst` in rank order; returns the list on dst,
    None elsewhere.  Shards may differ in size (2048 over 3 ranks): counts are
    exchanged first and short shards padded with empty entries, which dst drops
    (a serialized proof is never empty).  raw=True returns, on dst, the
    gathered [rank] tensors of packed rows ([n][8 + slot] uint8, on `device`)
    and the per-rank counts instead of Python bytes objects (what a consumer
    reading the packed buffer needs; no per-proof host copies)."""
    import torch
    rank, world = dist.get_rank(), dist.get_world_size()
    # a bad shard is reported through the count exchange (-1), so every rank
    # raises the same error instead of its peers blocking in the gather
    bad = any(len(p) == 0 or len(p) > slot for p in proofs)
    cnt = torch.tensor([-1 if bad else len(proofs)], dtype=torch.int64, device=device)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt)
    bad_ranks = [r for r, c in enumerate(counts) if int(c.item()) < 0]
    if bad_ranks:
        raise ValueError(f"empty or oversized proof in the shard of rank(s) {bad_ranks}")
    most = int(max(int(c.item()) for c in counts))
    t = torch.from_numpy(pack_proofs(list(proofs) + [b""] * (most - len(proofs)), slot)).to(device)
    bufs = [torch.empty_like(t) for _ in range(world)] if rank == dst else None
    dist.gather(t, bufs, dst=dst)
    if rank != dst:
        return None
    if raw:
        return bufs, [int(c.item()) for c in counts]
    out = []
    for b in bufs:
        out.extend(p for p in unpack_proofs(b.cpu().numpy()) if p)
    return out


def run_steps(prove_share, nprovers, steps, dist=None, slot=0, device="cpu", pipelined=True, on_leaves=None):
    """bench.py's timed loop: `steps` steps of every prover's share of the batch,
    then each step's leaf proofs to rank 0 (the aggregator's input).

    prove_share(i) -> list of serialized proofs: prover i's share of one step
    (its own HIP stream and host thread).  pipelined: each prover thread runs
    its share of ALL steps back to back (no prover idles the GPU while the
    slowest finishes a step) and the K per-step gathers follow; otherwise the
    threads are joined after every step.  With dist (world > 1) every step's
    proofs are gathered in raw mode (gather_proofs); on_leaves(step, result)
    receives, on rank 0, the gathered (buffers, counts) -- or the step's local
    proofs when dist is None.  Returns the last step's local proofs."""
    import threading
    outs = [[None] * steps for _ in range(nprovers)]
    errors = []

    def run(i, ks):
        try:
            for s in ks:
                outs[i][s] = prove_share(i)
        except BaseException as e:  # surfaced on the calling thread
            errors.append(e)

    def launch(ks):
        if nprovers == 1:
            run(0, ks)
        else:
            th = [threading.Thread(target=run, args=(i, ks)) for i in range(nprovers)]
            for t in th:
                t.start()
            for t in th:
                t.join()
        if errors:
            raise RuntimeError("a prover thread failed") from errors[0]

    def finish(s):
        proofs = [p for i in range(nprovers) for p in outs[i][s]]
        res = proofs
        if dist is not None:
            res = gather_proofs(proofs, slot, dist, device=device, raw=True)
        if on_leaves is not None and (dist is None or dist.get_rank() == 0):
            on_leaves(s, res)
        return proofs

    last = None
    if pipelined and nprovers > 1:
        launch(range(steps))
        for s in range(steps):
            last = finish(s)
    else:
        for s in range(steps):
            launch([s])
            last = finish(s)
    return last


def log_exact(n: int, base: int):
    """k with base**k == n (k >= 0), else None."""
    if n < 1 or base < 2:
        return None
    k, p = 0, 1
    while p < n:
        p, k = p * base, k + 1
    return k if p == n else None


def check_subtree_shards(n_local: int, branching: int, dist, device="cpu"):
    """Cross-rank preconditions of per-rank subtree aggregation, checked on every
    rank through one all_gather of the local leaf counts BEFORE any aggregation
    or gather: all ranks hold the same number of leaves, a power (>= 1) of the
    branching factor, and the world size is a power of it.  Every rank raises
    the same error otherwise (no rank is left waiting in a collective, and no
    rank aggregates roots of subtrees of different depths)."""
    import torch
    world = dist.get_world_size()
    valid = log_exact(n_local, branching) not in (None, 0)
    cnt = torch.tensor([n_local if valid else -1], dtype=torch.int64, device=device)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt)
    counts = [int(c.item()) for c in counts]
    bad = [r for r, c in enumerate(counts) if c < 0]
    if bad:
        raise ValueError(f"rank(s) {bad} hold a leaf count that is not a power (>= 1) of the branching factor "
                         f"{branching} (counts {counts})")
    if len(set(counts)) != 1:
        raise ValueError(f"ranks hold different leaf counts {counts}: subtree roots would come from circuits of "
                         f"different depths")
    if log_exact(world, branching) is None:
        raise ValueError(f"world size {world} is not a power of the branching factor {branching}")


def aggregate_subtrees(local_proofs, common: bytes, verifier_only: bytes, branching: int, dist,
                       device="cpu", gpu: int = 0, dst: int = 0, backend=None, timings=None):
    """Per-rank subtree aggregation (the levels of tree.rs:92-103
    are independent per chunk): each rank aggregates its own leaf proofs into one
    subtree root (aggregate_to_tree with depth log_branching(local count)); only
    the roots cross the interconnect (one gather of world proofs instead of every
    leaf); rank dst aggregates the roots into the tree root.  Every rank must hold
    branching**k leaves (equal k) and world must be a power of branching
    (check_subtree_shards, before any work).  dist=None: one rank.
    Returns the root AggregatedProof on dst (or, when the tree's top level
    needs a circuit beyond the GPU prover, the list of the highest level's
    proofs, with timings["top_stopped"] saying why), None elsewhere; timings
    (a dict) receives the seconds of the stages: subtree_s, gather_s, top_s."""
    import time
    from .aggregator import TreeAggregationConfig, aggregate_to_tree
    if dist is not None:
        check_subtree_shards(len(local_proofs), branching, dist, device)
    elif log_exact(len(local_proofs), branching) in (None, 0):
        raise ValueError(f"{len(local_proofs)} local proofs are not a power (>= 1) of the branching factor "
                         f"{branching}")
    depth = log_exact(len(local_proofs), branching)
    tm = timings if timings is not None else {}
    t0 = time.perf_counter()
    sub = aggregate_to_tree(local_proofs, common, verifier_only, TreeAggregationConfig.new(branching, depth),
                            gpu, backend)
    tm["subtree_s"] = time.perf_counter() - t0
    return _roots_to_top(sub, branching, dist, device, gpu, dst, backend, tm)


def _roots_to_top(sub, branching: int, dist, device, gpu: int, dst: int, backend, tm):
    """Each rank's subtree root -> rank dst (one gather of world proofs), which
    aggregates them into the tree root (aggregate_subtrees' last two stages)."""
    import time
    from .aggregator import TreeAggregationConfig, aggregate_to_tree
    from .prover import ProofWithPublicInputs
    world, rank = (dist.get_world_size(), dist.get_rank()) if dist is not None else (1, 0)
    t1 = time.perf_counter()
    if dist is not None:
        roots = gather_proofs([sub.proof.to_bytes()], len(sub.proof.to_bytes()), dist, device=device, dst=dst)
    else:
        roots = [sub.proof.to_bytes()]
    t2 = time.perf_counter()
    tm["gather_s"] = t2 - t1
    tm["top_s"] = 0.0
    if rank != dst:
        return None
    if world == 1:
        return sub
    cd = sub.circuit_data
    from .aggregator import CircuitTooLarge
    try:
        root = aggregate_to_tree([ProofWithPublicInputs(r, []) for r in roots], cd.common, cd.verifier_only,
                                 TreeAggregationConfig.new(branching, log_exact(world, branching)), gpu, backend)
    except CircuitTooLarge as e:
        # the top of a deep tree (e.g. 2048 leaves: the root registers 32,768
        # public inputs, 2^15 rows) is beyond the GPU prover: the proofs of the
        # highest level it could prove are returned instead of the root
        root = e.proofs
        tm["top_stopped"] = str(e)
    tm["top_s"] = time.perf_counter() - t2
    return root


def pipeline_aggregate_step_streamed(prove_part, parts: int, part_leaves: int, common: bytes,
                                     verifier_only: bytes, branching: int, dist=None, device="cpu", gpu: int = 0,
                                     dst: int = 0, backend=None):
    """pipeline_aggregate_step with the rank's leaves proved in `parts`
    consecutive parts (prove_part(i) -> the part's part_leaves serialized
    proofs, called in order on a producer thread) and each part's sub-tree
    aggregated as soon as its leaves exist (aggregator.aggregate_to_tree_streamed),
    while the next part's leaves are proved: the sub-trees' latency-bound upper
    levels overlap the later parts' leaf kernels.  The same leaves and chunks as
    pipeline_aggregate_step, so the same root.  Returns (root on dst / None,
    stage seconds: leaves_s = when the last part's leaves were done, subtree_s
    = the local root, gather_s, top_s)."""
    import threading
    import time
    from .aggregator import TreeAggregationConfig, aggregate_to_tree_streamed
    n_local = parts * part_leaves
    if dist is not None:
        check_subtree_shards(n_local, branching, dist, device)
    elif log_exact(n_local, branching) in (None, 0) or log_exact(parts, branching) is None:
        raise ValueError(f"{parts} parts of {part_leaves} leaves do not form a {branching}-ary tree")
    ready = [threading.Event() for _ in range(parts)]
    got = [None] * parts
    errors = []
    tm = {}
    t0 = time.perf_counter()

    def producer():
        try:
            for i in range(parts):
                got[i] = prove_part(i)
                if len(got[i]) != part_leaves:
                    raise ValueError(f"part {i}: {len(got[i])} leaf proofs, expected {part_leaves}")
                ready[i].set()
            tm["leaves_s"] = time.perf_counter() - t0
        except BaseException as e:  # re-raised on the calling thread
            errors.append(e)
            for ev in ready:
                ev.set()

    def leaves_of(i):
        ready[i].wait()
        if errors:
            raise RuntimeError("the leaf producer failed") from errors[0]
        return got[i]

    th = threading.Thread(target=producer, daemon=True)
    th.start()
    try:
        sub = aggregate_to_tree_streamed(leaves_of, parts, common, verifier_only,
                                         TreeAggregationConfig.new(branching, log_exact(n_local, branching)), gpu,
                                         backend)
    finally:
        th.join()
    if errors:
        raise errors[0]
    tm["subtree_s"] = time.perf_counter() - t0
    return _roots_to_top(sub, branching, dist, device, gpu, dst, backend, tm), tm


def pipeline_aggregate_step(prove_leaves, common: bytes, verifier_only: bytes, branching: int, dist=None,
                            device="cpu", gpu: int = 0, dst: int = 0, backend=None):
    """BASELINE configs[3] as one step ("Batch 2048 proofs sharded 8xMI355X,
    RCCL-gather leaves into recursive aggregator"; wormhole/aggregator/src/
    aggregator.rs:74-92, circuits/tree.rs:55-103): every rank proves its batch
    of leaves (prove_leaves() -> serialized proofs), aggregates them into its
    subtree root on its own GPU, the roots are gathered to dst over RCCL, and dst
    aggregates them into the tree root.  Returns (root on dst / None, stage
    seconds {leaves_s, subtree_s, gather_s, top_s})."""
    import time
    t0 = time.perf_counter()
    leaves = prove_leaves()
    tm = {"leaves_s": time.perf_counter() - t0}
    root = aggregate_subtrees(leaves, common, verifier_only, branching, dist, device=device, gpu=gpu, dst=dst,
                              backend=backend, timings=tm)
    return root, tm


def pipeline_aggregate_steps(prove_leaves, steps: int, common: bytes, verifier_only: bytes, branching: int,
                             dist=None, device="cpu", gpu: int = 0, dst: int = 0, backend=None):
    """configs[3] as a stream of batches: `steps` pipeline_aggregate_step's with
    batch k+1's leaves proved (a leaf thread: prove_leaves() on the leaf
    provers' own streams) while batch k is aggregated into its root (this
    thread: the level provers' streams, the roots gather, rank dst's top
    levels).  The subtree's narrow top levels are latency-bound (one proof's
    sequential Poseidon chains), so the leaf proofs of the next batch fill the
    GPU they leave idle.  At most one finished batch waits in between.  Only
    this thread issues collectives, in the same order on every rank; each step
    starts with an all-reduce of a per-rank ok flag, so a leaf failure on one
    rank stops every rank at that step (each raises).  Returns
    ([root per step on dst / None], [stage seconds per step])."""
    import queue
    import threading
    import time
    q = queue.Queue(maxsize=1)
    errors = []
    stop = threading.Event()

    def leaf_worker():
        try:
            for _ in range(steps):
                if stop.is_set():
                    return
                t = time.perf_counter()
                leaves = prove_leaves()
                q.put((leaves, time.perf_counter() - t))
        except BaseException as e:  # re-raised on the calling thread
            errors.append(e)
            q.put(None)

    th = threading.Thread(target=leaf_worker, daemon=True)
    th.start()
    roots, tms = [], []
    def all_ok(ok):
        # every rank stops at the same step when one rank's leaf step failed
        # (its peers would otherwise wait in this step's collectives forever)
        if dist is None:
            return ok
        import torch
        t = torch.tensor([1 if ok else 0], dtype=torch.int64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    try:
        for _ in range(steps):
            item = q.get()
            if not all_ok(item is not None):
                if item is not None:
                    errors.append(RuntimeError("another rank's leaf step failed"))
                break
            leaves, lt = item
            tm = {"leaves_s": lt}
            roots.append(aggregate_subtrees(leaves, common, verifier_only, branching, dist, device=device, gpu=gpu,
                                            dst=dst, backend=backend, timings=tm))
            tms.append(tm)
    finally:
        stop.set()
        while th.is_alive():
            try:
                q.get(timeout=0.1)
            except queue.Empty:
                pass
        th.join()
    if errors:
        raise errors[0]
    return roots, tms
