"""Multi-process path on CPU (gloo, world size 2): shard assignment and the
leaf-proof gather that bench.py and the aggregator hand-off use over RCCL."""
import os
import socket

import pytest

from qp_wormhole.distributed import pack_proofs, shard, unpack_proofs


@pytest.mark.parametrize("total", [0, 1, 7, 256, 2048])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shards_partition_the_batch(total, world):
    seen = []
    for r in range(world):
        s = shard(total, r, world)
        seen.extend(s)
        assert len(s) in (total // world, total // world + 1)
    assert seen == list(range(total))


def test_pack_roundtrip():
    proofs = [bytes([i]) * (100 + i) for i in range(5)]
    assert unpack_proofs(pack_proofs(proofs, 200)) == proofs
    with pytest.raises(ValueError):
        pack_proofs([b"x" * 300], 200)


def test_pack_fixed_size_fast_path():
    """Fixed-size proofs (the prover's case) take the one-copy path; same rows."""
    proofs = [bytes([i]) * 64 for i in range(7)]
    fast = pack_proofs(proofs, 64)
    slow = pack_proofs(proofs + [b"z"], 64)[:7]
    assert (fast == slow).all()
    assert unpack_proofs(fast) == proofs


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from qp_wormhole.distributed import gather_proofs
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = [bytes([rank * 16 + i]) * (1000 + rank) for i in shard(8, rank, world)]
    got = gather_proofs(mine, 2048, dist)
    if rank == 0:
        q.put(got)
    dist.barrier()
    dist.destroy_process_group()


def _run(target, world, *args):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=180)
        assert p.exitcode == 0
    return got


def test_gather_world2_gloo():
    got = _run(_worker, 2)
    expect = [bytes([r * 16 + i]) * (1000 + r) for r in range(2) for i in shard(8, r, 2)]
    assert got == expect


def _worker_raw(rank, world, port, q):
    import torch.distributed as dist
    from qp_wormhole.distributed import gather_proofs
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = [bytes([rank * 16 + i]) * 512 for i in shard(7, rank, world)]  # uneven shards, fixed size
    got = gather_proofs(mine, 512, dist, raw=True)
    if rank == 0:
        bufs, counts = got
        q.put((counts, [unpack_proofs(b.numpy()) for b in bufs]))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_raw_world3_gloo():
    """raw=True (the bench's mode): the dst rank gets the packed per-rank
    buffers and counts; rows past a rank's count are padding."""
    counts, rows = _run(_worker_raw, 3)
    assert counts == [len(shard(7, r, 3)) for r in range(3)]
    for r in range(3):
        want = [bytes([r * 16 + i]) * 512 for i in shard(7, r, 3)]
        assert [p for p in rows[r] if p] == want


def _worker_real(rank, world, port, q, total):
    """Each rank ships its shard of the reference's own current-circuit proofs
    (tests/golden/dummy_proof{,_zk}.bin, 132,712 B each, alternating); rank 0
    verifies every gathered proof under the reconstructed verifier data."""
    import torch.distributed as dist

    from qp_wormhole.distributed import gather_proofs
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle_lib import golden
    fixtures = [golden("dummy_proof.bin"), golden("dummy_proof_zk.bin")]
    mine = [fixtures[i % 2] for i in shard(total, rank, world)]
    got = gather_proofs(mine, 140000, dist)
    if rank == 0:
        from current_circuit_vd import current_circuit_verifier_data
        from oracle_lib import lib as olib
        from test_oracle_golden import current_common_bytes
        vd = current_circuit_verifier_data(current_common_bytes())[0]
        ok = [olib().ora_verify(vd, len(vd), p, len(p)) == 0 for p in got]
        q.put((len(got), [p == fixtures[i % 2] for i, p in enumerate(got)], ok))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 2), (3, 4)])
def test_gather_real_proofs_verify(world, total):
    """Uneven shards (4 over 3 ranks) gather in order and every proof verifies on rank 0."""
    n, same, ok = _run(_worker_real, world, total)
    assert n == total and all(same) and all(ok)


def _worker_steps(rank, world, port, q, pipelined):
    """bench.py's timed loop (distributed.run_steps) with a stub prover: 3 prover
    threads per rank, 3 steps; every step's leaf proofs reach rank 0 through
    the raw gather, in rank/prover order."""
    import torch.distributed as dist

    from qp_wormhole.distributed import run_steps, unpack_proofs
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = {}

    def prove_share(i):
        k = calls.get(i, 0)
        calls[i] = k + 1
        return [bytes([rank, i, k, j]) * 64 for j in range(2 + i)]
    got = []

    def on_leaves(s, res):
        bufs, counts = res
        got.append((s, counts, [unpack_proofs(b.numpy()) for b in bufs]))
    last = run_steps(prove_share, 3, 3, dist=dist, slot=256, pipelined=pipelined, on_leaves=on_leaves)
    if rank == 0:
        q.put((got, len(last)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("pipelined", [True, False])
def test_bench_step_loop_world2_gloo(pipelined):
    got, nlast = _run(_worker_steps, 2, pipelined)
    assert nlast == 2 + 3 + 4
    assert [s for s, _, _ in got] == [0, 1, 2]
    for s, counts, rows in got:
        assert counts == [9, 9]
        for r in range(2):
            want = [bytes([r, i, s, j]) * 64 for i in range(3) for j in range(2 + i)]
            assert rows[r] == want


def _worker_subtrees(rank, world, port, q):
    """Per-rank subtree aggregation: every rank aggregates its own
    leaves (the reference's two proofs) into a subtree root; only the roots are
    gathered; rank 0 aggregates them.  The prover is the oracle CPU stand-in."""
    import struct

    import torch.distributed as dist

    from agg_oracle_backend import oracle_backend
    from qp_wormhole.distributed import aggregate_subtrees
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from current_circuit_vd import current_circuit_verifier_data
    from oracle_lib import golden, lib as olib
    from test_oracle_golden import current_common_bytes
    cb = current_common_bytes()
    vd = current_circuit_verifier_data(cb)[0]
    leaves = [golden("dummy_proof.bin"), golden("dummy_proof_zk.bin")]
    if rank == 1:
        leaves = leaves[::-1]
    root = aggregate_subtrees(leaves, cb, vd[:len(vd) - len(cb)], 2, dist, backend=oracle_backend)
    if rank == 0:
        rvd = root.circuit_data.verifier_data()
        ok = olib().ora_verify(rvd, len(rvd), root.proof.to_bytes(), len(root.proof.to_bytes())) == 0
        want = []
        for r in range(world):
            ls = [golden("dummy_proof.bin"), golden("dummy_proof_zk.bin")]
            for pf in (ls if r == 0 else ls[::-1]):
                want += list(struct.unpack_from("<16Q", pf, len(pf) - 128))
        q.put((ok, [int(x) for x in root.proof.public_inputs] == want))
    dist.barrier()
    dist.destroy_process_group()


def test_subtree_aggregation_world2_gloo():
    ok, pis_ok = _run(_worker_subtrees, 2)
    assert ok and pis_ok


def _worker_uneven(rank, world, port, q, counts):
    """aggregate_subtrees with invalid or unequal shards: every rank raises the
    same error from the count exchange, before any aggregation (no rank is left
    in a collective; no backend call happens)."""
    import torch.distributed as dist

    from qp_wormhole.distributed import aggregate_subtrees
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []

    def backend(*a):
        calls.append(a)
        raise AssertionError("aggregation must not start")
    try:
        aggregate_subtrees([b"x"] * counts[rank], b"", b"", 2, dist, backend=backend)
        msg = None
    except ValueError as e:
        msg = str(e)
    dist.barrier()
    q.put((rank, msg, len(calls)))
    dist.destroy_process_group()


def _run_all(target, world, *args):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=180)
        assert p.exitcode == 0
    return got


@pytest.mark.parametrize("world,counts,frag", [(2, (4, 2), "different leaf counts"),
                                               (2, (3, 4), "rank(s) [0]"),
                                               (3, (2, 2, 2), "world size 3")])
def test_subtree_shards_checked_on_every_rank(world, counts, frag):
    got = _run_all(_worker_uneven, world, counts)
    msgs = {m for _, m, _ in got}
    assert len(msgs) == 1 and frag in msgs.pop()
    assert all(c == 0 for _, _, c in got)


def _worker_pipeline(rank, world, port, q):
    """BASELINE configs[3] as bench.py times it (distributed.pipeline_aggregate_step):
    each rank proves its leaves (stub: the reference's two proofs), aggregates
    its subtree, the roots are gathered, rank 0 aggregates them.  Oracle CPU
    prover as the backend."""
    import struct

    import torch.distributed as dist

    from agg_oracle_backend import oracle_backend
    from qp_wormhole.distributed import pipeline_aggregate_step
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from current_circuit_vd import current_circuit_verifier_data
    from oracle_lib import golden, lib as olib
    from test_oracle_golden import current_common_bytes
    cb = current_common_bytes()
    vd = current_circuit_verifier_data(cb)[0]
    fx = [golden("dummy_proof.bin"), golden("dummy_proof_zk.bin")]

    def prove_leaves():
        return fx if rank == 0 else fx[::-1]
    root, tm = pipeline_aggregate_step(prove_leaves, cb, vd[:len(vd) - len(cb)], 2, dist, backend=oracle_backend)
    if rank == 0:
        rvd = root.circuit_data.verifier_data()
        ok = olib().ora_verify(rvd, len(rvd), root.proof.to_bytes(), len(root.proof.to_bytes())) == 0
        want = []
        for r in range(world):
            for pf in (fx if r == 0 else fx[::-1]):
                want += list(struct.unpack_from("<16Q", pf, len(pf) - 128))
        q.put((ok, [int(x) for x in root.proof.public_inputs] == want, sorted(tm)))
    else:
        assert root is None
    dist.barrier()
    dist.destroy_process_group()


def test_configs3_pipeline_step_world2_gloo():
    ok, pis_ok, stages = _run(_worker_pipeline, 2)
    assert ok and pis_ok
    assert stages == ["gather_s", "leaves_s", "subtree_s", "top_s"]


def _worker_pipeline_steps(rank, world, port, q):
    """configs[3] as a stream of batches (distributed.pipeline_aggregate_steps):
    three batches, each rank's next leaves proved on a leaf thread while the
    previous batch is aggregated; every batch's root verifies and carries its
    own leaves' public inputs (the batches differ), in order."""
    import struct

    import torch.distributed as dist

    from agg_oracle_backend import oracle_backend
    from qp_wormhole.distributed import pipeline_aggregate_steps
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from current_circuit_vd import current_circuit_verifier_data
    from oracle_lib import golden, lib as olib
    from test_oracle_golden import current_common_bytes
    cb = current_common_bytes()
    vd = current_circuit_verifier_data(cb)[0]
    fx = [golden("dummy_proof.bin"), golden("dummy_proof_zk.bin")]
    order = [[0, 1], [1, 0], [1, 1]]
    calls = []

    def prove_leaves():
        k = len(calls)
        calls.append(k)
        o = order[(k + rank) % 3]
        return [fx[i] for i in o]
    roots, tms = pipeline_aggregate_steps(prove_leaves, 3, cb, vd[:len(vd) - len(cb)], 2, dist,
                                          backend=oracle_backend)
    if rank == 0:
        res = []
        for k, root in enumerate(roots):
            rvd = root.circuit_data.verifier_data()
            ok = olib().ora_verify(rvd, len(rvd), root.proof.to_bytes(), len(root.proof.to_bytes())) == 0
            want = []
            for r in range(world):
                for i in order[(k + r) % 3]:
                    pf = fx[i]
                    want += list(struct.unpack_from("<16Q", pf, len(pf) - 128))
            res.append(ok and [int(x) for x in root.proof.public_inputs] == want)
        q.put((res, len(calls), [sorted(t) for t in tms]))
    else:
        assert roots == [None] * 3 and len(calls) == 3
    dist.barrier()
    dist.destroy_process_group()


def test_configs3_pipelined_steps_world2_gloo():
    res, ncalls, stages = _run(_worker_pipeline_steps, 2)
    assert res == [True] * 3 and ncalls == 3
    assert stages == [["gather_s", "leaves_s", "subtree_s", "top_s"]] * 3


def _worker_pipeline_steps_fail(rank, world, port, q):
    """A leaf failure on rank 1 at batch 2 of 3: every rank stops at that
    step's ok-flag all-reduce and raises (none waits in the roots gather)."""
    import torch.distributed as dist

    from agg_oracle_backend import oracle_backend
    from qp_wormhole.distributed import pipeline_aggregate_steps
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from current_circuit_vd import current_circuit_verifier_data
    from oracle_lib import golden
    from test_oracle_golden import current_common_bytes
    cb = current_common_bytes()
    vd = current_circuit_verifier_data(cb)[0]
    fx = [golden("dummy_proof.bin"), golden("dummy_proof_zk.bin")]
    calls = []

    def prove_leaves():
        calls.append(1)
        if rank == 1 and len(calls) == 2:
            raise ValueError("leaf failure on rank 1")
        return fx
    try:
        pipeline_aggregate_steps(prove_leaves, 3, cb, vd[:len(vd) - len(cb)], 2, dist, backend=oracle_backend)
        err = None
    except Exception as e:  # noqa: BLE001
        err = str(e)
    q.put((rank, err))
    dist.barrier()
    dist.destroy_process_group()


def test_configs3_pipelined_leaf_failure_stops_every_rank():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_pipeline_steps_fail, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=180)
        assert p.exitcode == 0
    assert got[1] == "leaf failure on rank 1"
    assert got[0] == "another rank's leaf step failed"


def test_configs3_streamed_step_equals_the_batch_step():
    """pipeline_aggregate_step_streamed (leaves proved part by part on a
    producer thread, each part's sub-tree aggregated as soon as its leaves
    exist) gives the same root as pipeline_aggregate_step over the same leaves:
    the same chunks in the same order (oracle backend, one rank)."""
    from agg_oracle_backend import oracle_backend
    from current_circuit_vd import current_circuit_verifier_data
    from oracle_lib import golden, lib as olib
    from qp_wormhole.distributed import pipeline_aggregate_step, pipeline_aggregate_step_streamed
    from test_oracle_golden import current_common_bytes
    cb = current_common_bytes()
    vd = current_circuit_verifier_data(cb)[0]
    vo = vd[:len(vd) - len(cb)]
    fx = [golden("dummy_proof.bin"), golden("dummy_proof_zk.bin")]
    leaves = [fx[0], fx[1], fx[1], fx[0]]
    calls = []

    def prove_part(i):
        calls.append(i)
        return leaves[2 * i:2 * i + 2]
    root_s, tm = pipeline_aggregate_step_streamed(prove_part, 2, 2, cb, vo, 2, backend=oracle_backend)
    root_b, _ = pipeline_aggregate_step(lambda: leaves, cb, vo, 2, backend=oracle_backend)
    assert calls == [0, 1]
    assert root_s.proof.to_bytes() == root_b.proof.to_bytes()
    rvd = root_s.circuit_data.verifier_data()
    assert olib().ora_verify(rvd, len(rvd), root_s.proof.to_bytes(), len(root_s.proof.to_bytes())) == 0
    assert sorted(tm) == ["gather_s", "leaves_s", "subtree_s", "top_s"]
    with pytest.raises(ValueError):
        pipeline_aggregate_step_streamed(prove_part, 3, 2, cb, vo, 2, backend=oracle_backend)
