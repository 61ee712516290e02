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
    if any(len(p) == 0 for p in proofs):
        raise ValueError("empty proof")
    cnt = torch.tensor([len(proofs)], dtype=torch.int64, device=device)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt)
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
