"""The opt-in k_quotient_fused (csrc/prover_kernels.hip) copies each routed
wire into an LDS slot as the Poseidon gate reads it and sweeps chunks of 8
routed wires at fixed read points.  This restates the gate's read order
(poseidon_gate_rd) and the kernel's slot and sweep rules, and checks that no
two pending wires share a slot and that every chunk is complete when it is
swept.  (GPU parity of the kernel: tests/test_gpu_prover.py.)"""

R = 80  # routed wires; chunks of 8


def gate_read_order():
    order = [24]
    for i in range(4):
        order += [25 + i, i, i + 4]
    order += list(range(8, 12))
    for r in range(1, 4):
        order += [29 + (r - 1) * 12 + i for i in range(12)]
    order += [65 + t for t in range(22)]
    for r in range(4):
        order += [87 + r * 12 + i for i in range(12)]
    order += [12 + i for i in range(12)]
    return order


def qf_slot(j):
    return 16 + (j - 8) if (j >> 3) == 1 and j < 12 else ((j >> 3) & 1) * 8 + (j & 7)


SWEEPS = {7: [0], 39: [3, 4], 47: [5], 63: [6, 7], 87: [8, 9], 23: [1, 2]}


def test_read_order_covers_every_wire_once():
    order = gate_read_order()
    assert sorted(order) == list(range(135))


def test_pending_wires_never_share_a_slot_and_chunks_are_complete():
    slots = {}       # slot -> wire currently held
    read = set()
    swept = set()
    for j in gate_read_order():
        read.add(j)
        if j < R:
            s = qf_slot(j)
            assert 0 <= s < 20
            assert s not in slots, f"wire {j} overwrites pending wire {slots.get(s)} in slot {s}"
            slots[s] = j
        for k in SWEEPS.get(j, []):
            wires = range(8 * k, 8 * k + 8)
            assert all(w in read for w in wires), f"chunk {k} swept at wire {j} before all its wires were read"
            for w in wires:
                assert slots.pop(qf_slot(w)) == w
            swept.add(k)
    assert swept == set(range(10)) and not slots
