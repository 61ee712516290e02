"""Python model of plonky2's CircuitBuilder row layout for the Wormhole circuit
(development tool for matching the reference's preprocessing; the product
builder is csrc/circuit.cpp).  Tracks gate kinds, gate constants, virtual
targets, copy constraints and constants, with knobs for the plonky2 behaviours
that decide row order.
"""
NOOP, CONST, PI, BSUM, ARITH, POS = range(6)
P = 0xFFFFFFFF00000001
NEG1 = P - 1


class B:
    def __init__(self, num_ops=20, limbs=63, dedup=True, special=True, num_consts=2):
        self.rows = []          # (kind, [consts])
        self.nv = 0
        self.copies = []
        self.c2t = {}
        self.t2c = {}
        self.slots = {}
        self.cache = {}
        self.pis = []
        self.num_ops, self.limbs, self.dedup, self.special, self.nc = num_ops, limbs, dedup, special, num_consts
        self.const_gens = []    # (row, const_idx, wire)

    # targets: ('v', i) or ('w', row, col)
    def virt(self):
        self.nv += 1
        return ('v', self.nv - 1)

    def virts(self, n):
        return [self.virt() for _ in range(n)]

    def add_gate(self, kind, consts=()):
        r = len(self.rows)
        c = list(consts)
        if kind == CONST:
            c = c + [0] * (self.nc - len(c))
            for i in range(self.nc):
                self.const_gens.append((r, i, i))
        elif kind == ARITH:
            c = c + [0] * (2 - len(c))
        self.rows.append((kind, c))
        return r

    def constant(self, c):
        c %= P
        if c in self.c2t:
            return self.c2t[c]
        t = self.virt()
        self.c2t[c] = t
        self.t2c[t] = c
        return t

    def zero(self):
        return self.constant(0)

    def one(self):
        return self.constant(1)

    def connect(self, a, b):
        self.copies.append((a, b))

    def arithmetic(self, c0, c1, m0, m1, a):
        c0 %= P
        c1 %= P
        if self.special:
            z = self.zero()
            k0, k1, ka = self.t2c.get(m0), self.t2c.get(m1), self.t2c.get(a)
            fz = c0 == 0 or m0 == z or m1 == z
            sz = c1 == 0 or a == z
            fc = 0 if fz else (k0 * k1 * c0 % P if (k0 is not None and k1 is not None) else None)
            sc = 0 if sz else (ka * c1 % P if ka is not None else None)
            if fc is not None and sc is not None:
                return self.constant(fc + sc)
            if fz and c1 == 1:
                return a
            if sz:
                if k0 is not None and k0 * c0 % P == 1:
                    return m1
                if k1 is not None and k1 * c0 % P == 1:
                    return m0
        key = (c0, c1, m0, m1, a)
        if self.dedup and key in self.cache:
            return self.cache[key]
        s = self.slots.get((c0, c1))
        if s is None:
            row, op = self.add_gate(ARITH, [c0, c1]), 0
        else:
            row, op = s
        if op == self.num_ops - 1:
            self.slots.pop((c0, c1), None)
        else:
            self.slots[(c0, c1)] = (row, op + 1)
        self.connect(m0, ('w', row, 4 * op))
        self.connect(m1, ('w', row, 4 * op + 1))
        self.connect(a, ('w', row, 4 * op + 2))
        out = ('w', row, 4 * op + 3)
        self.cache[key] = out
        return out

    def add(self, x, y):
        return self.arithmetic(1, 1, x, self.one(), y)

    def sub(self, x, y):
        return self.arithmetic(1, NEG1, x, self.one(), y)

    def mul(self, x, y):
        return self.arithmetic(1, 0, x, y, x)

    def mul_add(self, x, y, z):
        return self.arithmetic(1, 1, x, y, z)

    def mul_sub(self, x, y, z):
        return self.arithmetic(1, NEG1, x, y, z)

    def mul_const(self, c, x):
        return self.mul(self.constant(c), x)

    def mul_const_add(self, c, x, y):
        return self.mul_add(self.constant(c), x, y)

    def not_(self, b):
        return self.sub(self.one(), b)

    def and_(self, a, b):
        return self.mul(a, b)

    def or_(self, a, b):
        t = self.arithmetic(NEG1, 1, a, b, a)
        return self.add(t, b)

    def select(self, b, x, y):
        tmp = self.mul_sub(b, y, y)
        return self.mul_sub(b, x, tmp)

    def is_equal(self, x, y):
        z = self.zero()
        eq = self.virt()
        ne = self.not_(eq)
        inv = self.virt()
        d = self.sub(x, y)
        c1 = self.mul(eq, d)
        c2 = self.mul(d, inv)
        self.connect(c1, z)
        self.connect(c2, ne)
        return eq

    def split_le(self, x, nbits):
        k = -(-nbits // self.limbs)
        gates = [self.add_gate(BSUM) for _ in range(k)]
        bits = [('w', g, 1 + l) for g in gates for l in range(self.limbs)]
        for b in bits[nbits:]:
            self.connect(b, self.zero())
        bits = bits[:nbits]
        acc = self.zero()
        for g in reversed(gates):
            acc = self.mul_const_add(pow(2, self.limbs, P), acc, ('w', g, 0))
        self.connect(acc, x)
        return bits

    def range_check(self, x, n):
        self.split_le(x, n)

    def permute(self, state):
        r = self.add_gate(POS)
        self.connect(self.zero(), ('w', r, 24))
        for i in range(12):
            self.connect(state[i], ('w', r, i))
        return [('w', r, 12 + i) for i in range(12)]

    def hash_no_pad(self, inputs):
        z = self.zero()
        st = [z] * 12
        for o in range(0, len(inputs), 8):
            ch = inputs[o:o + 8]
            st[:len(ch)] = ch
            st = self.permute(st)
        return st[:4]

    def build_tail(self, sort_consts=True):
        pih = self.hash_no_pad(self.pis)
        pr = self.add_gate(PI)
        for i in range(4):
            self.connect(pih[i], ('w', pr, i))
        while len(self.c2t) > len(self.const_gens):
            self.add_gate(CONST)
        items = sorted(self.c2t.items()) if sort_consts else sorted(self.c2t.items(), key=lambda kv: kv[1][1])
        for (c, t), (row, ci, wi) in zip(items, self.const_gens):
            self.rows[row][1][ci] = c
            self.connect(('w', row, wi), t)
        return pr


def is_const_less_than(b, left, right, n_log):
    bits = b.split_le(right, n_log)
    lt = b.zero()
    eq = b.one()
    for i in reversed(range(n_log)):
        a = b.constant((left >> i) & 1)
        bb = bits[i]
        na = b.not_(a)
        nab = b.and_(na, bb)
        tl = b.and_(nab, eq)
        lt = b.or_(lt, tl)
        ab = b.mul(a, bb)
        two_ab = b.mul_const(2, ab)
        apb = b.add(a, bb)
        x = b.sub(apb, two_ab)
        nx = b.not_(x)
        eq = b.and_(eq, nx)
    return lt


def felt(s):
    bs = s.encode()
    return [int.from_bytes(bs[0:4], 'little'), int.from_bytes(bs[4:8], 'little')]


def wormhole(b, max_len=20, node=188):
    # CircuitTargets::new
    nul_hash = b.virts(4)
    b.pis += nul_hash
    nul_secret = b.virts(8)
    nul_tc = b.virts(2)
    un_acc = b.virts(4)
    un_secret = b.virts(8)
    proof_data = [b.virts(node) for _ in range(max_len)]
    indices = b.virts(max_len)
    root = b.virts(4)
    b.pis += root
    proof_len = b.virt()
    tc = b.virts(2)
    fa = b.virts(4)
    ta = b.virts(4)
    amt = b.virts(4)
    b.pis += amt
    exit_ = b.virts(4)
    b.pis += exit_
    # Nullifier
    s = felt("~nullif~")
    pre = [b.constant(s[0]), b.constant(s[1])] + nul_secret + nul_tc
    for t in pre:
        b.range_check(t, 32)
    inner = b.hash_no_pad(pre)
    comp = b.hash_no_pad(inner)
    for x, y in zip(comp, nul_hash):
        b.connect(x, y)
    # Unspendable
    s = felt("wormhole")
    pre = [b.constant(s[0]), b.constant(s[1])]
    for t in pre:
        b.range_check(t, 32)
    pre += un_secret
    inner = b.hash_no_pad(pre)
    gen = b.hash_no_pad(inner)
    for x, y in zip(gen, un_acc):
        b.connect(x, y)
    # Storage proof
    for t in tc + amt:
        b.range_check(t, 32)
    leaf_hash = b.hash_no_pad(tc + fa + ta + amt)
    two32 = b.constant(1 << 32)
    prev = root
    n_log = (max_len - 1).bit_length()
    for i in range(max_len):
        nd = proof_data[i]
        ipn = is_const_less_than(b, i, proof_len, n_log)
        it = b.constant(i)
        iln = b.is_equal(it, proof_len)
        ch = b.hash_no_pad(nd)
        for y in range(4):
            d = b.sub(ch[y], prev[y])
            r = b.mul(d, ipn)
            b.connect(r, b.zero())
        found = [b.zero()] * 4
        exp = indices[i]
        for j in range(node - 8):
            b.range_check(nd[j], 32)
            fi = b.constant(j)
            st = b.is_equal(fi, exp)

            def comb(lo, hi):
                hs = b.mul(hi, two32)
                return b.add(lo, hs)
            hh = [comb(nd[j + 2 * k], nd[j + 2 * k + 1]) for k in range(4)]
            for k in range(4):
                found[k] = b.select(st, hh[k], found[k])
        for j in range(node - 8, node):
            b.range_check(nd[j], 32)
        for y in range(1, 4):
            d = b.sub(leaf_hash[y], prev[y])
            r = b.mul(d, iln)
            b.connect(r, b.zero())
        prev = found
    # connect_shared_targets
    for x, y in zip(nul_secret, un_secret):
        b.connect(x, y)
    for x, y in zip(nul_tc, tc):
        b.connect(x, y)
    for x, y in zip(un_acc, ta):
        b.connect(x, y)
