"""The register-group layout algebra of k_rows (kernels.hip Groups<LOGS>) restated on the CPU:
every LDS exchange is a bijection between two register layouts, the per-exchange pads are
injective, fit the NP words per polynomial the kernel allocates and split into a per-thread base
plus an immediate offset, and the bank census (MI355X_MICROARCH.md §LDS: 32-lane groups, 32 banks
for 4-byte accesses) is conflict-free at n = 2048 and 4096 — the r2 PMC pass measured
SQ_LDS_BANK_CONFLICT = 0 for the C3 kernel (was 20 % of LDS cycles with e + (e >> 4) alone)."""
import collections

import pytest


class Groups:
    def __init__(self, logs):
        self.L = logs
        self.N = 1 << logs
        self.G = (logs + 3) // 4
        self.TP = self.N // 16
        self.NP = self.N + self.N // 16

    def S(self, g):
        return self.L // self.G + (1 if g < self.L % self.G else 0)

    def ST0(self, g):
        return sum(self.S(i) for i in range(g))

    def NS(self, g):
        return 16 >> self.S(g)

    def LR(self, g):
        return self.L - self.ST0(g) - self.S(g)

    def LNS(self, g):
        return 4 - self.S(g)

    def off(self, g, k):
        ns, lr, s = self.NS(g), self.LR(g), self.S(g)
        m, sidx = k // ns, k % ns
        if lr >= self.LNS(g):
            return sidx + (m << lr)
        return ((sidx >> lr) << (lr + s)) + (sidx & ((1 << lr) - 1)) + (m << lr)

    def base(self, g, j):
        lr, s, lns = self.LR(g), self.S(g), self.LNS(g)
        if lr >= lns:
            set0 = j << lns
            return ((set0 >> lr) << (lr + s)) + (set0 & ((1 << lr) - 1))
        return j << 4

    def padx(self, x, e):  # NTTMUL_PAD0 = 1 (kernels.hip Groups::PS/PT/PS2)
        if self.L in (9, 10):
            s, t = {10: ((6, 3), (4, 1)), 9: ((5, 0), (4, 1))}[self.L][x]
            s2 = 8 if (self.L == 10 or x == 1) else 7
            return e + ((e >> s) << t) + (e >> s2)
        pad0 = self.L >= 10 and self.G > 2
        s, t = (self.L - 4, self.L - 8) if (x == 0 and pad0) else (4, 0)
        return e + ((e >> s) << t)

    @property
    def NPmax(self):
        return max(self.N + self.N // 16, max(self.padx(x, self.N - 1) for x in range(self.G - 1)) + 1)


@pytest.mark.parametrize("logs", [8, 9, 10, 11, 12])
def test_layouts_and_pads(logs):
    Gr = Groups(logs)
    for g in range(Gr.G):
        elems = sorted(Gr.base(g, j) + Gr.off(g, k) for j in range(Gr.TP) for k in range(16))
        assert elems == list(range(Gr.N)), g          # each layout covers the polynomial once
        for j in range(Gr.TP):
            for k in range(16):
                assert Gr.base(g, j) & Gr.off(g, k) == 0  # bit-disjoint: pad splits
    for x in range(Gr.G - 1):
        p = [Gr.padx(x, e) for e in range(Gr.N)]
        assert len(set(p)) == Gr.N and max(p) < Gr.NPmax
        for g in (x, x + 1):
            for j in range(Gr.TP):
                for k in range(16):
                    e = Gr.base(g, j) + Gr.off(g, k)
                    assert Gr.padx(x, e) == Gr.padx(x, Gr.base(g, j)) + Gr.padx(x, Gr.off(g, k))


def _extra_cycles(Gr, x, g):
    extra = 0
    for k in range(16):
        for j0 in range(0, Gr.TP, 32):
            banks = collections.defaultdict(set)
            for j in range(j0, min(j0 + 32, Gr.TP)):
                a = Gr.padx(x, Gr.base(g, j) + Gr.off(g, k))
                banks[a % 32].add(a)
            extra += max(len(v) for v in banks.values()) - 1
    return extra


@pytest.mark.parametrize("logs,expected", [(12, 0), (11, 0), (10, 0), (9, 16), (8, 0)])
def test_bank_census(logs, expected):
    """Extra LDS cycles over all exchange accesses (both layouts of every exchange)."""
    Gr = Groups(logs)
    total = sum(_extra_cycles(Gr, x, g) for x in range(Gr.G - 1) for g in (x, x + 1))
    assert total == expected


class GroupsWT(Groups):
    """kernels.hip Groups<12, WT=true> (NTTMUL_WAVE_TYPED, an A/B variant): groups 1 and 2 take
    the type bit of the previous group's last stage (element bit 8 / 4) from thread bit 6."""

    def base(self, g, j):
        if g == 1:
            return ((j & 15) + (((j >> 4) & 1) << 9) + (((j >> 5) & 1) << 10) +
                    (((j >> 6) & 1) << 8) + (((j >> 7) & 1) << 11))
        if g == 2:
            return ((j & 63) << 5) + (((j >> 6) & 1) << 4) + (((j >> 7) & 1) << 11)
        return super().base(g, j)

    def padx(self, x, e):
        return e + (e >> 5)


def test_wave_typed_layouts():
    """The WT layouts are bijective and bit-disjoint, the type bit is wave-uniform (thread bit 6,
    the same for all 64 lanes of a wave), and e + (e >> 5) is conflict-free on both exchanges."""
    Gr = GroupsWT(12)
    for g in range(3):
        elems = sorted(Gr.base(g, j) + Gr.off(g, k) for j in range(Gr.TP) for k in range(16))
        assert elems == list(range(Gr.N))
        assert all(Gr.base(g, j) & Gr.off(g, k) == 0 for j in range(Gr.TP) for k in range(16))
    for g, bit in ((1, 8), (2, 4)):
        for w in range(4):
            types = {(Gr.base(g, j) >> bit) & 1 for j in range(64 * w, 64 * w + 64)}
            assert len(types) == 1 and types == {(w & 1)}
    assert sum(_extra_cycles(Gr, x, g) for x in range(2) for g in (x, x + 1)) == 0
