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


# --- the device server's two-wave n = 256 path (kernels.hip wl_elem / wl_swap_64 / wl_swap_42) ---

def wl_elem(p, t, i):
    """Element held by lane t, register i of layout p (register bits = element bits p, p + 1)."""
    return (t & ((1 << p) - 1)) | ((t >> p) << (p + 2)) | (i << p)


def permlane_swap(x, a, b, bit):
    """v_permlane16_swap (bit 4) / v_permlane32_swap (bit 5) of registers a (vdst) and b (vsrc):
    the lanes of a with the bit set trade places with the lanes of b with it clear."""
    xa, xb = list(x[a]), list(x[b])
    for t in range(64):
        if t & (1 << bit):
            xa[t], xb[t - (1 << bit)] = x[b][t - (1 << bit)], x[a][t]
    x[a], x[b] = xa, xb


def dpp_swap(x, a, b, sh):
    """wl_swap_dpp<SH, A, B>: row_shr / row_shl by SH lanes inside 16-lane rows and two selects."""
    up = [x[b][t - sh] if (t % 16) >= sh else 0 for t in range(64)]       # row_shr:SH of x[b]
    dn = [x[a][t + sh] if (t % 16) + sh < 16 else 0 for t in range(64)]   # row_shl:SH of x[a]
    x[a] = [up[t] if t & sh else x[a][t] for t in range(64)]
    x[b] = [x[b][t] if t & sh else dn[t] for t in range(64)]


def layout(p):
    return [[wl_elem(p, t, i) for t in range(64)] for i in range(4)]


def test_server_wide_layouts_are_bijections():
    """Each layout of the two-wave path holds every one of the 256 elements exactly once, and the
    LDS pad e + (e >> 5) stays inside the kernel's per-wave region (NP words at n = 256)."""
    for p in (6, 4, 2, 0):
        els = [e for reg in layout(p) for e in reg]
        assert sorted(els) == list(range(256)), p
    assert max(e + (e >> 5) for e in range(256)) < Groups(8).NP


def test_server_wide_in_wave_swaps():
    """The permlane and DPP sequences that replaced two LDS exchanges per transform move every
    element exactly where the next layout expects it (layouts 6 <-> 4 and 4 <-> 2, both ways)."""
    def swap_64(x):
        permlane_swap(x, 0, 1, 4)
        permlane_swap(x, 2, 3, 4)
        permlane_swap(x, 0, 2, 5)
        permlane_swap(x, 1, 3, 5)

    def swap_42(x):
        dpp_swap(x, 0, 1, 4)
        dpp_swap(x, 2, 3, 4)
        dpp_swap(x, 0, 2, 8)
        dpp_swap(x, 1, 3, 8)

    for f, src, dst in ((swap_64, 6, 4), (swap_64, 4, 6), (swap_42, 4, 2), (swap_42, 2, 4)):
        x = layout(src)
        f(x)
        assert x == layout(dst), (src, dst)


def test_server_wide_stage_pairs_and_twiddles():
    """In every layout the butterfly partners of a stage sit in the register pairs the kernel
    pairs (register bit 1 for a group's first stage, bit 0 for its second), and the twiddle entry
    the kernel loads for each pair (kernels.hip wide_tw) is the reference table's entry for that
    butterfly, 2^s + e >> (8 - s) with e the pair's lower element; the base block of lane t in
    layout 0 takes stage 5's entry 32 + t / 2 and is a -w block exactly for odd t."""
    def kernel_entry(s, t, pair_hi):  # wide_tw's index for stage s, the pair (0,1) or (2,3)/(1,3)
        k3, k5 = 8 + ((t >> 4) << 1), 32 + ((t >> 2) << 1)
        return {0: 1, 1: 2 + pair_hi, 2: 4 + (t >> 4), 3: k3 + pair_hi, 4: 16 + (t >> 2),
                5: k5 + pair_hi}[s]
    groups = {6: (0, 1), 4: (2, 3), 2: (4, 5)}
    for p, (s0, s1) in groups.items():
        for s, rbit in ((s0, 1), (s1, 0)):
            d = 128 >> s
            pairs = [(0, 2), (1, 3)] if rbit == 1 else [(0, 1), (2, 3)]
            for t in range(64):
                for hi, (i, j) in enumerate(pairs):
                    e, f = wl_elem(p, t, i), wl_elem(p, t, j)
                    assert f - e == d and not e & d, (p, s, t, i)
                    # the second-of-group stages pick the entry by the pair, the first by the lane
                    got = kernel_entry(s, t, hi if rbit == 0 else 0)
                    assert got == (1 << s) + (e >> (8 - s)), (p, s, t, i, got)
    for t in range(64):
        e0 = wl_elem(0, t, 0)
        assert e0 == 4 * t and 32 + (t >> 1) == 32 + (e0 >> 3) and ((e0 >> 2) & 1) == (t & 1)
