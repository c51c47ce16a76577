"""CPU model check of the leaf exchange (trace builds 53 / 54 / 59, csrc/traverse.hpp leaf_exchange).

The exchange hands a wave's (lane, reference) pairs of one divergent leaf round to the 64 lanes, 64 at a
time.  This restates its index arithmetic operation for operation -- the bit-sliced exclusive prefix of
the mask popcounts, the window's start marks in LDS (cleared, then written by the owners whose first pair
falls in the window), the shifted ballot and count of leading zeros that find a pair's start, the owner
and rank carried from one window into the next, and nth_bit's five-step popcount search -- and checks on
random waves that every (lane, mask bit) pair is handed out exactly once, in mask order within each
owner.  It also checks the two reductions against the per-lane loop they replace (kdtree.cpp:235-246,
309-320): the closest hit (smallest t, ties and +0 / -0 to the first in mask order, the loop's strict
t < tmax) and the shadow answer (an OR over the masked references other than the excluded one).
The GPU tests check the kernels themselves bit-exact against the oracle
(test_gpu_parity.py test_leaf_exchange_ties_and_windows_bitexact, test_wavefront_trace_builds_bitexact).
"""
import random
import struct

import pytest

M64 = (1 << 64) - 1


def popc(x):
    return bin(x).count("1")


def clz64(x):
    return 64 - x.bit_length()


def ballot(pred):
    return sum(1 << lane for lane, p in enumerate(pred) if p)


def mbcnt(bal, lane):
    """v_mbcnt_lo / hi: the set bits of bal below the lane."""
    return popc(bal & ((1 << lane) - 1))


def nth_bit(m, q):
    """traverse.hpp nth_bit: the position of the q-th (from 0) set bit of m."""
    pos = 0
    w = 16
    while w >= 1:
        c = popc(m & ((1 << w) - 1))
        up = q >= c
        q = q - c if up else q
        m = m >> w if up else m
        pos = pos + w if up else pos
        w >>= 1
    return pos


def exchange(masks, rng):
    """The pairs (owner, bit) in the order the exchange tests them: a list of windows, each a list of
    (lane, owner, bit) for its live lanes."""
    c = [popc(m) for m in masks]
    P = [0] * 64
    total = 0
    for b in range(6):  # bit-sliced prefix (c <= 32)
        bal = ballot([(ci >> b) & 1 for ci in c])
        for lane in range(64):
            P[lane] += mbcnt(bal, lane) << b
        total += popc(bal) << b
    pe = [P[lane] | ((P[lane] + c[lane]) << 16) for lane in range(64)]
    marks = [rng.getrandbits(32) for _ in range(64)]  # LDS holds garbage before the first clear
    carry = carry_q = 0
    windows = []
    base = 0
    while base < total:
        marks = [0] * 64
        for ln in range(64):
            p0, e0 = pe[ln] & 0xFFFF, pe[ln] >> 16
            if e0 > p0 and base <= p0 < base + 64:
                marks[p0 - base] = ln + 1
        mv = list(marks)
        starts = ballot([v != 0 for v in mv])
        owner, q = [0] * 64, [0] * 64
        for ln in range(64):
            upto = (starts << (63 - ln)) & M64
            back = clz64(upto) if upto else 0
            sm = mv[ln - back]  # ds_bpermute of the mark at lane ln - back
            owner[ln] = sm - 1 if upto else carry
            q[ln] = back if upto else ln + carry_q
        carry = owner[63]
        carry_q = q[63] + 1
        win = []
        for ln in range(64):
            if base + ln < total:
                win.append((ln, owner[ln], nth_bit(masks[owner[ln]], q[ln])))
        windows.append(win)
        base += 64
    return windows, P, c


def random_masks(rng, kind):
    masks = []
    for _ in range(64):
        r = rng.random()
        if kind == "sparse" and r < 0.7:
            masks.append(0)
        elif kind == "full" and r < 0.5:
            masks.append((1 << 32) - 1 if rng.random() < 0.5 else (1 << rng.randint(1, 32)) - 1)
        else:
            n = rng.choice([1, 2, 3, 5, 8, 16, 24, 32])
            masks.append(rng.getrandbits(n) << rng.randint(0, 32 - n) & 0xFFFFFFFF)
    return masks


@pytest.mark.parametrize("kind", ["sparse", "mixed", "full"])
def test_exchange_hands_out_every_pair_once_in_mask_order(kind):
    rng = random.Random(1234 + len(kind))
    multi = 0
    for _ in range(400):
        masks = random_masks(rng, kind)
        windows, P, c = exchange(masks, rng)
        multi += len(windows) > 1
        got = [(o, j) for w in windows for (_, o, j) in w]
        want = [(lane, j) for lane in range(64) for j in range(32) if (masks[lane] >> j) & 1]
        assert sorted(got) == want, masks
        assert len(got) == len(set(got)) == sum(c)
        for lane in range(64):  # each owner's pairs come in ascending bit (mask) order
            seq = [j for (o, j) in got if o == lane]
            assert seq == sorted(seq)
        # window lanes are consecutive pair indices: an owner's pairs in a window form the range
        # [P, P + c) clipped to the window, which is what the shadow OR reads from the ballot
        for wi, w in enumerate(windows):
            for (ln, o, _) in w:
                assert P[o] <= wi * 64 + ln < P[o] + c[o]
    if kind == "full":
        assert multi > 300  # most rounds take several windows


def test_nth_bit_is_select():
    rng = random.Random(7)
    for _ in range(20000):
        m = rng.getrandbits(32) | (1 << rng.randint(0, 31))
        bits = [j for j in range(32) if (m >> j) & 1]
        q = rng.randrange(len(bits))
        assert nth_bit(m, q) == bits[q]


def f32(x):
    return struct.unpack("<f", struct.pack("<f", x))[0]


def fbits(x):
    return struct.unpack("<I", struct.pack("<f", x))[0]


def sequential_closest(ts, tmax):
    """The per-lane loop: a hit when 0 <= t < the current tmax (tri_test), which then becomes tmax."""
    found, best_j, best_t = False, None, tmax
    for j, t in ts:
        if t >= 0.0 and t < best_t:
            found, best_j, best_t = True, j, t
    return (best_j, fbits(best_t)) if found else None


def exchange_closest(ts, tmax):
    """The exchange: every pair tested against the entry tmax, the accepting ones reduced in (window,
    lane) = mask order with a strict < on |t|'s bits."""
    found, best_j, best_t = False, None, 0.0
    for j, t in ts:
        if not (t >= 0.0 and t < tmax):
            continue
        if not found or (fbits(t) & 0x7FFFFFFF) < (fbits(best_t) & 0x7FFFFFFF):
            found, best_j, best_t = True, j, t
    return (best_j, fbits(best_t)) if found else None


def test_closest_reduction_equals_the_per_lane_loop():
    rng = random.Random(99)
    pool = [0.0, -0.0, 1.0, 1.0, 2.5, 2.5, 3.0, float("nan"), -1.0, 7.0, 1e-30, 5e-45]
    for _ in range(20000):
        n = rng.randint(1, 32)
        bits = sorted(rng.sample(range(32), n))
        ts = [(j, f32(rng.choice(pool) if rng.random() < 0.6 else rng.uniform(-1, 8))) for j in bits]
        tmax = f32(rng.choice([3.0, 2.5, 8.0, 0.0, float("inf")]))
        assert exchange_closest(ts, tmax) == sequential_closest(ts, tmax), (ts, tmax)


def test_shadow_or_equals_the_per_lane_loop():
    rng = random.Random(5)
    for _ in range(20000):
        n = rng.randint(1, 32)
        ids = rng.sample(range(100), n)
        acc = [rng.random() < 0.1 for _ in ids]
        exclude = rng.choice(ids + [1000])
        seq = False
        for i, a in zip(ids, acc):  # the loop: skip the excluded light triangle, stop at an occluder
            if i == exclude:
                continue
            if a:
                seq = True
                break
        assert any(a and i != exclude for i, a in zip(ids, acc)) == seq


def dpp_incl_scan(x):
    """traverse.hpp wave_incl_scan as the DPP modifiers define it: row_shr:n reads lane - n of the same
    row of 16 (0 outside it: bound_ctrl), row_bcast:15 gives rows 1 and 3 (row_mask 0xa) lane 15 of the
    row below, row_bcast:31 gives rows 2 and 3 (row_mask 0xc) lane 31; masked-off rows add 0 (old = 0)."""
    x = list(x)
    for n in (1, 2, 4, 8):
        src = [x[lane - n] if (lane % 16) >= n else 0 for lane in range(64)]
        x = [a + b for a, b in zip(x, src)]
    src = [x[16 * (lane // 16) - 1] if (lane // 16) in (1, 3) else 0 for lane in range(64)]
    x = [a + b for a, b in zip(x, src)]
    src = [x[31] if (lane // 16) in (2, 3) else 0 for lane in range(64)]
    return [a + b for a, b in zip(x, src)]


def test_dpp_prefix_equals_the_ballot_prefix():
    """Build 59's prefix (the inclusive DPP scan minus the lane's own count) against the bit-sliced
    ballot prefix of builds 53 / 54 and a plain running sum."""
    rng = random.Random(11)
    for _ in range(3000):
        c = [rng.choice([0, 0, 1, 2, 5, 16, 32, rng.randint(0, 32)]) for _ in range(64)]
        inc = dpp_incl_scan(c)
        P_dpp = [i - ci for i, ci in zip(inc, c)]
        P_bal = [0] * 64
        for b in range(6):
            bal = ballot([(ci >> b) & 1 for ci in c])
            for lane in range(64):
                P_bal[lane] += mbcnt(bal, lane) << b
        run = [sum(c[:lane]) for lane in range(64)]
        assert P_dpp == P_bal == run
        assert inc[63] == sum(c)
