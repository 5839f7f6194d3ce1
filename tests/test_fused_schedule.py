"""The fused int8 kernel's work split (qmha_fa_int8.hip, FL_FUSED), restated on the
CPU: which workgroup quantises which K/V groups, and whether every workgroup's wait is satisfied
without depending on a workgroup dispatched after it.

Model: the dispatcher deals workgroup ids round-robin over 8 XCDs (blockIdx % 8), xcd_remap gives
XCD x the contiguous logical range [c0, c1), dispatched in order, R resident at a time, all with the
same lifetime, so logical id c0 + pos runs in round pos // R.  A workgroup produces its "pre" items,
waits until every group of its head is flagged, then produces its "post" items.  The schedule is
sound when each group a workgroup waits for has a producer that (a) runs in an earlier round,
(b) runs in the same round and produces it before its own wait (the first round is resident at
once), or (c) was dispatched before it in the same range (its own wait depends only on workgroups
dispatched before it, so it finishes that wait and produces).  Anything else would leave a resident
workgroup waiting on one that cannot start until it finishes -- the kernel's bounded wait would then
quantise the group itself.
"""
import itertools

import pytest


def ranges(nwg):
    q, r = divmod(nwg, 8)
    out = []
    for x in range(8):
        lo = x * (q + 1) if x < r else r * (q + 1) + (x - r) * q
        out.append((lo, lo + (q + 1 if x < r else q)))
    return out


def production(wg, nwg, nqb, R, rng):
    """(pre, post) lists of workgroup ids whose own groups workgroup `wg` writes (the kernel's
    n_own / n_orph / v_ahead rule, mode 0)."""
    c0, c1 = rng
    pos = wg - c0
    j0 = c0 % nqb
    Rp = min(R, c1 - c0)
    first = pos < R
    v_ahead = wg + R
    ahead = v_ahead < c1
    early = ahead and (v_ahead // nqb) * nqb <= (c0 + Rp - 1 if first else wg)
    pre = [wg] if first else []
    if first and pos < j0:
        pre += [c0 - j0 + pos + m * Rp for m in range((j0 - 1 - pos) // Rp + 1)]
    if early:
        pre.append(v_ahead)
    post = [v_ahead] if ahead and not early else []
    return pre, post


def check(B, H, N, R, waves=4):
    G = N // 32
    nqb = -(-G // waves)
    nwg = B * H * nqb
    rgs = ranges(nwg)
    rng_of, round_of = {}, {}
    for c0, c1 in rgs:
        for v in range(c0, c1):
            rng_of[v] = (c0, c1)
            round_of[v] = (v - c0) // R
    producers = {}  # owner workgroup id -> [(producer, is_pre)]
    for w in range(nwg):
        pre, post = production(w, nwg, nqb, R, rng_of[w])
        for v in pre:
            producers.setdefault(v, []).append((w, True))
        for v in post:
            producers.setdefault(v, []).append((w, False))
    assert set(producers) == set(range(nwg)), "every workgroup's groups are produced"
    late = 0
    for w in range(nwg):
        h = w // nqb
        for v in range(h * nqb, min((h + 1) * nqb, nwg)):
            ok = any(round_of[p] < round_of[w] or
                     (round_of[p] == round_of[w] and (is_pre or (rng_of[p] == rng_of[w] and p < w)))
                     for p, is_pre in producers[v])
            late += not ok
    return late, nwg


@pytest.mark.parametrize("B,H,N,R", [
    (16, 16, 4096, 96),   # C4 at d = 64 (3 workgroups per CU x 32 CUs per XCD)
    (1, 16, 4096, 96),    # one C4 sequence per call: a single round
    (1, 32, 8192, 128),   # the reference's shape at d = 32 (4 per CU): two rounds
    (4, 32, 8192, 128),
    (2, 4, 2048, 64),     # d = 128 (2 per CU)
    (5, 3, 2080, 96),     # ragged: heads straddle the XCD ranges and the rounds
    (3, 2, 96, 96),       # nqb = 1
    (16, 16, 4096, 50),   # an occupancy that does not divide the head
])
def test_fused_split_is_sound(B, H, N, R):
    late, nwg = check(B, H, N, R)
    assert late == 0, (late, nwg)


def test_fused_split_sound_whenever_a_head_fits_a_round():
    """Random shapes with nqb <= R (a head's workgroups no more than one round of an XCD): never a
    late producer.  Longer heads (B2 N131072 at R = 96: 49152 late waits) are routed to the two
    launches by the launcher (fa_int8_fused_launch: nqb > R)."""
    import random
    rnd = random.Random(1)
    n = 0
    while n < 150:
        R = rnd.choice([32, 50, 64, 96, 128])
        B, H, N = rnd.randint(1, 12), rnd.randint(1, 20), 32 * rnd.randint(2, 400)
        if -(-(N // 32) // 4) > R:
            continue
        n += 1
        late, nwg = check(B, H, N, R)
        assert late == 0, (B, H, N, R, late, nwg)
    assert check(2, 1, 131072, 96)[0] > 0


@pytest.mark.parametrize("nwg", [8, 9, 64, 100, 8191, 8192])
def test_ranges_match_xcd_remap(nwg):
    """ranges() is the inverse image of qmha_common.hpp xcd_remap: blockIdx b of XCD b % 8 maps to
    c0(b % 8) + b // 8, and the map is a bijection onto [0, nwg)."""
    rg = ranges(nwg)
    q, r = divmod(nwg, 8)

    def xcd_remap(orig):
        xcd, slot = orig % 8, orig // 8
        return (xcd * (q + 1) if xcd < r else r * (q + 1) + (xcd - r) * q) + slot
    img = [xcd_remap(b) for b in range(nwg)]
    assert sorted(img) == list(range(nwg))
    for b in range(nwg):
        c0, c1 = rg[b % 8]
        assert c0 <= img[b] < c1 and img[b] - c0 == b // 8
    assert list(itertools.chain.from_iterable(range(*x) for x in rg)) == list(range(nwg))


@pytest.mark.parametrize("B,H,N,R", [
    (16, 16, 4096, 64),   # C3 at d = 64: 8-wave workgroups (2 per CU x 32 CUs per XCD)
    (1, 16, 4096, 64),    # one C3 sequence per call
    (2, 4, 2048, 64),     # d = 128 keeps 4-wave workgroups (checked above); a smaller R here
    (5, 3, 2080, 48),     # ragged
    (3, 2, 96, 64),
])
def test_fused_split_is_sound_8_wave_workgroups(B, H, N, R):
    """The same split for the fp16 kernel's 8-wave workgroups (256 query rows, 8 groups produced per workgroup,
    qmha_fa_f16.hip F16_FUSED)."""
    late, nwg = check(B, H, N, R, waves=8)
    assert late == 0, (late, nwg)
