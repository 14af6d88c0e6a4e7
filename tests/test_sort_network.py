"""CPU model of the merge's register sort (pmm_kernels.hip, wave_sort128_desc):
the lane permutations it builds from DPP controls, and the bitonic network with
its compile-time keep-the-larger lane masks (sort128_keepmax), replayed on
random keys.  The GPU suite runs the kernel itself (every merge forced onto
the sort with PMM_MERGE_RANK=0 in round 6's A/B runs); this pins the network's
derivation where no GPU is needed."""
import numpy as np


def dpp(v, ctrl):
    """v_mov_b32_dpp on 64 lanes: lane l receives v[src(l)]."""
    out = np.empty_like(v)
    for l in range(64):
        if ctrl <= 0xFF:  # quad_perm
            sel = (ctrl >> (2 * (l & 3))) & 3
            src = (l & ~3) | sel
        elif ctrl == 0x140:  # row_mirror: within 16
            src = (l & ~15) | (15 - (l & 15))
        elif ctrl == 0x141:  # row_half_mirror: within 8
            src = (l & ~7) | (7 - (l & 7))
        else:
            raise ValueError(ctrl)
        out[l] = v[src]
    return out


def lane_xor(v, s):
    if s == 1:
        return dpp(v, 0xB1)
    if s == 2:
        return dpp(v, 0x4E)
    if s == 4:
        return dpp(dpp(v, 0x141), 0x1B)
    if s == 8:
        return dpp(dpp(v, 0x140), 0x141)
    if s == 16:  # ds_bpermute
        return v[np.arange(64) ^ 16]
    # v_permlane32_swap(v, v): r0 = both halves' low half, r1 = the high half
    r0 = np.concatenate([v[:32], v[:32]])
    r1 = np.concatenate([v[32:], v[32:]])
    return np.where(np.arange(64) < 32, r1, r0)


def keepmax(size, s, r):
    m = np.zeros(64, dtype=bool)
    for l in range(64):
        lower = (l & s) == 0
        d = True if size > 64 else (r == 0 if size == 64 else (l & size) == 0)
        m[l] = lower == d
    return m


def sort128(y0, y1):
    def step(size, s):
        nonlocal y0, y1
        p0, p1 = lane_xor(y0, s), lane_xor(y1, s)
        t0 = (y0 > p0) ^ keepmax(size, s, 0)
        t1 = (y1 > p1) ^ keepmax(size, s, 1)
        y0 = np.where(t0, p0, y0)
        y1 = np.where(t1, p1, y1)

    size = 2
    while size <= 64:
        s = size // 2
        while s >= 1:
            step(size, s)
            s //= 2
        size *= 2
    y0, y1 = np.maximum(y0, y1), np.minimum(y0, y1)
    s = 32
    while s >= 1:
        step(128, s)
        s //= 2
    return y0, y1


def test_lane_permutations_are_xors():
    v = np.arange(64)
    for s in (1, 2, 4, 8, 16, 32):
        assert np.array_equal(lane_xor(v, s), v ^ s), s


def test_register_bitonic_sorts_descending():
    rng = np.random.default_rng(0)
    for trial in range(200):
        n = int(rng.integers(0, 129))
        keys = np.unique(rng.integers(1, 1 << 62, size=n, dtype=np.uint64))  # distinct, as composites are
        n = len(keys)
        slots = np.zeros(128, dtype=np.uint64)  # empty slots are 0, sorted last
        slots[:n] = keys
        rng.shuffle(slots)
        y0, y1 = sort128(slots[:64].copy(), slots[64:].copy())
        out = np.concatenate([y0, y1])
        assert np.array_equal(out, np.sort(slots)[::-1]), trial
