"""CPU tests of the in-process multi-GPU path's memory plan (pmm_shard_plan,
the pure planner topk_sharded runs).  The one-GPU test box
can only list device 0 repeatedly, which collapses every shard into one plan;
these tests cover the distinct-device plans that only a multi-GPU node runs."""
import numpy as np
import pytest

from polars_matmul import _native

M, N, D, K = 1000, 100_003, 768, 100
LIST = 2 * M * K * 4


def al256(x):
    return (x + 255) & ~255


@pytest.mark.parametrize("compute", [_native.COMPUTE_F32, _native.COMPUTE_BF16])
@pytest.mark.parametrize("host_rows", [True, False])
def test_distinct_devices_one_plan_each(compute, host_rows):
    devs = [0, 1, 2, 3, 4, 5, 6, 7]
    plan_of, plans, offs = _native.shard_plan(devs, M, N, D, K, _native.METRIC_COSINE, compute, host_rows)
    assert plan_of == list(range(8))
    assert [p[0] for p in plans] == devs
    # root (device 0) additionally holds the gathered [G][2][M][k] lists and the output
    sizes = [p[1] for p in plans]
    assert sizes[0] - max(sizes[1:]) >= 9 * LIST - (1 << 16)  # shards differ by <= 1 row
    for j in range(1, 8):
        assert sizes[j] >= LIST + M * D * (2 if compute else 4)
        assert offs[j] + LIST <= sizes[j]
    # shards differ by at most one row, so the non-root plans differ by little
    assert max(sizes[1:]) - min(sizes[1:]) <= 1 << 16


def test_repeated_device_shares_one_plan_disjoint_lists():
    plan_of, plans, offs = _native.shard_plan([0, 0, 1], M, N, D, K, _native.METRIC_DOT)
    assert plan_of == [0, 0, 1]
    assert [p[0] for p in plans] == [0, 1]
    # the two shards on device 0 have their own rows and lists, not overlapping
    rows0 = N // 3
    lo, hi = sorted(offs[:2])
    assert hi - lo >= al256(LIST) + rows0 * D * 4
    assert offs[2] + LIST <= plans[1][1]


def test_root_is_first_listed_device():
    plan_of, plans, _ = _native.shard_plan([3, 1, 3, 2], M, N, D, K, _native.METRIC_EUCLIDEAN)
    assert plan_of == [0, 1, 0, 2]
    assert [p[0] for p in plans] == [3, 1, 2]
    assert plans[0][1] > plans[1][1]  # the root also holds the gather buffer


def test_resident_rows_plan_smaller_than_host_rows():
    _, ph, _ = _native.shard_plan([0, 1], M, N, D, K, _native.METRIC_COSINE, host_rows=True)
    _, pr, _ = _native.shard_plan([0, 1], M, N, D, K, _native.METRIC_COSINE, host_rows=False)
    for (dh, bh), (dr, br) in zip(ph, pr):
        assert dh == dr and bh - br >= (N // 2) * D * 4


def test_shard_plan_rejects_bad_sizes():
    with pytest.raises(_native.PmmError):
        _native.shard_plan([0, 1], M, 1, D, K, _native.METRIC_COSINE)  # fewer rows than shards
    with pytest.raises(_native.PmmError):
        _native.shard_plan([0], M, N, D, 2000, _native.METRIC_COSINE)  # k beyond the fused path
