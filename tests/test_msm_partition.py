"""bench.py's multi-GPU MSM partitions (msm_partition: point shards, the window
split and the hybrid; auto = the library's plan, tachyon_mi355x_msm_shard_plan):
for every curve and world size the ranks' (point range, window range) shares
tile the (point, window) pairs of the MSM exactly once -- the property that
makes the all-gather + group sum of the partials the MSM -- and the shard the
library's sharded entry takes says the same.  Host logic only (the library
loads without a GPU; the plan is pure host code)."""
import argparse
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from tachyon_amd import dist as D  # noqa: E402


def _args(split, window_groups=2, window_bits=0):
    return argparse.Namespace(msm_split=split, window_groups=window_groups, window_bits=window_bits)


def _tiles(curve, world, args, n_total):
    cover = {}
    for rank in range(world):
        split, start, n, wrange, c, p, q, shard = bench.msm_partition(args, curve, world, rank, n_total)
        W = D._windows_for(curve, c) if c else 1
        w0, w1 = wrange if wrange is not None else (0, W)
        if shard is not None:  # the library's shard record agrees
            assert (shard.start, shard.count, shard.point_groups, shard.window_groups) == (start, n, p, q)
            if q > 1:
                assert (shard.window_bits, shard.w_begin, shard.w_end) == (c, w0, w1)
        for w in range(w0, w1):
            cover.setdefault(w, []).append((start, start + n))
        assert p * q == world
    return cover, W


@pytest.mark.parametrize("curve", ["bn254_g1", "bls12_381_g1", "bls12_381_g2"])
@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("split", ["auto", "points", "windows", "hybrid"])
def test_partition_tiles_every_point_window_pair_once(curve, world, split):
    n_total = 1000 + 7 * world  # ragged shards
    cover, W = _tiles(curve, world, _args(split), n_total)
    assert sorted(cover) == list(range(W))
    for w, ranges in cover.items():
        ranges.sort()
        assert ranges[0][0] == 0 and ranges[-1][1] == n_total, (w, ranges)
        for (a0, a1), (b0, b1) in zip(ranges, ranges[1:]):
            assert a1 == b0, (w, ranges)


def test_auto_follows_the_plan_table():
    plans = bench.hybrid_plans()
    # the measured table in capi.hip (kHybridPlans)
    assert plans == {("bn254_g1", 8): (2, 19), ("bls12_381_g2", 4): (2, 19), ("bls12_381_g2", 8): (4, 16)}
    for (curve, world), (q, c) in plans.items():
        split, _, n, wrange, cc, p, qq, _ = bench.msm_partition(_args("auto"), curve, world, 0, 1 << 20)
        assert (split, qq, cc, p) == ("hybrid", q, c, world // q)
        assert n == (1 << 20) // p and wrange == D.window_range(D._windows_for(curve, c), 0, q)
    # no plan: point shards (BN254 at 2 and 4 GPUs measured no faster as the hybrid)
    for world in (2, 4):
        assert bench.msm_partition(_args("auto"), "bn254_g1", world, 1, 1 << 20)[0] == "points"
    assert bench.msm_partition(_args("auto"), "bn254_g1", 1, 0, 1 << 20)[0] == "points"


def test_library_shard_plan_refuses_bad_ranks():
    from tachyon_amd import msm as M
    with pytest.raises(ValueError):
        M.shard_plan("bn254_g1", 100, 4, 4)
    with pytest.raises(ValueError):
        M.shard_plan("bn254_g1", 100, 0, 0)
    s = M.shard_plan("bn254_g1", 0, 8, 7)  # an empty MSM: empty shards
    assert s.count == 0
