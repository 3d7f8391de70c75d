"""CPU checks of the statistical-outlier-removal oracle (oracle/sor_ref.py).

The oracle restates Open3D's RemoveStatisticalOutliers (refine_point_cloud,
backend/app.py:252-269; open3d>=0.17.0 is absent here, so parity with Open3D itself
is unpinned).  Its KD-tree kNN is pinned to exhaustive search here, including ties
and coincident points.
"""
import numpy as np
import pytest

from oracle import sor_ref


def _cloud(n, seed, dup=0):
    rng = np.random.Generator(np.random.PCG64(seed))
    p = rng.normal(0.0, 1.0, (n, 3)).astype(np.float32)
    p[: n // 50] *= 8.0                                   # a few far outliers
    if dup:
        p[-dup:] = p[0]                                   # coincident points
    return p


@pytest.mark.parametrize("k", [1, 5, 20, 32])
def test_kdtree_matches_brute_force(k):
    p = _cloud(700, 3, dup=30)
    a = sor_ref.knn_mean_distances(p, k)
    b = sor_ref.knn_mean_distances_brute(p, k)
    assert a.tobytes() == b.tobytes()


def test_grid_lattice_ties_match_brute_force():
    # integer lattice: many equal distances at the k-th neighbour
    g = np.stack(np.meshgrid(np.arange(9), np.arange(9), np.arange(3), indexing="ij"), -1).reshape(-1, 3)
    p = g.astype(np.float32) * 0.5
    assert sor_ref.knn_mean_distances(p, 20).tobytes() == sor_ref.knn_mean_distances_brute(p, 20).tobytes()


def test_selection_rule():
    p = _cloud(2000, 4)
    ind, avg, thr = sor_ref.remove_statistical_outlier(p, 20, 2.0)
    assert np.all(np.diff(ind) > 0)
    keep = (avg > 0) & (avg < thr)
    assert np.array_equal(np.nonzero(keep)[0], ind)
    mean = np.mean(avg[avg > 0])
    std = np.std(avg[avg > 0], ddof=1)
    assert abs(thr - (mean + 2.0 * std)) < 1e-9 * thr
    assert len(ind) < len(p)                          # the scaled points are dropped


def test_edge_cases():
    # n < k: every point is a neighbour of every other
    p = _cloud(7, 5)
    ind, avg, _ = sor_ref.remove_statistical_outlier(p, 20, 2.0)
    assert avg.tobytes() == sor_ref.knn_mean_distances_brute(p, 7).tobytes()
    # one point: its only neighbour is itself (avg 0) -> nothing kept
    ind, avg, _ = sor_ref.remove_statistical_outlier(p[:1], 20, 2.0)
    assert len(ind) == 0 and avg[0] == 0.0
    # all coincident: avg 0 everywhere -> nothing kept
    ind, _, _ = sor_ref.remove_statistical_outlier(np.zeros((50, 3), np.float32), 20, 2.0)
    assert len(ind) == 0
    # empty
    ind, avg, _ = sor_ref.remove_statistical_outlier(np.zeros((0, 3), np.float32))
    assert len(ind) == 0
    with pytest.raises(ValueError):
        sor_ref.remove_statistical_outlier(p, 0, 2.0)
    with pytest.raises(ValueError):
        sor_ref.remove_statistical_outlier(p, 20, 0.0)


def test_refine_point_cloud_shapes():
    p = _cloud(500, 6)
    c = np.random.default_rng(0).integers(0, 256, (500, 3)).astype(np.float32)
    pf, cf = sor_ref.refine_point_cloud(p, c)
    ind, _, _ = sor_ref.remove_statistical_outlier(p)
    assert np.array_equal(pf, p[ind]) and np.array_equal(cf, c[ind])
    e = np.zeros((0, 3), np.float32)
    assert sor_ref.refine_point_cloud(e, e)[0] is e
