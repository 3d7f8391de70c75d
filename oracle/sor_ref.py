"""CPU restatement of the reference's statistical outlier removal.  TEST INFRASTRUCTURE ONLY.

backend/app.py:252-269 (`refine_point_cloud`) hands the float64 copy of the cloud to
Open3D's `PointCloud.remove_statistical_outlier(nb_neighbors=20, std_ratio=2.0)`
(open3d>=0.17.0, backend/requirements.txt:14) and keeps `points[ind]`.  Open3D is not
installed here, so this restates its published algorithm (PointCloud::
RemoveStatisticalOutliers):

  * avg[i]  -- mean of the Euclidean distances from point i to its k = min(nb_neighbors, n)
               nearest points of the cloud; the KD-tree query returns point i itself
               (distance 0).  Squared distances are nanoflann's L2 metric in float64,
               ((dx*dx + dy*dy) + dz*dz); they come back sorted ascending, are square-
               rooted, and std::accumulate sums them in that order;
  * mean    -- (sum over avg[i] > 0, in index order) / n   (n = points with neighbours);
  * std     -- sqrt(sum over avg[i] > 0 of (avg[i] - mean)^2 / (n - 1))  (Bessel);
  * keep i  iff 0 < avg[i] < mean + std_ratio * std, ascending indices.

Parity against Open3D itself is unpinned (no Open3D in this image); the exact kNN here
is scipy's cKDTree (eps = 0), checked against brute force in tests/test_sor.py.  The
sequential sums use np.cumsum, which accumulates left to right like std::accumulate.
"""
from __future__ import annotations

import numpy as np


def _check(nb_neighbors: int, std_ratio: float) -> None:
    if nb_neighbors < 1 or not std_ratio > 0:
        # Open3D: "Illegal input parameters, the number of neighbors and standard deviation
        # ratio must be positive."
        raise ValueError("Illegal input parameters, the number of neighbors and standard deviation ratio "
                         "must be positive.")


def _avg_from_neighbours(p: np.ndarray, idx: np.ndarray) -> np.ndarray:
    d = p[:, None, :] - p[idx]                                   # query - neighbour (nanoflann order)
    d2 = (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]
    d2.sort(axis=1)                                              # ascending, as the KNN result set
    s = np.sqrt(d2)
    return np.cumsum(s, axis=1)[:, -1] / s.shape[1]


def knn_mean_distances(points, nb_neighbors: int = 20) -> np.ndarray:
    """avg[i] of RemoveStatisticalOutliers (float64 [n])."""
    from scipy.spatial import cKDTree
    p = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 3)
    n = len(p)
    k = min(int(nb_neighbors), n)
    _, idx = cKDTree(p).query(p, k=k, workers=-1)
    return _avg_from_neighbours(p, np.asarray(idx).reshape(n, k))


def knn_mean_distances_brute(points, nb_neighbors: int = 20) -> np.ndarray:
    """The same quantity by exhaustive search (small n only; pins the KD-tree path)."""
    p = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 3)
    n = len(p)
    k = min(int(nb_neighbors), n)
    d = p[:, None, :] - p[None, :, :]
    d2 = (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]
    d2.sort(axis=1)
    s = np.sqrt(d2[:, :k])
    return np.cumsum(s, axis=1)[:, -1] / k


def threshold(avg: np.ndarray, std_ratio: float) -> tuple:
    """(mean, std, threshold) exactly as Open3D forms them from avg."""
    n = len(avg)
    pos = np.where(avg > 0, avg, 0.0)
    mean = np.cumsum(pos)[-1] / n
    dev = np.where(avg > 0, (avg - mean) * (avg - mean), 0.0)
    sq = np.cumsum(dev)[-1]
    with np.errstate(all="ignore"):
        std = np.sqrt(sq / np.float64(n - 1))
    return float(mean), float(std), float(mean + std_ratio * std)


def remove_statistical_outlier(points, nb_neighbors: int = 20, std_ratio: float = 2.0, avg=None):
    """-> (ind int64 ascending, avg float64 [n], threshold)."""
    _check(nb_neighbors, std_ratio)
    p = np.asarray(points).reshape(-1, 3)
    if len(p) == 0:
        return np.zeros(0, np.int64), np.zeros(0), float("nan")
    if avg is None:
        avg = knn_mean_distances(p, nb_neighbors)
    _, _, thr = threshold(avg, std_ratio)
    ind = np.nonzero((avg > 0) & (avg < thr))[0].astype(np.int64)
    return ind, avg, thr


def refine_point_cloud(points, colors, nb_neighbors: int = 20, std_ratio: float = 2.0):
    """backend/app.py:252-269 with the Open3D call restated."""
    if points is None or len(points) == 0:
        return points, colors
    ind, _, _ = remove_statistical_outlier(points, nb_neighbors, std_ratio)
    cols = colors[ind] if colors is not None and len(colors) == len(points) else colors
    return points[ind], cols
