"""CPU model of the tile-bound threshold (no GPU): the per-(term, tile) f16
maxima rounded down (build_bmax_kernel), the threshold from them
(bound_keys_kernel) and from the same bounds pooled over groups of 4 tiles
(pool_bounds_kernel, option bound_pool) — both must stay at or below the
k-th best fp32 score, the pooled one at or below the per-tile one
(DESIGN.md §4).  The scores come from the canonical oracle's arithmetic
(fp32, terms in query order)."""
import numpy as np
import pytest

TILE = 2048


def _f16_down(x: np.ndarray) -> np.ndarray:
    """f16 rounded to nearest, then one step down where that rounded up
    (build_bmax_kernel: a bound <= the real maximum)."""
    h = x.astype(np.float16)
    up = h.astype(np.float32) > x
    h[up] = np.nextafter(h[up], np.float16(-np.inf))
    return h.astype(np.float32)


def _case(seed, N, V):
    rng = np.random.default_rng(seed)
    cols = []
    for t in range(V):
        df = int(rng.integers(1, N // (3 if t < 10 else 200)))
        idx = np.unique(rng.integers(0, N, df)).astype(np.int64)  # sorted, unique
        val = (rng.uniform(0.1, 1.0, len(idx)) * (1.0 if t < 10 else 6.0)).astype(np.float32)
        cols.append((idx, val))
    return cols


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_pooled_tile_bound_threshold_is_a_lower_bound(seed):
    N, V, T = 300_000, 80, 8
    ntiles = (N + TILE - 1) // TILE
    cols = _case(seed, N, V)
    bmax = np.zeros((V, ntiles), np.float32)
    for t, (idx, val) in enumerate(cols):
        tiles, start = np.unique(idx // TILE, return_index=True)  # (idx sorted)
        m = np.zeros(ntiles, np.float32)
        m[tiles] = np.maximum.reduceat(val, start)
        bmax[t] = _f16_down(m)
    rng = np.random.default_rng(100 + seed)
    for _ in range(12):
        q = rng.choice(V, T, replace=False)
        acc = np.zeros(N, np.float32)
        for t in q:  # fp32, query order: each doc once per term
            idx, val = cols[t]
            acc[idx] += val
        best = np.sort(acc)[::-1]
        lb = bmax[q].max(axis=0)                            # per tile
        ng = (ntiles + 3) // 4
        lbp = np.pad(lb, (0, ng * 4 - ntiles)).reshape(ng, 4).max(axis=1)  # per group of 4
        for k in (1, 5, 20, ng):  # (k <= the groups: one key each)
            th_tile = np.sort(lb)[::-1][k - 1]
            th_pool = np.sort(lbp)[::-1][k - 1]
            assert th_pool <= th_tile <= best[k - 1], (k, th_pool, th_tile, best[k - 1])
