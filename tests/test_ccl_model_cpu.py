"""CPU model of the bit-plane run labelling of csrc/ipp_ccl.hip (k_ccl_label,
k_ccl_border, k_ccl_bbox) checked against scipy on random masks.

It restates, in NumPy/Python, the rules the kernels rely on:
  * a run starting at (x, y) has the run-start index
    G = ((y >> 1) * wb + (x >> 1)) * 2 + (y & 1), unique per run start;
  * a component's minimum block-raster pixel is a run start, and G orders
    run starts the way block-raster order orders pixels, so the union-find
    root (min G) is the component OpenCV numbers first (the tie rule,
    pixels_isolés.py:38-44);
  * components that touch no 64×64 tile edge are final inside their tile
    ("closed"), and their 64-bit key orders them by (area, smaller root).
The kernels themselves are checked on the GPU (tests/test_gpu_parity.py).
"""
import numpy as np
import pytest
from scipy import ndimage

TW = TH = 64


def run_starts(mask):
    left = np.zeros_like(mask)
    left[:, 1:] = mask[:, :-1]
    return mask & ~left


def gidx(x, y, wb):
    return ((y >> 1) * wb + (x >> 1)) * 2 + (y & 1)


def block_raster_key(x, y, wb):
    return (((y >> 1) * wb + (x >> 1)) << 2) + ((y & 1) << 1) + (x & 1)


def closed_key(area, G, bx0, by0, bx1, by1):
    return (area << 51) | ((~G & 0x7FFFFF) << 24) | (bx0 | (by0 << 6) | ((bx1 - 1) << 12) | ((by1 - 1) << 18))


def decode_closed(k):
    return k >> 51, (~(k >> 24)) & 0x7FFFFF, k & 63, (k >> 6) & 63, ((k >> 12) & 63) + 1, ((k >> 18) & 63) + 1


def label_runs(mask):
    """Union-find over run starts (8-connectivity between consecutive rows),
    union by min G, as k_ccl_label + k_ccl_border do (tile boundaries only
    change where the unions happen, not their result)."""
    h, w = mask.shape
    wb = (w + 1) // 2
    par = {}
    runs = []
    for y in range(h):
        x = 0
        while x < w:
            if mask[y, x]:
                a = x
                while x < w and mask[y, x]:
                    x += 1
                G = gidx(a, y, wb)
                par[G] = G
                runs.append((y, a, x - 1, G))
            else:
                x += 1

    def find(g):
        while par[g] != g:
            par[g] = par[par[g]]
            g = par[g]
        return g

    by_row = {}
    for r in runs:
        by_row.setdefault(r[0], []).append(r)
    for (y, a, b, G) in runs:
        for (_, c, d, H) in by_row.get(y - 1, []):
            if c <= b + 1 and a <= d + 1:
                ra, rb = find(G), find(H)
                if ra != rb:
                    par[max(ra, rb)] = min(ra, rb)
    lab = np.zeros(mask.shape, np.int64) - 1
    for (y, a, b, G) in runs:
        lab[y, a:b + 1] = find(G)
    return lab


@pytest.mark.parametrize("seed,shape,dens", [(0, (70, 90), 0.3), (1, (64, 64), 0.45), (2, (131, 67), 0.55),
                                             (3, (33, 129), 0.2), (4, (1, 50), 0.5), (5, (50, 1), 0.5)])
def test_run_labelling_matches_scipy_and_root_is_opencv_first(seed, shape, dens):
    rng = np.random.default_rng(seed)
    mask = rng.random(shape) < dens
    h, w = shape
    wb = (w + 1) // 2
    lab = label_runs(mask)
    ref, n = ndimage.label(mask, structure=np.ones((3, 3), int))
    # same partition
    assert n == len(np.unique(lab[lab >= 0]))
    for k in range(1, n + 1):
        roots = np.unique(lab[ref == k])
        assert len(roots) == 1
        ys, xs = np.nonzero(ref == k)
        # the min block-raster pixel is a run start, and its G is the root
        i = np.argmin(block_raster_key(xs, ys, wb))
        assert run_starts(mask)[ys[i], xs[i]]
        assert roots[0] == gidx(xs[i], ys[i], wb)


def test_run_start_index_is_unique_and_ordered():
    rng = np.random.default_rng(7)
    mask = rng.random((97, 83)) < 0.5
    wb = (83 + 1) // 2
    ys, xs = np.nonzero(run_starts(mask))
    G = gidx(xs, ys, wb)
    assert len(np.unique(G)) == len(G)
    order_g = np.argsort(G, kind="stable")
    order_b = np.argsort(block_raster_key(xs, ys, wb), kind="stable")
    assert np.array_equal(order_g, order_b)


def test_closed_key_orders_by_area_then_smaller_root_and_round_trips():
    rng = np.random.default_rng(3)
    keys = []
    for _ in range(500):
        area = int(rng.integers(1, 4097))
        G = int(rng.integers(0, 1 << 23))
        bx0, by0 = (int(v) for v in rng.integers(0, 64, 2))
        bx1, by1 = bx0 + int(rng.integers(1, 65 - bx0)), by0 + int(rng.integers(1, 65 - by0))
        k = closed_key(area, G, bx0, by0, bx1, by1)
        assert decode_closed(k) == (area, G, bx0, by0, bx1, by1)
        keys.append((k, area, G))
    best = max(keys)
    ref = max(keys, key=lambda t: (t[1], -t[2]))
    assert best == ref


def test_closed_components_never_touch_a_tile_edge():
    """A component with no pixel on a 64×64 tile's edge rows/columns lies in
    one tile and is final there (no border union can reach it)."""
    rng = np.random.default_rng(11)
    mask = rng.random((200, 190)) < 0.3
    ref, n = ndimage.label(mask, structure=np.ones((3, 3), int))
    edge = np.zeros(mask.shape, bool)
    edge[::TH, :] = edge[TH - 1::TH, :] = True
    edge[:, ::TW] = edge[:, TW - 1::TW] = True
    for k in range(1, n + 1):
        ys, xs = np.nonzero(ref == k)
        if not edge[ys, xs].any():
            assert len(np.unique(ys // TH)) == 1 and len(np.unique(xs // TW)) == 1
