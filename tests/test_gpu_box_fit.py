"""KLT box propagation (tbdk_box_propagate) vs the getRTMatrix restatement
(oracle/box_fit_oracle.py).  The fit sums are the reference's own arithmetic;
the reference solves the 4x4 normal system by Jacobi eigen-decomposition, the
kernel in closed form, so the two agree to double rounding scaled by the
system's condition number: |dM| <= 64 * eps * cond(A) * max(1, |M|), the
propagated centre within 1e-4 px (far below the 0.5 px that could move the
track's rounded box), identical point counts and validity."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import box_fit_oracle as BF  # noqa: E402

pytestmark = pytest.mark.gpu

def run(gpu, prev, nxt, status, offsets, boxes, min_points):
    from opencv_amd import klt

    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    return klt.box_propagate(d(prev), d(nxt), None if status is None else d(status.astype(np.uint8)),
                             d(offsets.astype(np.int32)), d(np.asarray(boxes, np.int32).reshape(-1, 4)),
                             min_points, ctx=gpu)


def make_case(rng, nboxes, max_pts):
    prev, nxt, st, offs, boxes, truth = [], [], [], [0], [], []
    for _ in range(nboxes):
        n = int(rng.integers(0, max_pts + 1))
        x, y = rng.uniform(0, 1700), rng.uniform(0, 900)
        w, h = int(rng.integers(20, 220)), int(rng.integers(20, 220))
        a = np.stack([rng.uniform(x, x + w, n), rng.uniform(y, y + h, n)], 1).astype(np.float32)
        ang, s = rng.uniform(-0.05, 0.05), rng.uniform(0.9, 1.1)
        R = s * np.array([[np.cos(ang), -np.sin(ang)], [np.sin(ang), np.cos(ang)]])
        t = rng.uniform(-8, 8, 2)
        b = (a @ R.T + t + rng.normal(0, 0.3, (n, 2))).astype(np.float32)
        prev.append(a)
        nxt.append(b)
        st.append((rng.random(n) > 0.15).astype(np.uint8))
        offs.append(offs[-1] + n)
        boxes.append((int(x), int(y), w, h))
        truth.append((R, t))
    cat = lambda L: np.concatenate(L) if L else np.zeros((0, 2), np.float32)  # noqa: E731
    return cat(prev), cat(nxt), np.concatenate(st), np.array(offs), boxes


@pytest.mark.parametrize("seed,nboxes,max_pts", [(1, 128, 256), (2, 40, 600), (3, 16, 5)])
def test_box_propagate_matches_getrtmatrix(gpu, seed, nboxes, max_pts):
    rng = np.random.default_rng(seed)
    prev, nxt, st, offs, boxes = make_case(rng, nboxes, max_pts)
    min_points = 4
    got = run(gpu, prev, nxt, st, offs, boxes, min_points)
    for i, box in enumerate(boxes):
        sel = st[offs[i]:offs[i + 1]] != 0
        a, b = prev[offs[i]:offs[i + 1]][sel], nxt[offs[i]:offs[i + 1]][sel]
        assert got["npoints"][i] == len(a)
        if len(a) < 2:
            continue
        M = BF.get_rt_matrix(a, b)
        cx, cy = BF.propagate_box(M, box)
        scale = np.hypot(M[0, 0], M[1, 0])
        want_valid = len(a) >= min_points and 0.5 < scale < 2.0
        assert bool(got["valid"][i]) == want_valid, (i, len(a), scale)
        gm = got["m"][i].reshape(2, 3)
        sa, _ = BF.rt_sums(a, b)
        tol = 64 * np.finfo(np.float64).eps * np.linalg.cond(sa)
        assert np.all(np.abs(gm - M) <= tol * np.maximum(1.0, np.abs(M))), (i, gm - M, tol)
        assert abs(got["cx"][i] - cx) <= 1e-4 and abs(got["cy"][i] - cy) <= 1e-4


def test_box_propagate_exact_similarity_and_degenerate(gpu):
    # exact similarity on integer-valued points: recovered to rounding; degenerate sets invalid
    a = np.array([[10, 10], [50, 12], [30, 60], [70, 70], [15, 45]], np.float32)
    R = np.array([[1.0, -0.0], [0.0, 1.0]])
    b = (a @ R.T + [3, -2]).astype(np.float32)
    same = np.repeat(a[:1], 5, 0)
    prev = np.concatenate([a, same])
    nxt = np.concatenate([b, same + 1])
    got = run(gpu, prev, nxt, None, np.array([0, 5, 10]), [(10, 10, 60, 60), (0, 0, 10, 10)], 4)
    assert got["valid"][0] == 1 and np.allclose(got["m"][0], [1, 0, 3, 0, 1, -2], atol=1e-9)
    assert abs(got["cx"][0] - 43.0) < 1e-9 and abs(got["cy"][0] - 38.0) < 1e-9
    assert got["valid"][1] == 0 and got["npoints"][1] == 5  # all points identical: singular
