"""box_fit_oracle.py — restatement of the 4-DOF similarity fit the KLT box
propagation uses: the non-full-affine branch of getRTMatrix
(modules/video/src/lkpyramid.cpp:1398-1470) solved like the reference, with
cv::solve(DECOMP_EIG) = Jacobi eigen-decomposition + SVBkSb back-substitution
dropping eigenvalues <= 2*DBL_EPSILON*sum(w) (core/src/lapack.cpp:663-760,
1330-1362).  TEST INFRASTRUCTURE ONLY.

The sums reproduce the reference's arithmetic exactly (Point2f products and
sums in float32, accumulated into double in point order); the eigen solve is
numpy's (LAPACK), which agrees with Jacobi to double rounding, so parity for
the fit is stated as a tolerance (tests/test_gpu_box_fit.py)."""
import numpy as np


def rt_sums(a: np.ndarray, b: np.ndarray):
    """sa (4x4) and sb (4) of getRTMatrix (:1441-1461) for float32 pairs a -> b."""
    a = np.asarray(a, np.float32).reshape(-1, 2)
    b = np.asarray(b, np.float32).reshape(-1, 2)
    ax, ay, bx, by = a[:, 0], a[:, 1], b[:, 0], b[:, 1]

    def seq(v):  # float terms promoted to double and added in point order (np.cumsum is sequential)
        v = np.asarray(v).astype(np.float64)
        return float(np.cumsum(v)[-1]) if len(v) else 0.0

    # each product and the float add / subtract round to float32 (numpy applies
    # one ufunc per operator, never a fused multiply-add)
    s00 = seq(ax * ax + ay * ay)
    s02, s03 = seq(ax), seq(ay)
    b0 = seq(ax * bx + ay * by)
    b1 = seq(ax * by - ay * bx)
    b2, b3 = seq(bx), seq(by)
    n = float(len(a))
    sa = np.array([[s00, 0.0, s02, s03],
                   [0.0, s00, -s03, s02],
                   [s02, -s03, n, 0.0],
                   [s03, s02, 0.0, n]])
    return sa, np.array([b0, b1, b2, b3])


def solve_eig(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    w, v = np.linalg.eigh(A)
    thr = 2 * np.finfo(np.float64).eps * w.sum()
    x = np.zeros(4)
    for i in range(4):
        if abs(w[i]) <= thr:
            continue
        x += (v[:, i] @ B) / w[i] * v[:, i]
    return x


def get_rt_matrix(a, b) -> np.ndarray:
    """2x3 [m0 -m1 m2; m1 m0 m3] of getRTMatrix(fullAffine=false)."""
    sa, sb = rt_sums(a, b)
    m = solve_eig(sa, sb)
    return np.array([[m[0], -m[1], m[2]], [m[1], m[0], m[3]]])


def propagate_box(M: np.ndarray, box) -> tuple[float, float]:
    x, y, w, h = box
    cx0, cy0 = float(x + w // 2), float(y + h // 2)
    return M[0, 0] * cx0 + M[0, 1] * cy0 + M[0, 2], M[1, 0] * cx0 + M[1, 1] * cy0 + M[1, 2]
