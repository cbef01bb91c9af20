"""ctypes binding of oracle/liboracle.so — the CPU checker (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
# TBDK_ORACLE_LIB: another build of the same sources (bench.py's CPU baseline
# builds one with -O3 -march=native on the host it runs on)
ORACLE_LIB = os.environ.get("TBDK_ORACLE_LIB") or os.path.join(ORACLE_DIR, "liboracle.so")

ACCUM_SSE2 = 0
ACCUM_EXACT = 1
MAX_LEVELS = 8


class Plane(C.Structure):
    _fields_ = [("data", C.c_void_p), ("w", C.c_int), ("h", C.c_int), ("pitch", C.c_int), ("pad", C.c_int),
                ("cn", C.c_int)]


class OPyr(C.Structure):
    _fields_ = [("nlevels", C.c_int), ("lv", Plane * MAX_LEVELS)]


class LkParams(C.Structure):
    _fields_ = [
        ("winW", C.c_int), ("winH", C.c_int), ("maxLevel", C.c_int), ("maxCount", C.c_int),
        ("epsilon", C.c_double), ("flags", C.c_int), ("minEigThreshold", C.c_float), ("accum", C.c_int),
        ("nthreads", C.c_int),
    ]


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(ORACLE_LIB):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
    lib = C.CDLL(ORACLE_LIB)
    lib.orc_build_pyramid.restype = C.c_int
    lib.orc_build_pyramid.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                      C.POINTER(OPyr)]
    lib.orc_build_pyramid_cn.restype = C.c_int
    lib.orc_build_pyramid_cn.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                         C.c_int, C.POINTER(OPyr)]
    lib.orc_scharr_cn.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int]
    lib.orc_free_pyramid.argtypes = [C.POINTER(OPyr)]
    lib.orc_pyr_down.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int]
    lib.orc_scharr.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int]
    lib.orc_lk.restype = C.c_int
    lib.orc_lk.argtypes = [C.POINTER(OPyr), C.POINTER(OPyr), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                           C.POINTER(LkParams), C.c_void_p]
    lib.orc_lk_gate.restype = C.c_int
    lib.orc_lk_gate.argtypes = [C.POINTER(OPyr), C.POINTER(OPyr), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                C.c_int, C.POINTER(LkParams), C.c_void_p, C.c_void_p]
    lib.orc_synth_frames.restype = C.c_int
    lib.orc_synth_frames.argtypes = [C.c_uint32, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                     C.c_void_p]
    lib.orc_reflect101.restype = C.c_int
    lib.orc_reflect101.argtypes = [C.c_int, C.c_int]
    lib.orc_now.restype = C.c_double
    _lib = lib
    return lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class Pyramid:
    """Oracle pyramid (host memory), freed on GC."""

    def __init__(self, img: np.ndarray, win=(21, 21), max_level=3, pad=32):
        """img: (H, W) u8, or (H, W, cn) interleaved channels"""
        lib = load()
        img = np.ascontiguousarray(img, dtype=np.uint8)
        self.cn = 1 if img.ndim == 2 else img.shape[2]
        self.p = OPyr()
        lib.orc_build_pyramid_cn(_ptr(img), img.shape[1], img.shape[0], img.strides[0], self.cn, win[0], win[1],
                                 max_level, pad, C.byref(self.p))
        self.nlevels = self.p.nlevels

    def level(self, i: int, with_border=False) -> np.ndarray:
        L = self.p.lv[i]
        cn = self.cn
        full = np.ctypeslib.as_array(C.cast(L.data, C.POINTER(C.c_uint8)), shape=(L.h + 2 * L.pad, L.pitch)).copy()
        if with_border:
            out = full[:, :(L.w + 2 * L.pad) * cn]
        else:
            out = full[L.pad:L.pad + L.h, L.pad * cn:(L.pad + L.w) * cn]
        return out if cn == 1 else out.reshape(out.shape[0], -1, cn)

    def __del__(self):
        if _lib is not None and getattr(self, "p", None) is not None:
            _lib.orc_free_pyramid(C.byref(self.p))
            self.p = None


def pyr_down(img: np.ndarray) -> np.ndarray:
    lib = load()
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    out = np.empty(((h + 1) // 2, (w + 1) // 2), dtype=np.uint8)
    lib.orc_pyr_down(_ptr(img), w, h, img.strides[0], _ptr(out), out.shape[1], out.shape[0], out.strides[0])
    return out


def scharr(img: np.ndarray) -> np.ndarray:
    """calcSharrDeriv: (H, W, 2) int16 for (H, W) u8; (H, W, 2cn) for (H, W, cn)"""
    lib = load()
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape[:2]
    cn = 1 if img.ndim == 2 else img.shape[2]
    out = np.empty((h, w, 2 * cn), dtype=np.int16)
    lib.orc_scharr_cn(_ptr(img), w, h, img.strides[0], cn, _ptr(out), 2 * cn * w)
    return out


def lk(prev: Pyramid, nxt: Pyramid, pts: np.ndarray, win=(21, 21), max_level=3, max_count=30, eps=0.01, flags=0,
       min_eig=1e-4, accum=ACCUM_SSE2, nthreads=8, init: np.ndarray | None = None, want_err: bool = True,
       gate: np.ndarray | None = None):
    """calcOpticalFlowPyrLK; want_err=False passes err = noArray(), which also
    skips the level-0 error pass and its bounds check (lkpyramid.cpp:654-693).
    gate: optional float32 (n,) out, per point the smallest relative margin
    |v - thr| / |thr| of any minEig / determinant / bounds gate evaluated
    (orc_lk_gate; SURVEY.md §8(c)'s threshold clause)."""
    lib = load()
    pts = np.ascontiguousarray(pts, dtype=np.float32).reshape(-1, 2)
    n = pts.shape[0]
    nxt_pts = np.zeros((n, 2), dtype=np.float32) if init is None else np.ascontiguousarray(init, np.float32).copy()
    status = np.zeros(n, dtype=np.uint8)
    err = np.zeros(n, dtype=np.float32)
    iters = np.zeros(n, dtype=np.int32)
    prm = LkParams(win[0], win[1], max_level, max_count, eps, flags, min_eig, accum, nthreads)
    if n:
        if gate is not None:
            assert gate.dtype == np.float32 and gate.flags.c_contiguous and gate.shape == (n,)
            lib.orc_lk_gate(C.byref(prev.p), C.byref(nxt.p), _ptr(pts), _ptr(nxt_pts), _ptr(status),
                            _ptr(err) if want_err else None, n, C.byref(prm), _ptr(iters), _ptr(gate))
        else:
            lib.orc_lk(C.byref(prev.p), C.byref(nxt.p), _ptr(pts), _ptr(nxt_pts), _ptr(status),
                       _ptr(err) if want_err else None, n, C.byref(prm), _ptr(iters))
    return nxt_pts, status, err, iters


# ---- the fp16 pixel path (oracle/klt16_oracle.c) ------------------------------

class Level16(C.Structure):
    _fields_ = [("px", C.c_void_p), ("d", C.c_void_p), ("w", C.c_int), ("h", C.c_int), ("f32", C.c_int),
                ("cn", C.c_int)]


class OPyr16(C.Structure):
    _fields_ = [("nlevels", C.c_int), ("lv", Level16 * MAX_LEVELS)]


def _lib16():
    lib = load()
    if not getattr(lib, "_f16_ready", False):
        lib.orc16_pyr_down.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int]
        lib.orc16_scharr.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
        lib.orc32_pyr_down.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int]
        lib.orc32_scharr.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
        lib.orc32_pyr_down_cn.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int,
                                          C.c_int]
        lib.orc32_scharr_cn.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
        lib.orc16_lk.restype = C.c_int
        lib.orc16_lk.argtypes = [C.POINTER(OPyr16), C.POINTER(OPyr16), C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_void_p, C.c_int, C.POINTER(LkParams), C.c_void_p]
        lib._f16_ready = True
    return lib


def pyr_down16(img: np.ndarray) -> np.ndarray:
    """pyrDown_<FltCast<float,8>> scalar order in fp32, rounded to fp16 (float16 in / out)."""
    lib = _lib16()
    img = np.ascontiguousarray(img, dtype=np.float16)
    h, w = img.shape
    out = np.empty(((h + 1) // 2, (w + 1) // 2), dtype=np.float16)
    lib.orc16_pyr_down(_ptr(img), w, h, w, _ptr(out), out.shape[1], out.shape[0], out.shape[1])
    return out


def scharr16(img: np.ndarray) -> np.ndarray:
    """calcSharrDeriv's formula in fp32 on an fp16 level: (H, W, 2) float16 (Ix, Iy)."""
    lib = _lib16()
    img = np.ascontiguousarray(img, dtype=np.float16)
    h, w = img.shape
    out = np.empty((h, w, 2), dtype=np.float16)
    lib.orc16_scharr(_ptr(img), w, h, w, _ptr(out))
    return out


def pyr_down32(img: np.ndarray) -> np.ndarray:
    """the fp32 pixel path's pyrDown (pyr_down16's order, no rounding); (H, W)
    or (H, W, cn) interleaved channels, each filtered on its own."""
    lib = _lib16()
    img = np.ascontiguousarray(img, dtype=np.float32)
    h, w = img.shape[:2]
    cn = 1 if img.ndim == 2 else img.shape[2]
    out = np.empty(((h + 1) // 2, (w + 1) // 2) + img.shape[2:], dtype=np.float32)
    lib.orc32_pyr_down_cn(_ptr(img), w, h, w * cn, cn, _ptr(out), out.shape[1], out.shape[0], out.shape[1] * cn)
    return out


def scharr32(img: np.ndarray) -> np.ndarray:
    """calcSharrDeriv's formula in fp32 on an fp32 level: (H, W, 2) float32 (Ix, Iy);
    (H, W, cn) interleaved channels -> (H, W, 2 cn), (Ix_c, Iy_c) per channel."""
    lib = _lib16()
    img = np.ascontiguousarray(img, dtype=np.float32)
    h, w = img.shape[:2]
    cn = 1 if img.ndim == 2 else img.shape[2]
    out = np.empty((h, w, 2 * cn), dtype=np.float32)
    lib.orc32_scharr_cn(_ptr(img), w, h, w * cn, cn, _ptr(out))
    return out


class Pyramid16:
    """fp16 oracle pyramid: levels (float16) and their fp16 derivative planes;
    the level rule of cv::buildOpticalFlowPyramid (lkpyramid.cpp:782-787).
    f32=True: the fp32 pixel path (float32 levels and derivative pairs; a
    uint8 / uint16 / float32 frame converts exactly); an (H, W, cn) frame
    (f32 only) gives interleaved cn-channel levels."""

    def __init__(self, img: np.ndarray, win=(21, 21), max_level=3, f32: bool = False):
        dt = np.float32 if f32 else np.float16
        l0 = np.ascontiguousarray(img.astype(dt) if img.dtype != dt else img)
        down, sch = (pyr_down32, scharr32) if f32 else (pyr_down16, scharr16)
        self.levels = [l0]
        w, h = l0.shape[1], l0.shape[0]
        for _ in range(max_level):
            w, h = (w + 1) // 2, (h + 1) // 2
            if w <= win[0] or h <= win[1]:
                break
            self.levels.append(down(self.levels[-1]))
        self.derivs = [sch(L) for L in self.levels]
        self.nlevels = len(self.levels)
        self.cn = 1 if l0.ndim == 2 else l0.shape[2]
        assert self.cn == 1 or f32, "multi-channel frames: the fp32 pixel path only"
        self.p = OPyr16()
        self.p.nlevels = self.nlevels
        for i, (L, D) in enumerate(zip(self.levels, self.derivs)):
            self.p.lv[i] = Level16(L.ctypes.data, D.ctypes.data, L.shape[1], L.shape[0], int(f32), self.cn)


def lk16(prev: Pyramid16, nxt: Pyramid16, pts: np.ndarray, win=(21, 21), max_level=3, max_count=30, eps=0.01,
         flags=0, min_eig=1e-4, nthreads=8, init: np.ndarray | None = None, want_err: bool = True):
    """sparse LK of the fp16 pixel path (bit-exact definition of klt_f16.hip)."""
    lib = _lib16()
    pts = np.ascontiguousarray(pts, dtype=np.float32).reshape(-1, 2)
    n = pts.shape[0]
    nxt_pts = np.zeros((n, 2), dtype=np.float32) if init is None else np.ascontiguousarray(init, np.float32).copy()
    status = np.zeros(n, dtype=np.uint8)
    err = np.zeros(n, dtype=np.float32)
    iters = np.zeros(n, dtype=np.int32)
    prm = LkParams(win[0], win[1], max_level, max_count, eps, flags, min_eig, ACCUM_EXACT, nthreads)
    if n:
        rc = lib.orc16_lk(C.byref(prev.p), C.byref(nxt.p), _ptr(pts), _ptr(nxt_pts), _ptr(status),
                          _ptr(err) if want_err else None, n, C.byref(prm), _ptr(iters))
        assert rc == 0, rc
    return nxt_pts, status, err, iters


def synth(seed: int, W: int, H: int, nobj: int, t0: int, nframes: int):
    lib = load()
    out = np.zeros((nframes, H, W), dtype=np.uint8)
    gt = np.zeros((nframes, max(nobj, 1), 5), dtype=np.int32)
    rc = lib.orc_synth_frames(seed, W, H, nobj, t0, nframes, _ptr(out), W, _ptr(gt))
    assert rc == 0
    return out, gt[:, :nobj]


def synth_gt(seed: int, W: int, H: int, nobj: int, t0: int, nframes: int):
    """the sequence's ground-truth boxes (nframes, nobj, 5) without rendering frames"""
    lib = load()
    gt = np.zeros((nframes, max(nobj, 1), 5), dtype=np.int32)
    rc = lib.orc_synth_frames(seed, W, H, nobj, t0, nframes, None, W, _ptr(gt))
    assert rc == 0
    return gt[:, :nobj]


def read_png_gray(path: str) -> np.ndarray:
    """Minimal PNG decoder (8-bit gray / RGB / RGBA, non-interlaced) -> uint8 gray.

    Gray conversion (RGB) uses cv::cvtColor's integer BGR2GRAY weights
    (R*4899 + G*9617 + B*1868 + 8192) >> 14 (imgproc/src/color_rgb.simd.hpp).
    """
    import struct
    import zlib

    with open(path, "rb") as f:
        data = f.read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n", "not a PNG"
    pos, idat, hdr = 8, b"", None
    while pos < len(data):
        ln, = struct.unpack(">I", data[pos:pos + 4])
        typ = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + ln]
        if typ == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", body)
        elif typ == b"IDAT":
            idat += body
        elif typ == b"IEND":
            break
        pos += 12 + ln
    w, h, depth, ctype, _, _, interlace = hdr
    assert depth == 8 and interlace == 0, "unsupported PNG"
    ch = {0: 1, 2: 3, 4: 2, 6: 4}[ctype]
    raw = zlib.decompress(idat)
    stride = w * ch
    out = np.zeros((h, stride), dtype=np.int32)
    prev = np.zeros(stride, dtype=np.int32)
    p = 0
    for y in range(h):
        ft = raw[p]
        line = np.frombuffer(raw[p + 1:p + 1 + stride], dtype=np.uint8).astype(np.int32)
        p += 1 + stride
        cur = np.zeros(stride, dtype=np.int32)
        if ft == 0:
            cur = line
        elif ft == 1:
            for x in range(stride):
                cur[x] = (line[x] + (cur[x - ch] if x >= ch else 0)) & 255
        elif ft == 2:
            cur = (line + prev) & 255
        elif ft == 3:
            for x in range(stride):
                cur[x] = (line[x] + (((cur[x - ch] if x >= ch else 0) + prev[x]) >> 1)) & 255
        elif ft == 4:
            for x in range(stride):
                a = cur[x - ch] if x >= ch else 0
                b = prev[x]
                c = prev[x - ch] if x >= ch else 0
                pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
                pr = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
                cur[x] = (line[x] + pr) & 255
        out[y] = cur
        prev = cur
    img = out.reshape(h, w, ch)
    if ch == 1:
        return img[:, :, 0].astype(np.uint8)
    if ch == 2:
        return img[:, :, 0].astype(np.uint8)
    r, g, b = img[:, :, 0], img[:, :, 1], img[:, :, 2]
    return ((r * 4899 + g * 9617 + b * 1868 + 8192) >> 14).astype(np.uint8)


def gftt(img: np.ndarray, max_corners=1000, quality=0.01, min_distance=0.0) -> np.ndarray:
    lib = load()
    lib.orc_gftt.restype = C.c_int
    lib.orc_gftt.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, C.c_void_p]
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    out = np.zeros((max(max_corners, 1), 2), dtype=np.float32)
    n = lib.orc_gftt(_ptr(img), w, h, img.strides[0], max_corners, quality, min_distance, _ptr(out))
    return out[:n]


def min_eig(img: np.ndarray) -> np.ndarray:
    lib = load()
    lib.orc_min_eig.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    out = np.zeros((h, w), dtype=np.float32)
    lib.orc_min_eig(_ptr(img), w, h, img.strides[0], _ptr(out))
    return out


def gftt_ex(img: np.ndarray, max_corners=1000, quality=0.01, min_distance=0.0, block=3, harris=False,
            k=0.04) -> np.ndarray:
    """goodFeaturesToTrack with blockSize / useHarrisDetector / harrisK"""
    lib = load()
    lib.orc_gftt_ex.restype = C.c_int
    lib.orc_gftt_ex.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, C.c_int,
                                C.c_int, C.c_double, C.c_void_p]
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    out = np.zeros((max(max_corners, 1), 2), dtype=np.float32)
    n = lib.orc_gftt_ex(_ptr(img), w, h, img.strides[0], max_corners, quality, min_distance, block, int(harris), k,
                        _ptr(out))
    return out[:n]


def corner_response(img: np.ndarray, block=3, harris=False, k=0.04) -> np.ndarray:
    """cornerMinEigenVal / cornerHarris (ksize 3) of an isolated u8 image"""
    lib = load()
    lib.orc_corner_response.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double,
                                        C.c_void_p]
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    out = np.zeros((h, w), dtype=np.float32)
    lib.orc_corner_response(_ptr(img), w, h, img.strides[0], block, int(harris), k, _ptr(out))
    return out


def gftt_rois(frame: np.ndarray, rois, max_corners=256, quality=0.01, min_distance=3.0, block=3, harris=False,
              k=0.04):
    """Per-ROI goodFeaturesToTrack on isolated ROIs; corners in frame coordinates."""
    res = []
    for (x, y, w, h) in rois:
        c = gftt_ex(frame[y:y + h, x:x + w], max_corners, quality, min_distance, block, harris, k)
        res.append(c + np.float32([x, y]))
    return res


# border modes / flags (reference values: core/base.hpp, imgproc.hpp)
BORDER_CONSTANT, BORDER_REPLICATE, BORDER_REFLECT, BORDER_WRAP, BORDER_REFLECT_101, BORDER_TRANSPARENT = range(6)
INTER_NEAREST, INTER_LINEAR, INTER_CUBIC, INTER_AREA = 0, 1, 2, 3
WARP_INVERSE_MAP = 16


def warp_affine(src: np.ndarray, M, dsize, flags=INTER_LINEAR, border=BORDER_CONSTANT, bval=0,
                dst: np.ndarray | None = None) -> np.ndarray:
    """cv::warpAffine for CV_8UC1 (oracle/warp_oracle.c). dsize = (width, height).
    `dst` (optional) supplies the initial contents (BORDER_TRANSPARENT keeps them)."""
    lib = load()
    lib.orc_warp_affine_u8.restype = C.c_int
    lib.orc_warp_affine_u8.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                       C.c_void_p, C.c_int, C.c_int, C.c_int]
    src = np.ascontiguousarray(src, dtype=np.uint8)
    sh, sw = src.shape
    dw, dh = dsize
    out = np.zeros((dh, dw), np.uint8) if dst is None else np.ascontiguousarray(dst, dtype=np.uint8).copy()
    m = np.ascontiguousarray(np.asarray(M, np.float64).reshape(6))
    rc = lib.orc_warp_affine_u8(_ptr(src), sw, sh, src.strides[0], _ptr(out), dw, dh, out.strides[0], _ptr(m),
                                flags, border, bval)
    if rc != 0:
        raise ValueError("unsupported warpAffine mode")
    return out


def invert_affine(M) -> np.ndarray:
    lib = load()
    lib.orc_invert_affine.argtypes = [C.c_void_p, C.c_void_p]
    m = np.ascontiguousarray(np.asarray(M, np.float64).reshape(6))
    out = np.zeros(6, np.float64)
    lib.orc_invert_affine(_ptr(m), _ptr(out))
    return out.reshape(2, 3)


# ---- dense Farneback (oracle/farneback_oracle.c) ----
FARNEBACK_GAUSSIAN = 256
OPTFLOW_USE_INITIAL_FLOW = 4
OPTFLOW_LK_GET_MIN_EIGENVALS = 8


def _fb_lib():
    lib = load()
    lib.orc_fb_calc.restype = C.c_int
    lib.orc_fb_calc.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_double,
                                C.c_int, C.c_int, C.c_int, C.c_double, C.c_int]
    lib.orc_fb_calc_mode.restype = C.c_int
    lib.orc_fb_calc_mode.argtypes = lib.orc_fb_calc.argtypes + [C.c_int]
    lib.orc_fb_gauss_blur.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_double]
    lib.orc_fb_resize_linear.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int]
    lib.orc_fb_poly_exp.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_double, C.c_void_p]
    lib.orc_fb_gaussian_kernel.argtypes = [C.c_int, C.c_double, C.c_void_p]
    lib.orc_fb_resize_area_fx.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int,
                                          C.c_double, C.c_double]
    return lib


def resize_area(src: np.ndarray, size, inv_scale=None) -> np.ndarray:
    """resize(src, size, INTER_AREA) of a float (H, W) or (H, W, cn) image;
    inv_scale=(fx, fy) when the reference call passes fx/fy instead of a size."""
    lib = _fb_lib()
    s = np.ascontiguousarray(src, dtype=np.float32)
    h, w = s.shape[:2]
    cn = 1 if s.ndim == 2 else s.shape[2]
    dw, dh = size
    fx, fy = inv_scale if inv_scale is not None else (dw / w, dh / h)
    out = np.empty((dh, dw) + s.shape[2:], np.float32)
    lib.orc_fb_resize_area_fx(_ptr(s), w, h, cn, _ptr(out), dw, dh, float(fx), float(fy))
    return out


def fb_level_image(img: np.ndarray, size, smooth_size: int, sigma: float) -> np.ndarray:
    """resize(GaussianBlur(float(img), ksize, sigma), size, INTER_LINEAR) (optflowgf.cpp:1170-1172)."""
    lib = _fb_lib()
    f = np.ascontiguousarray(img, dtype=np.float32)
    h, w = f.shape
    blur = np.empty_like(f)
    lib.orc_fb_gauss_blur(_ptr(f), w, h, _ptr(blur), int(smooth_size), float(sigma))
    dw, dh = size
    if (dw, dh) == (w, h):
        return blur
    out = np.empty((dh, dw), np.float32)
    lib.orc_fb_resize_linear(_ptr(blur), w, h, 1, _ptr(out), dw, dh)
    return out


def fb_poly_exp(src: np.ndarray, n: int, sigma: float) -> np.ndarray:
    """FarnebackPolyExp -> (H, W, 5) float32."""
    lib = _fb_lib()
    s = np.ascontiguousarray(src, dtype=np.float32)
    h, w = s.shape
    out = np.empty((h, w, 5), np.float32)
    lib.orc_fb_poly_exp(_ptr(s), w, h, int(n), float(sigma), _ptr(out))
    return out


def gaussian_kernel(n: int, sigma: float) -> np.ndarray:
    lib = _fb_lib()
    out = np.empty(n, np.float32)
    lib.orc_fb_gaussian_kernel(int(n), float(sigma), _ptr(out))
    return out


def farneback(prev: np.ndarray, nxt: np.ndarray, pyr_scale=0.5, levels=5, winsize=13, iterations=10, poly_n=5,
              poly_sigma=1.1, flags=0, box_direct=False, init_flow: np.ndarray | None = None) -> np.ndarray:
    """cv::calcOpticalFlowFarneback -> (H, W, 2) float32.  box_direct: exact-order
    box window sums (the GPU's order) instead of the reference's running sums."""
    lib = _fb_lib()
    a = np.ascontiguousarray(prev, dtype=np.uint8)
    b = np.ascontiguousarray(nxt, dtype=np.uint8)
    h, w = a.shape
    flow = np.zeros((h, w, 2), np.float32) if init_flow is None else np.ascontiguousarray(init_flow, np.float32).copy()
    rc = lib.orc_fb_calc_mode(_ptr(a), _ptr(b), w, h, a.strides[0], _ptr(flow), int(levels), float(pyr_scale),
                              int(winsize), int(iterations), int(poly_n), float(poly_sigma), int(flags),
                              int(bool(box_direct)))
    if rc != 0:
        raise ValueError("unsupported Farneback arguments")
    return flow


# ---- HOG people detector (oracle/hog_oracle.c) ----
class HogParams(C.Structure):
    _fields_ = [("win_w", C.c_int), ("win_h", C.c_int), ("block_w", C.c_int), ("block_h", C.c_int),
                ("bstride_x", C.c_int), ("bstride_y", C.c_int), ("cell_w", C.c_int), ("cell_h", C.c_int),
                ("nbins", C.c_int), ("win_sigma", C.c_double), ("l2hys", C.c_double), ("gamma", C.c_int),
                ("signed_grad", C.c_int), ("wstride_x", C.c_int), ("wstride_y", C.c_int)]


def hog_params(win=(64, 128), block=(16, 16), bstride=(8, 8), cell=(8, 8), nbins=9, win_sigma=-1.0, l2hys=0.2,
               gamma=True, signed=False, wstride=(8, 8)) -> HogParams:
    return HogParams(win[0], win[1], block[0], block[1], bstride[0], bstride[1], cell[0], cell[1], nbins,
                     win_sigma, l2hys, int(gamma), int(signed), wstride[0], wstride[1])


def _hog_lib():
    lib = load()
    P = C.POINTER(HogParams)
    lib.orc_hog_resize_exact.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                         C.c_int, C.c_int]
    lib.orc_hog_gradient.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                     C.c_void_p, C.c_void_p]
    lib.orc_hog_blocks.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, P, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.orc_hog_detect.restype = C.c_int
    lib.orc_hog_detect.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, P, C.c_void_p, C.c_int,
                                   C.c_double, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.orc_hog_group.restype = C.c_int
    lib.orc_hog_group.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_int, C.c_int]
    lib.orc_hog_detect_multiscale.restype = C.c_int
    lib.orc_hog_detect_multiscale.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, P, C.c_void_p,
                                              C.c_int, C.c_double, C.c_int, C.c_double, C.c_int, C.c_void_p,
                                              C.c_void_p, C.c_int]
    return lib


def _img(img):
    a = np.ascontiguousarray(img, dtype=np.uint8)
    cn = 1 if a.ndim == 2 else a.shape[2]
    return a, a.shape[1], a.shape[0], a.strides[0], cn


def hog_resize(img: np.ndarray, size) -> np.ndarray:
    """resize(img, size, 0, 0, INTER_LINEAR_EXACT) of a u8 image."""
    a, w, h, pitch, cn = _img(img)
    dw, dh = size
    out = np.empty((dh, dw) + a.shape[2:], np.uint8)
    _hog_lib().orc_hog_resize_exact(_ptr(a), w, h, pitch, cn, _ptr(out), dw, dh, out.strides[0])
    return out


def hog_gradient(img: np.ndarray, nbins=9, gamma=True, signed=False):
    """HOGDescriptor::computeGradient -> (grad (H, W, 2) f32, qangle (H, W, 2) u8)."""
    a, w, h, pitch, cn = _img(img)
    grad = np.empty((h, w, 2), np.float32)
    qa = np.empty((h, w, 2), np.uint8)
    _hog_lib().orc_hog_gradient(_ptr(a), w, h, pitch, cn, nbins, int(gamma), int(signed), _ptr(grad), _ptr(qa))
    return grad, qa


def hog_blocks(grad: np.ndarray, qangle: np.ndarray, prm: HogParams) -> np.ndarray:
    """Normalized block histograms on the cache grid -> (nby, nbx, block_hist_size)."""
    h, w = grad.shape[:2]
    csx, csy = np.gcd(prm.wstride_x, prm.bstride_x), np.gcd(prm.wstride_y, prm.bstride_y)
    nbx, nby = (w - prm.block_w) // csx + 1, (h - prm.block_h) // csy + 1
    sz = (prm.block_w // prm.cell_w) * (prm.block_h // prm.cell_h) * prm.nbins
    out = np.empty((nby, nbx, sz), np.float32)
    gx, gy = C.c_int(), C.c_int()
    _hog_lib().orc_hog_blocks(_ptr(np.ascontiguousarray(grad)), _ptr(np.ascontiguousarray(qangle)), w, h,
                              C.byref(prm), _ptr(out), C.byref(gx), C.byref(gy))
    return out


def hog_detect(img: np.ndarray, prm: HogParams, svm: np.ndarray, hit_threshold=0.0):
    """HOGDescriptor::detect (padding 0) -> (xy (n, 2) i32, scores (n,) f64) in window order."""
    a, w, h, pitch, cn = _img(img)
    nwin = max((w - prm.win_w) // prm.wstride_x + 1, 0) * max((h - prm.win_h) // prm.wstride_y + 1, 0) + 1
    xs, ys = np.empty(nwin, np.int32), np.empty(nwin, np.int32)
    sc = np.empty(nwin, np.float64)
    s = np.ascontiguousarray(svm, np.float32)
    n = _hog_lib().orc_hog_detect(_ptr(a), w, h, pitch, cn, C.byref(prm), _ptr(s), s.size, float(hit_threshold),
                                  _ptr(xs), _ptr(ys), _ptr(sc))
    return np.stack([xs[:n], ys[:n]], 1), sc[:n]


def hog_group(rects: np.ndarray, weights: np.ndarray, group_threshold: int, img_size, eps=0.2):
    r = np.ascontiguousarray(rects, np.int32).copy()
    wt = np.ascontiguousarray(weights, np.float64).copy()
    n = _hog_lib().orc_hog_group(_ptr(r), _ptr(wt), len(r), int(group_threshold), float(eps), img_size[0],
                                 img_size[1])
    return r[:n], wt[:n]


def hog_detect_multiscale(img: np.ndarray, prm: HogParams, svm: np.ndarray, hit_threshold=0.0, nlevels=64,
                          scale0=1.05, group_threshold=2, max_rects=1 << 16):
    """HOGDescriptor::detectMultiScale(img, rects, weights, hit, winStride, Size(), scale0, group) -> (rects, weights)."""
    a, w, h, pitch, cn = _img(img)
    rects = np.empty((max_rects, 4), np.int32)
    wts = np.empty(max_rects, np.float64)
    s = np.ascontiguousarray(svm, np.float32)
    n = _hog_lib().orc_hog_detect_multiscale(_ptr(a), w, h, pitch, cn, C.byref(prm), _ptr(s), s.size,
                                             float(hit_threshold), int(nlevels), float(scale0), int(group_threshold),
                                             _ptr(rects), _ptr(wts), max_rects)
    return rects[:n], wts[:n]
