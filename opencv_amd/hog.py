"""HOG people detector over libtbdk (HIP, gfx950).

  * HOG <- cv::cuda::HOG (modules/cudaobjdetect/include/opencv2/cudaobjdetect.hpp:75-180,
        impl modules/cudaobjdetect/src/hog.cpp): create / setters / getters /
        setSVMDetector / getDefaultPeopleDetector / detect / detectMultiScale.

Detections equal the CPU cv::HOGDescriptor's (objdetect/src/hog.cpp), whose
detectMultiScale the sample calls in CPU mode (samples/gpu/tbd.cpp:603-605).
Images are u8 torch tensors on the HIP device: (H, W) gray, (H, W, 3) BGR or
(H, W, 4) BGRA (alpha ignored).  Invalid arguments raise TbdkError.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch

from . import _lib
from .klt import Context, _stream_ptr

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def _detector(name: str) -> np.ndarray:
    return np.fromfile(os.path.join(_DATA, name), dtype="<f4")


class HOG:
    """cv::cuda::HOG with the CPU HOGDescriptor's results."""

    def __init__(self, win_size=(64, 128), block_size=(16, 16), block_stride=(8, 8), cell_size=(8, 8), nbins=9,
                 ctx: Context | None = None):
        self.p = _lib.HogParams()
        _lib.check(_lib.load().tbdk_hog_default_params(C.byref(self.p)), "tbdk_hog_default_params")
        self.p.win_w, self.p.win_h = map(int, win_size)
        self.p.block_w, self.p.block_h = map(int, block_size)
        self.p.block_stride_x, self.p.block_stride_y = map(int, block_stride)
        self.p.cell_w, self.p.cell_h = map(int, cell_size)
        self.p.nbins = int(nbins)
        self.p.win_stride_x, self.p.win_stride_y = map(int, block_stride)  # win_stride_(block_stride)
        self.getDescriptorSize()  # HOG_Impl's asserts (cudaobjdetect/src/hog.cpp:252-256)
        self.svm = np.zeros(0, np.float32)
        self.ctx = ctx

    @staticmethod
    def create(win_size=(64, 128), block_size=(16, 16), block_stride=(8, 8), cell_size=(8, 8), nbins=9, **kw):
        return HOG(win_size, block_size, block_stride, cell_size, nbins, **kw)

    # ---- setters / getters (cudaobjdetect.hpp:103-160) ----
    def setGammaCorrection(self, v: bool): self.p.gamma_correction = int(bool(v))
    def getGammaCorrection(self) -> bool: return bool(self.p.gamma_correction)
    def setL2HysThreshold(self, v: float): self.p.l2hys_threshold = float(v)
    def getL2HysThreshold(self) -> float: return self.p.l2hys_threshold
    def setNumLevels(self, v: int): self.p.nlevels = int(v)
    def getNumLevels(self) -> int: return self.p.nlevels
    def setHitThreshold(self, v: float): self.p.hit_threshold = float(v)
    def getHitThreshold(self) -> float: return self.p.hit_threshold
    def setWinStride(self, v): self.p.win_stride_x, self.p.win_stride_y = map(int, v)
    def getWinStride(self): return (self.p.win_stride_x, self.p.win_stride_y)
    def setScaleFactor(self, v: float): self.p.scale0 = float(v)
    def getScaleFactor(self) -> float: return self.p.scale0
    def setGroupThreshold(self, v: int): self.p.group_threshold = int(v)
    def getGroupThreshold(self) -> int: return self.p.group_threshold
    def setWinSigma(self, v: float): self.p.win_sigma = float(v)
    def getWinSigma(self) -> float:
        return self.p.win_sigma if self.p.win_sigma > 0 else (self.p.block_w + self.p.block_h) / 8.0
    def setSignedGradient(self, v: bool): self.p.signed_gradient = int(bool(v))

    def getDescriptorSize(self) -> int:
        n = C.c_int()
        _lib.check(_lib.load().tbdk_hog_descriptor_size(C.byref(self.p), C.byref(n)), "HOG: invalid geometry")
        return n.value

    def getBlockHistogramSize(self) -> int:
        return (self.p.block_w // self.p.cell_w) * (self.p.block_h // self.p.cell_h) * self.p.nbins

    def setSVMDetector(self, detector):
        d = np.ascontiguousarray(np.asarray(detector, dtype=np.float32).ravel())
        n = self.getDescriptorSize()
        if d.size not in (n, n + 1):  # CV_Assert(detector.cols == descriptor_size (+1))
            raise _lib.TbdkError(f"setSVMDetector: {d.size} coefficients, descriptor size {n}")
        self.svm = d

    def getDefaultPeopleDetector(self) -> np.ndarray:
        """HOG_Impl::getDefaultPeopleDetector (cudaobjdetect/src/hog.cpp:326-334):
        the 64x128 default people detector or the 48x96 (Daimler) one."""
        win = (self.p.win_w, self.p.win_h)
        if win == (64, 128):
            return _detector("hog_people_64x128.f32")
        if win == (48, 96):
            return _detector("hog_people_48x96.f32")
        raise _lib.TbdkError("getDefaultPeopleDetector: win_size must be 64x128 or 48x96")

    # ---- detection ----
    def _img(self, img: torch.Tensor):
        if img.dtype != torch.uint8 or not img.is_cuda or img.dim() not in (2, 3):
            raise _lib.TbdkError("HOG: image must be a u8 device tensor (H, W) or (H, W, 3|4)")
        cn = 1 if img.dim() == 2 else img.shape[2]
        if cn not in (1, 3, 4) or img.stride(-1) != 1 or (img.dim() == 3 and img.stride(1) != cn):
            raise _lib.TbdkError("HOG: image must be gray, BGR or BGRA with packed pixels")
        if self.svm.size == 0:
            raise _lib.TbdkError("HOG: setSVMDetector first")
        h, w = img.shape[:2]
        return w, h, img.stride(0), cn

    def detectMultiScale(self, img: torch.Tensor, confidences: bool = False, stream=None):
        """-> list of (x, y, w, h) rects [, list of weights] (grouped and clipped)."""
        w, h, pitch, cn = self._img(img)
        ctx = self.ctx or Context.get(img.device.index or 0)
        cap = 4096
        while True:
            rects = np.empty((cap, 4), np.int32)
            wts = np.empty(cap, np.float64)
            n = C.c_int()
            rc = ctx.lib.tbdk_hog_detect_multiscale(ctx.handle, C.c_void_p(img.data_ptr()), w, h, pitch, cn,
                                                    C.byref(self.p), self.svm.ctypes.data_as(C.c_void_p),
                                                    self.svm.size, rects.ctypes.data_as(C.c_void_p),
                                                    wts.ctypes.data_as(C.c_void_p), cap, C.byref(n),
                                                    _stream_ptr(stream))
            if rc == _lib.TBDK_ENOMEM and n.value == cap:
                cap *= 4
                continue
            _lib.check(rc, "tbdk_hog_detect_multiscale")
            break
        out = [tuple(int(v) for v in r) for r in rects[:n.value]]
        return (out, list(wts[:n.value])) if confidences else out

    def detect(self, img: torch.Tensor, confidences: bool = False, stream=None):
        """One level (HOGDescriptor::detect): -> window corners [(x, y)] [, scores]."""
        w, h, pitch, cn = self._img(img)
        ctx = self.ctx or Context.get(img.device.index or 0)
        cap = max(((w - self.p.win_w) // self.p.win_stride_x + 1) * ((h - self.p.win_h) // self.p.win_stride_y + 1),
                  1)
        xy = np.empty((cap, 2), np.int32)
        sc = np.empty(cap, np.float64)
        n = C.c_int()
        _lib.check(ctx.lib.tbdk_hog_detect(ctx.handle, C.c_void_p(img.data_ptr()), w, h, pitch, cn, C.byref(self.p),
                                           self.svm.ctypes.data_as(C.c_void_p), self.svm.size,
                                           xy.ctypes.data_as(C.c_void_p), sc.ctypes.data_as(C.c_void_p), cap,
                                           C.byref(n), _stream_ptr(stream)), "tbdk_hog_detect")
        pts = [(int(x), int(y)) for x, y in xy[:n.value]]
        return (pts, list(sc[:n.value])) if confidences else pts


# ---- stage hooks (parity tests) ----

def resize_exact(img: torch.Tensor, size, ctx: Context | None = None, stream=None) -> torch.Tensor:
    """resize(img, size, 0, 0, INTER_LINEAR_EXACT) of a u8 image."""
    h, w = img.shape[:2]
    cn = 1 if img.dim() == 2 else img.shape[2]
    dw, dh = size
    out = torch.empty((dh, dw) + tuple(img.shape[2:]), dtype=torch.uint8, device=img.device)
    ctx = ctx or Context.get(img.device.index or 0)
    _lib.check(ctx.lib.tbdk_hog_resize(ctx.handle, C.c_void_p(img.data_ptr()), w, h, img.stride(0), cn,
                                       C.c_void_p(out.data_ptr()), dw, dh, out.stride(0), _stream_ptr(stream)),
               "tbdk_hog_resize")
    return out


def gradient(img: torch.Tensor, hog: HOG, ctx: Context | None = None, stream=None):
    """HOGDescriptor::computeGradient -> (grad (H, W, 2) f32, qangle (H, W, 2) u8)."""
    h, w = img.shape[:2]
    cn = 1 if img.dim() == 2 else img.shape[2]
    grad = torch.empty((h, w, 2), dtype=torch.float32, device=img.device)
    qa = torch.empty((h, w, 2), dtype=torch.uint8, device=img.device)
    ctx = ctx or Context.get(img.device.index or 0)
    _lib.check(ctx.lib.tbdk_hog_gradient(ctx.handle, C.c_void_p(img.data_ptr()), w, h, img.stride(0), cn,
                                         C.byref(hog.p), C.c_void_p(grad.data_ptr()), 8 * w,
                                         C.c_void_p(qa.data_ptr()), 2 * w, _stream_ptr(stream)), "tbdk_hog_gradient")
    return grad, qa


def blocks(grad: torch.Tensor, qangle: torch.Tensor, hog: HOG, ctx: Context | None = None, stream=None):
    """Normalized block histograms on the cache grid -> (nby, nbx, hist_size) f32."""
    h, w = grad.shape[:2]
    p = hog.p
    csx, csy = np.gcd(p.win_stride_x, p.block_stride_x), np.gcd(p.win_stride_y, p.block_stride_y)
    nbx, nby = (w - p.block_w) // csx + 1, (h - p.block_h) // csy + 1
    out = torch.empty((nby, nbx, hog.getBlockHistogramSize()), dtype=torch.float32, device=grad.device)
    ctx = ctx or Context.get(grad.device.index or 0)
    _lib.check(ctx.lib.tbdk_hog_blocks(ctx.handle, C.c_void_p(grad.data_ptr()), 8 * w, C.c_void_p(qangle.data_ptr()),
                                       2 * w, w, h, C.byref(p), C.c_void_p(out.data_ptr()), _stream_ptr(stream)),
               "tbdk_hog_blocks")
    return out
