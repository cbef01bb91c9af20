"""Host-side mirror of the reference's KLT operator interfaces over libtbdk.

Device memory is plain torch tensors on a HIP device (plumbing only; every
computation runs in the HIP kernels of libtbdk.so).  The classes keep the
shape of the reference's CUDA interfaces:

  * SparsePyrLKOpticalFlow  <- cv::cuda::SparsePyrLKOpticalFlow
        (modules/cudaoptflow/include/opencv2/cudaoptflow.hpp:160-180)
  * Pyramid / build_pyramid <- cv::buildOpticalFlowPyramid
        (modules/video/src/lkpyramid.cpp:697-793)
  * pyr_down                <- cv::cuda::pyrDown
        (modules/cudawarping/include/opencv2/cudawarping.hpp:201)

Argument meaning and error behaviour follow the reference: `calc` accepts
images or prebuilt pyramids, empty point sets return empty outputs
(pyrlk.cpp:221-227), invalid arguments raise (CV_Assert -> TbdkError).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib

_ctx_cache: dict[int, "Context"] = {}


def _stream_ptr(stream) -> C.c_void_p:
    if stream is None:
        stream = torch.cuda.current_stream()
    return C.c_void_p(stream.cuda_stream)


class Context:
    """One tbdk_ctx per HIP device (the C ABI allows one per thread x device)."""

    def __init__(self, device: int = 0):
        self.lib = _lib.load()
        h = C.c_void_p()
        _lib.check(self.lib.tbdk_ctx_create(int(device), C.byref(h)), "tbdk_ctx_create")
        self.handle = h
        self.device = int(device)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and h.value:
            try:
                self.lib.tbdk_ctx_destroy(h)
            except Exception:
                pass
            self.handle = None

    @staticmethod
    def get(device: int = 0) -> "Context":
        c = _ctx_cache.get(device)
        if c is None:
            c = Context(device)
            _ctx_cache[device] = c
        return c

    def timing_enable(self, on: bool = True) -> None:
        _lib.check(self.lib.tbdk_timing_enable(self.handle, int(bool(on))), "tbdk_timing_enable")

    def set_option(self, name: str, value: int) -> None:
        """tbdk_ctx_set_option (see include/tbdk.h)."""
        _lib.check(self.lib.tbdk_ctx_set_option(self.handle, name.encode(), int(value)), "tbdk_ctx_set_option")

    def timing_select(self, names=None) -> None:
        """Record only these kernels (iterable of names; None = all)."""
        arg = ",".join(names).encode() if names else None
        _lib.check(self.lib.tbdk_timing_select(self.handle, arg), "tbdk_timing_select")

    def timing_calls(self, name: str) -> int:
        """Selected launches of `name` since timing_enable, timed or not (ctx option timing_every)."""
        n = C.c_int64()
        _lib.check(self.lib.tbdk_timing_calls(self.handle, name.encode(), C.byref(n)), "tbdk_timing_calls")
        return int(n.value)

    def timing_query(self, name: str) -> tuple[int, float]:
        n = C.c_int64()
        ms = C.c_double()
        _lib.check(self.lib.tbdk_timing_query(self.handle, name.encode(), C.byref(n), C.byref(ms)),
                   "tbdk_timing_query")
        return int(n.value), float(ms.value)


DEPTH_8U, DEPTH_16F = 0, 7  # TBDK_DEPTH_* (cv::Mat depth codes; 7 = OpenCV 4's CV_16F)


class Pyramid:
    """A padded pyramid in device memory (tbdk_pyr): u8 levels with int16 Scharr
    planes, or (dtype=torch.float16) the fp16 pixel path's fp16 levels with fp16
    (Ix, Iy) planes, or (dtype=torch.float32) the fp32 pixel path (16U / 32F
    frames) with fp32 levels and planes."""

    def __init__(self, ctx: Context, width: int, height: int, max_level: int = 3, win=(21, 21),
                 dtype: torch.dtype = torch.uint8, derivs: bool = True, channels: int = 1):
        """derivs=False (u8 only): levels without derivative planes
        (tbdk_pyr_create_levels); PyrLK then derives the window's Scharr values
        itself, with the same results.  channels 2..4: interleaved multi-channel
        frames, u8 (tbdk_pyr_create_cn) or the fp32 pixel path for 16U / 32F
        frames (tbdk_pyr_create_f32_cn)."""
        if dtype not in (torch.uint8, torch.float16, torch.float32):
            raise _lib.TbdkError("Pyramid dtype must be torch.uint8, torch.float16 or torch.float32")
        if not derivs and dtype != torch.uint8:
            raise _lib.TbdkError("levels-only pyramids are u8")
        if channels != 1 and (dtype == torch.float16 or not derivs):
            raise _lib.TbdkError("multi-channel pyramids are u8 or fp32, with derivative planes")
        self.ctx = ctx
        self.dtype = dtype
        self.channels = int(channels)
        self.pyr = _lib.Pyr()
        if channels != 1 and dtype == torch.float32:
            _lib.check(ctx.lib.tbdk_pyr_create_f32_cn(ctx.handle, int(width), int(height), int(channels),
                                                      int(max_level), int(win[0]), int(win[1]), C.byref(self.pyr)),
                       "tbdk_pyr_create_f32_cn")
        elif channels != 1:
            _lib.check(ctx.lib.tbdk_pyr_create_cn(ctx.handle, int(width), int(height), int(channels), int(max_level),
                                                  int(win[0]), int(win[1]), C.byref(self.pyr)), "tbdk_pyr_create_cn")
        else:
            create = ctx.lib.tbdk_pyr_create_f16 if dtype == torch.float16 else \
                ctx.lib.tbdk_pyr_create_f32 if dtype == torch.float32 else \
                ctx.lib.tbdk_pyr_create if derivs else ctx.lib.tbdk_pyr_create_levels
            _lib.check(create(ctx.handle, int(width), int(height), int(max_level), int(win[0]), int(win[1]),
                              C.byref(self.pyr)), "tbdk_pyr_create")
        self.width, self.height = int(width), int(height)

    @property
    def nlevels(self) -> int:
        return int(self.pyr.nlevels)

    def build(self, img: torch.Tensor, stream=None) -> "Pyramid":
        """From a 2-D uint8 frame (either depth) or, for an fp16 pyramid, a float16 frame;
        a multi-channel pyramid from an (H, W, C) uint8 frame (fp32 multi-channel
        pyramids also uint16 / float32)."""
        if self.channels != 1:
            ok_types = (torch.uint8, torch.uint16, torch.float32) if self.dtype == torch.float32 else (torch.uint8,)
            if img.dim() != 3 or not img.is_cuda or img.dtype not in ok_types or \
                    tuple(img.shape) != (self.height, self.width, self.channels) or img.stride(2) != 1 or \
                    img.stride(1) != self.channels:
                raise _lib.TbdkError("Pyramid.build expects an (H, W, C) device tensor of the pyramid's size and "
                                     "depth")
            fn = {torch.uint8: self.ctx.lib.tbdk_pyr_build, torch.uint16: self.ctx.lib.tbdk_pyr_build_u16,
                  torch.float32: self.ctx.lib.tbdk_pyr_build_f32}[img.dtype]
            _lib.check(fn(self.ctx.handle, C.c_void_p(img.data_ptr()), int(img.stride(0)) * img.element_size(),
                          C.byref(self.pyr), _stream_ptr(stream)), "tbdk_pyr_build (multi-channel)")
            return self
        if self.dtype == torch.float32 and img.dim() == 2 and img.is_cuda and img.stride(1) == 1 and \
                img.dtype in (torch.uint16, torch.float32):
            if img.shape[0] != self.height or img.shape[1] != self.width:
                raise _lib.TbdkError("image size does not match the pyramid")
            fn = self.ctx.lib.tbdk_pyr_build_u16 if img.dtype == torch.uint16 else self.ctx.lib.tbdk_pyr_build_f32
            _lib.check(fn(self.ctx.handle, C.c_void_p(img.data_ptr()), int(img.stride(0)) * img.element_size(),
                          C.byref(self.pyr), _stream_ptr(stream)), "tbdk_pyr_build (fp32 path)")
            return self
        if img.dim() != 2 or not img.is_cuda or not (img.dtype == torch.uint8 or
                                                     (img.dtype == torch.float16 and self.dtype == torch.float16)):
            raise _lib.TbdkError("Pyramid.build expects a 2-D uint8 (or, fp16 pyramid, float16) device tensor")
        if img.shape[0] != self.height or img.shape[1] != self.width or img.stride(1) != 1:
            raise _lib.TbdkError("image size / layout does not match the pyramid")
        if img.dtype == torch.float16:
            _lib.check(self.ctx.lib.tbdk_pyr_build_f16(self.ctx.handle, C.c_void_p(img.data_ptr()),
                                                       int(img.stride(0)) * 2, C.byref(self.pyr),
                                                       _stream_ptr(stream)), "tbdk_pyr_build_f16")
        else:
            _lib.check(self.ctx.lib.tbdk_pyr_build(self.ctx.handle, C.c_void_p(img.data_ptr()), int(img.stride(0)),
                                                   C.byref(self.pyr), _stream_ptr(stream)), "tbdk_pyr_build")
        return self

    def build_borrowed(self, img: torch.Tensor, stream=None) -> "Pyramid":
        """Levels-only u8 pyramid whose level 0 is `img` itself (no padded copy;
        tbdk_pyr_build_borrowed, the reference GPU class's pyramid,
        cudaoptflow/src/pyrlk.cpp:144-145).  `img` must stay alive and unchanged
        while the pyramid is read; the pyramid keeps a reference to it."""
        if self.dtype != torch.uint8 or self.channels != 1:
            raise _lib.TbdkError("borrowed level 0: u8 single-channel levels-only pyramids")
        if img.dim() != 2 or not img.is_cuda or img.dtype != torch.uint8 or img.shape[0] != self.height or \
                img.shape[1] != self.width or img.stride(1) != 1:
            raise _lib.TbdkError("Pyramid.build_borrowed expects a 2-D uint8 device tensor of the pyramid's size")
        _lib.check(self.ctx.lib.tbdk_pyr_build_borrowed(self.ctx.handle, C.c_void_p(img.data_ptr()),
                                                        int(img.stride(0)), C.byref(self.pyr), _stream_ptr(stream)),
                   "tbdk_pyr_build_borrowed")
        self._borrowed = img
        return self

    def level(self, i: int, with_border: bool = False):
        """Host copy of level i as a (H, W) numpy array, uint8 or float16 (test / download helper)."""
        import numpy as np
        L = self.pyr.lv[i]
        h = L.height + (2 * L.pad if with_border else 0)
        w = L.width + (2 * L.pad if with_border else 0)
        dt = {torch.float16: np.float16, torch.float32: np.float32}.get(self.dtype, np.uint8)
        out = np.empty((h, w) if self.channels == 1 else (h, w, self.channels), dtype=dt)
        _lib.check(self.ctx.lib.tbdk_pyr_download(self.ctx.handle, C.byref(self.pyr), int(i),
                                                  out.ctypes.data_as(C.c_void_p), out.strides[0],
                                                  int(bool(with_border))),
                   "tbdk_pyr_download")
        return out

    def deriv(self, i: int):
        """Host copy of the Scharr derivative plane of level i: (H, W, 2) (Ix, Iy), int16
        (or float16 for an fp16 pyramid)."""
        import numpy as np
        L = self.pyr.dv[i]
        out = np.empty((L.height, L.width, 2 * self.channels),
                       dtype={torch.float16: np.float16, torch.float32: np.float32}.get(self.dtype, np.int16))
        _lib.check(self.ctx.lib.tbdk_pyr_download_deriv(self.ctx.handle, C.byref(self.pyr), int(i),
                                                        out.ctypes.data_as(C.c_void_p), out.strides[0]),
                   "tbdk_pyr_download_deriv")
        return out

    def __del__(self):
        if getattr(self, "pyr", None) is not None and self.pyr.storage:
            try:
                self.ctx.lib.tbdk_pyr_destroy(self.ctx.handle, C.byref(self.pyr))
            except Exception:
                pass


def build_pyramid(img: torch.Tensor, win=(21, 21), max_level: int = 3, ctx: Context | None = None,
                  stream=None, dtype: torch.dtype | None = None, derivs: bool = True) -> Pyramid:
    """cv::buildOpticalFlowPyramid (withDerivatives = derivs); dtype
    torch.float16 (or a float16 frame) selects the fp16 pixel path, torch.float32
    (or a uint16 / float32 frame) the fp32 pixel path; an (H, W, C) uint8 frame
    (C = 2..4, interleaved) a multi-channel pyramid."""
    ctx = ctx or Context.get(img.device.index or 0)
    dtype = dtype or (torch.float16 if img.dtype == torch.float16 else
                      torch.float32 if img.dtype in (torch.uint16, torch.float32) else torch.uint8)
    cn = int(img.shape[2]) if img.dim() == 3 else 1
    return Pyramid(ctx, img.shape[1], img.shape[0], max_level, win, dtype, derivs, channels=cn).build(img, stream)


def pyr_down(src: torch.Tensor, ctx: Context | None = None, stream=None) -> torch.Tensor:
    """cv::cuda::pyrDown for CV_8UC1: ((w+1)/2, (h+1)/2), bit-exact with the CPU pyrDown."""
    if src.dtype != torch.uint8 or src.dim() != 2 or not src.is_cuda or src.stride(1) != 1:
        raise _lib.TbdkError("pyr_down expects a 2-D uint8 device tensor")
    ctx = ctx or Context.get(src.device.index or 0)
    h, w = src.shape
    dst = torch.empty(((h + 1) // 2, (w + 1) // 2), dtype=torch.uint8, device=src.device)
    _lib.check(ctx.lib.tbdk_pyr_down_u8(ctx.handle, C.c_void_p(src.data_ptr()), w, h, src.stride(0),
                                        C.c_void_p(dst.data_ptr()), dst.stride(0), _stream_ptr(stream)),
               "tbdk_pyr_down_u8")
    return dst


def corner_min_eigen_val(src: torch.Tensor, ctx: Context | None = None, stream=None) -> torch.Tensor:
    """cv::cuda::createMinEigenValCorner(CV_8UC1, 3, 3)->compute: float32 (h, w)
    minimum-eigenvalue map, bit-exact with the CPU cornerMinEigenVal."""
    if src.dtype != torch.uint8 or src.dim() != 2 or not src.is_cuda or src.stride(1) != 1:
        raise _lib.TbdkError("corner_min_eigen_val expects a 2-D uint8 device tensor")
    ctx = ctx or Context.get(src.device.index or 0)
    h, w = src.shape
    dst = torch.empty((h, w), dtype=torch.float32, device=src.device)
    _lib.check(ctx.lib.tbdk_corner_min_eig_val(ctx.handle, C.c_void_p(src.data_ptr()), w, h, src.stride(0),
                                               C.c_void_p(dst.data_ptr()), dst.stride(0) * 4, _stream_ptr(stream)),
               "tbdk_corner_min_eig_val")
    return dst


def corner_response(src: torch.Tensor, block_size: int = 3, harris: bool = False, k: float = 0.04,
                    ctx: Context | None = None, stream=None) -> torch.Tensor:
    """cv::cuda::createMinEigenValCorner(CV_8UC1, blockSize, 3) / createHarrisCorner(CV_8UC1,
    blockSize, 3, k) ->compute (cudaimgproc.hpp:548-566): float32 (h, w) response map with
    the CPU cornerMinEigenVal / cornerHarris numerics (corner.cpp:52-152,237-326)."""
    if src.dtype != torch.uint8 or src.dim() != 2 or not src.is_cuda or src.stride(1) != 1:
        raise _lib.TbdkError("corner_response expects a 2-D uint8 device tensor")
    ctx = ctx or Context.get(src.device.index or 0)
    h, w = src.shape
    dst = torch.empty((h, w), dtype=torch.float32, device=src.device)
    _lib.check(ctx.lib.tbdk_corner_response(ctx.handle, C.c_void_p(src.data_ptr()), w, h, src.stride(0),
                                            C.c_void_p(dst.data_ptr()), dst.stride(0) * 4, int(block_size),
                                            1 if harris else 0, float(k), _stream_ptr(stream)),
               "tbdk_corner_response")
    return dst


# numpy mirror of tbdk_box_fit (include/tbdk.h)
BOX_FIT_DTYPE = np.dtype([("m", "<f8", 6), ("cx", "<f8"), ("cy", "<f8"), ("npoints", "<i4"), ("valid", "<i4")])


def box_propagate(prev_pts: torch.Tensor, next_pts: torch.Tensor, status, offsets: torch.Tensor,
                  boxes: torch.Tensor, min_points: int = 4, ctx: Context | None = None, stream=None) -> np.ndarray:
    """tbdk_box_propagate: per box b, the 4-DOF similarity (getRTMatrix, non
    full-affine) fitted to points offsets[b]..offsets[b+1] (status != 0 only)
    and the box centre it carries.  Device tensors: prev/next float32 (N, 2),
    status uint8 (N) or None, offsets int32 (nboxes + 1), boxes int32
    (nboxes, 4).  Returns a BOX_FIT_DTYPE array (synchronises the stream)."""
    for t in (prev_pts, next_pts, offsets, boxes) + ((status,) if status is not None else ()):
        if not t.is_cuda or not t.is_contiguous():
            raise _lib.TbdkError("box_propagate expects contiguous device tensors")
    nb = boxes.shape[0]
    if offsets.dtype != torch.int32 or boxes.dtype != torch.int32 or offsets.numel() != nb + 1:
        raise _lib.TbdkError("offsets: int32 (nboxes + 1), boxes: int32 (nboxes, 4)")
    ctx = ctx or Context.get(prev_pts.device.index or 0)
    out = torch.zeros(max(1, nb) * BOX_FIT_DTYPE.itemsize, dtype=torch.uint8, device=prev_pts.device)
    ptr = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    _lib.check(ctx.lib.tbdk_box_propagate(ctx.handle, ptr(prev_pts), ptr(next_pts), ptr(status), ptr(offsets),
                                          ptr(boxes), nb, int(min_points), ptr(out), _stream_ptr(stream)),
               "tbdk_box_propagate")
    res = out.cpu().numpy()
    return np.frombuffer(res.tobytes(), BOX_FIT_DTYPE)[:nb].copy()


# interpolation flags / border modes (reference values, imgproc.hpp / core/base.hpp)
INTER_NEAREST, INTER_LINEAR, INTER_CUBIC, INTER_AREA, WARP_INVERSE_MAP = 0, 1, 2, 3, 16
BORDER_CONSTANT, BORDER_REPLICATE, BORDER_REFLECT, BORDER_WRAP, BORDER_REFLECT_101, BORDER_TRANSPARENT = range(6)


def warp_affine(src: torch.Tensor, M, dsize, flags: int = INTER_LINEAR, borderMode: int = BORDER_CONSTANT,
                borderValue: int = 0, dst: torch.Tensor | None = None, ctx: Context | None = None,
                stream=None) -> torch.Tensor:
    """cv::cuda::warpAffine(src, dst, M, dsize, flags, borderMode, borderValue) for CV_8UC1
    (cudawarping.hpp:126) with the CPU cv::warpAffine's fixed-point numerics (bit-exact).
    M: 2x3 (host array-like); dsize = (width, height).  `dst` may be passed to keep its
    contents where BORDER_TRANSPARENT leaves pixels untouched."""
    if src.dtype != torch.uint8 or src.dim() != 2 or not src.is_cuda or src.stride(1) != 1:
        raise _lib.TbdkError("warp_affine expects a 2-D uint8 device tensor")
    ctx = ctx or Context.get(src.device.index or 0)
    dw, dh = int(dsize[0]), int(dsize[1])
    if dst is None:
        dst = torch.zeros((dh, dw), dtype=torch.uint8, device=src.device)
    elif dst.shape != (dh, dw) or dst.dtype != torch.uint8 or dst.stride(1) != 1:
        raise _lib.TbdkError("dst must be a (height, width) uint8 device tensor")
    m = (C.c_double * 6)(*[float(v) for v in np.asarray(M, dtype=np.float64).reshape(6)])
    h, w = src.shape
    _lib.check(ctx.lib.tbdk_warp_affine_u8(ctx.handle, C.c_void_p(src.data_ptr()), w, h, src.stride(0),
                                           C.c_void_p(dst.data_ptr()), dw, dh, dst.stride(0), m, int(flags),
                                           int(borderMode), int(borderValue), _stream_ptr(stream)),
               "tbdk_warp_affine_u8")
    return dst


@dataclass
class LkResult:
    next_pts: torch.Tensor
    status: torch.Tensor
    err: torch.Tensor | None
    iters: torch.Tensor | None


class SparsePyrLKOpticalFlow:
    """cv::cuda::SparsePyrLKOpticalFlow with the CPU calcOpticalFlowPyrLK numerics.

    create(winSize=(21,21), maxLevel=3, iters=30, useInitialFlow=False) mirrors
    cudaoptflow.hpp:175-179; epsilon / minEigThreshold / getMinEigenVals are the
    CPU calcOpticalFlowPyrLK parameters (video/include/opencv2/video/tracking.hpp:178-183).
    """

    def __init__(self, winSize=(21, 21), maxLevel: int = 3, iters: int = 30, useInitialFlow: bool = False,
                 epsilon: float = 0.01, minEigThreshold: float = 1e-4, getMinEigenVals: bool = False,
                 device: int = 0, impl: int = 0):
        self.win = (int(winSize[0]), int(winSize[1]))
        self.max_level = int(maxLevel)
        self.iters = int(iters)
        self.use_initial_flow = bool(useInitialFlow)
        self.epsilon = float(epsilon)
        self.min_eig = float(minEigThreshold)
        self.get_min_eig = bool(getMinEigenVals)
        self.impl = int(impl)
        self.ctx = Context.get(device)

    @staticmethod
    def create(winSize=(21, 21), maxLevel: int = 3, iters: int = 30, useInitialFlow: bool = False, **kw):
        return SparsePyrLKOpticalFlow(winSize, maxLevel, iters, useInitialFlow, **kw)

    # getters / setters of cudaoptflow.hpp:163-173
    def getWinSize(self):
        return self.win

    def setWinSize(self, win):
        self.win = (int(win[0]), int(win[1]))

    def getMaxLevel(self):
        return self.max_level

    def setMaxLevel(self, v):
        self.max_level = int(v)

    def getNumIters(self):
        return self.iters

    def setNumIters(self, v):
        self.iters = int(v)

    def getUseInitialFlow(self):
        return self.use_initial_flow

    def setUseInitialFlow(self, v):
        self.use_initial_flow = bool(v)

    def params(self) -> _lib.LkParams:
        flags = 0
        if self.use_initial_flow:
            flags |= _lib.OPTFLOW_USE_INITIAL_FLOW
        if self.get_min_eig:
            flags |= _lib.OPTFLOW_LK_GET_MIN_EIGENVALS
        return _lib.LkParams(self.win[0], self.win[1], self.max_level, self.iters, self.epsilon, flags,
                             self.min_eig, self.impl)

    def _as_pyr(self, img) -> Pyramid:
        if isinstance(img, Pyramid):
            return img  # prebuilt pyramids: any channel count, as calcOpticalFlowPyrLK
        if torch.is_tensor(img) and img.dim() == 3 and img.shape[2] == 2:
            # the CUDA class takes 1, 3 or 4 channels (CV_Assert, cudaoptflow/src/pyrlk.cpp:142,228)
            raise _lib.TbdkError("SparsePyrLKOpticalFlow.calc: frames must have 1, 3 or 4 channels")
        return build_pyramid(img, self.win, self.max_level, self.ctx)

    def calc(self, prevImg, nextImg, prevPts: torch.Tensor, nextPts: torch.Tensor | None = None,
             want_err: bool = True, want_iters: bool = False, stream=None) -> LkResult:
        if prevPts.dtype != torch.float32 or not prevPts.is_cuda:
            raise _lib.TbdkError("prevPts must be a float32 device tensor of shape (N, 2)")
        pts = prevPts.reshape(-1, 2).contiguous()
        n = pts.shape[0]
        dev = pts.device
        if n == 0:
            return LkResult(torch.empty((0, 2), dtype=torch.float32, device=dev),
                            torch.empty((0,), dtype=torch.uint8, device=dev), None, None)
        P, N = self._as_pyr(prevImg), self._as_pyr(nextImg)
        if self.use_initial_flow:
            if nextPts is None or nextPts.numel() != 2 * n:
                raise _lib.TbdkError("useInitialFlow requires nextPts of the same size as prevPts")
            out = nextPts.reshape(-1, 2).to(torch.float32).contiguous().clone()
        else:
            out = torch.empty((n, 2), dtype=torch.float32, device=dev)
        status = torch.empty((n,), dtype=torch.uint8, device=dev)
        err = torch.empty((n,), dtype=torch.float32, device=dev) if want_err else None
        iters = torch.empty((n,), dtype=torch.int32, device=dev) if want_iters else None
        prm = self.params()
        _lib.check(self.ctx.lib.tbdk_lk_sparse(
            self.ctx.handle, C.byref(P.pyr), C.byref(N.pyr), C.c_void_p(pts.data_ptr()), C.c_void_p(out.data_ptr()),
            C.c_void_p(status.data_ptr()), C.c_void_p(err.data_ptr()) if err is not None else None,
            C.c_void_p(iters.data_ptr()) if iters is not None else None, n, C.byref(prm), _stream_ptr(stream)),
            "tbdk_lk_sparse")
        return LkResult(out, status, err, iters)


class DensePyrLKOpticalFlow(SparsePyrLKOpticalFlow):
    """cv::cuda::DensePyrLKOpticalFlow (cudaoptflow.hpp:182-208; impl
    cudaoptflow/src/pyrlk.cpp:238-299): create(winSize=(13,13), maxLevel=3,
    iters=30, useInitialFlow=False); calc(I0, I1) -> (H, W, 2) float32 flow.
    Numerics: the CPU calcOpticalFlowPyrLK at every pixel (tbdk_lk_dense)."""

    def __init__(self, winSize=(13, 13), maxLevel: int = 3, iters: int = 30, useInitialFlow: bool = False, **kw):
        super().__init__(winSize, maxLevel, iters, useInitialFlow, **kw)

    @staticmethod
    def create(winSize=(13, 13), maxLevel: int = 3, iters: int = 30, useInitialFlow: bool = False, **kw):
        return DensePyrLKOpticalFlow(winSize, maxLevel, iters, useInitialFlow, **kw)

    def calc(self, prevImg, nextImg, flow: torch.Tensor | None = None, want_status: bool = False, stream=None):
        P, N = self._as_pyr(prevImg), self._as_pyr(nextImg)
        w, h = P.pyr.lv[0].width, P.pyr.lv[0].height
        dev = torch.device("cuda", self.ctx.device)
        if flow is None:
            flow = torch.empty((h, w, 2), dtype=torch.float32, device=dev)
        if flow.shape != (h, w, 2) or flow.dtype != torch.float32 or not flow.is_contiguous():
            raise _lib.TbdkError("DensePyrLKOpticalFlow.calc: flow must be a contiguous (H, W, 2) float32 tensor")
        status = torch.empty((h, w), dtype=torch.uint8, device=dev) if want_status else None
        prm = self.params()
        _lib.check(self.ctx.lib.tbdk_lk_dense(
            self.ctx.handle, C.byref(P.pyr), C.byref(N.pyr), C.c_void_p(flow.data_ptr()), 8 * w,
            C.c_void_p(status.data_ptr()) if status is not None else None, w, C.byref(prm), _stream_ptr(stream)),
            "tbdk_lk_dense")
        return (flow, status) if want_status else flow


class GoodFeaturesToTrackDetector:
    """cv::cuda::createGoodFeaturesToTrackDetector(CV_8UC1, maxCorners, qualityLevel,
    minDistance, blockSize=3, useHarrisDetector=False, harrisK=0.04)
    (cudaimgproc.hpp:603-604) with the CPU goodFeaturesToTrack semantics, applied
    to a batch of box ROIs of one image."""

    def __init__(self, maxCorners: int = 1000, qualityLevel: float = 0.01, minDistance: float = 0.0,
                 blockSize: int = 3, useHarrisDetector: bool = False, harrisK: float = 0.04, device: int = 0):
        self.prm = _lib.GfttParams(int(maxCorners), float(qualityLevel), float(minDistance), int(blockSize),
                                   1 if useHarrisDetector else 0, float(harrisK))
        self.ctx = Context.get(device)

    def detect_rois(self, image: torch.Tensor, rois, stream=None):
        """rois: iterable of (x, y, w, h).  Returns (corners (nroi, maxCorners, 2) f32,
        counts (nroi,) i32) device tensors; corners are in image coordinates."""
        if image.dtype != torch.uint8 or image.dim() != 2 or not image.is_cuda or image.stride(1) != 1:
            raise _lib.TbdkError("detect expects a 2-D uint8 device tensor")
        rois = list(rois)
        n = len(rois)
        arr = (_lib.Roi * max(n, 1))(*[_lib.Roi(int(x), int(y), int(w), int(h)) for (x, y, w, h) in rois])
        corners = torch.zeros((n, self.prm.max_corners, 2), dtype=torch.float32, device=image.device)
        counts = torch.zeros((n,), dtype=torch.int32, device=image.device)
        _lib.check(self.ctx.lib.tbdk_gftt_rois(self.ctx.handle, C.c_void_p(image.data_ptr()), image.shape[1],
                                               image.shape[0], image.stride(0), arr, n, C.byref(self.prm),
                                               C.c_void_p(corners.data_ptr()), C.c_void_p(counts.data_ptr()),
                                               _stream_ptr(stream)), "tbdk_gftt_rois")
        return corners, counts

    def detect(self, image: torch.Tensor, stream=None) -> torch.Tensor:
        """Whole image as one ROI -> (K, 2) corners (CornersDetector::detect without mask)."""
        c, n = self.detect_rois(image, [(0, 0, image.shape[1], image.shape[0])], stream)
        k = int(n[0].item())
        if k < 0:
            raise _lib.TbdkError("candidate buffer overflow (image too large for one ROI)")
        return c[0, :k]


def hbm_copy(dst: torch.Tensor, src: torch.Tensor, ctx: Context | None = None, stream=None):
    """dst <- src (contiguous device tensors of equal byte size, a multiple of
    16) through libtbdk's 16-byte-per-lane stream-copy kernel (tbdk_hbm_copy;
    bench.py's HBM copy peak)."""
    nbytes = src.numel() * src.element_size()
    if not (src.is_cuda and dst.is_cuda and src.is_contiguous() and dst.is_contiguous()) or \
            dst.numel() * dst.element_size() != nbytes:
        raise ValueError("hbm_copy: contiguous device tensors of equal byte size")
    ctx = ctx or Context.get(src.device.index)
    _lib.check(ctx.lib.tbdk_hbm_copy(ctx.handle, C.c_void_p(dst.data_ptr()), C.c_void_p(src.data_ptr()), nbytes,
                                     _stream_ptr(stream)), "tbdk_hbm_copy")
    return dst


def synth_render(seed: int, width: int, height: int, nobj: int, t0: int, nframes: int, device: int = 0,
                 ctx: Context | None = None, stream=None):
    """Render frames [t0, t0+nframes) of the synthetic sequence into HBM.

    Returns (frames uint8 (nframes, H, W) device tensor, gt int32 (nframes, nobj, 5) host tensor)."""
    ctx = ctx or Context.get(device)
    frames = torch.empty((nframes, height, width), dtype=torch.uint8, device=f"cuda:{device}")
    gt = torch.zeros((nframes, max(nobj, 1), 5), dtype=torch.int32)
    _lib.check(ctx.lib.tbdk_synth_render(ctx.handle, seed, width, height, nobj, t0, nframes,
                                         C.c_void_p(frames.data_ptr()), width, C.c_void_p(gt.data_ptr()),
                                         _stream_ptr(stream)), "tbdk_synth_render")
    return frames, gt[:, :nobj]
