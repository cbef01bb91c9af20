"""Dense Farneback optical flow over libtbdk (HIP, gfx950).

  * FarnebackOpticalFlow <- cv::cuda::FarnebackOpticalFlow
        (modules/cudaoptflow/include/opencv2/cudaoptflow.hpp:210-252,
         impl modules/cudaoptflow/src/farneback.cpp:164-196)

Numerics follow the CPU cv::calcOpticalFlowFarneback
(modules/video/src/optflowgf.cpp:1096-1190).  Frames are u8 torch tensors on
the HIP device; the flow is a (H, W, 2) float32 tensor (CV_32FC2).  Invalid
arguments raise TbdkError (the reference's CV_Assert).
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from .klt import Context, _stream_ptr

OPTFLOW_FARNEBACK_GAUSSIAN = _lib.OPTFLOW_FARNEBACK_GAUSSIAN
OPTFLOW_USE_INITIAL_FLOW = _lib.OPTFLOW_USE_INITIAL_FLOW


class FarnebackOpticalFlow:
    """cv::cuda::FarnebackOpticalFlow (create / getters / setters / calc)."""

    def __init__(self, numLevels: int = 5, pyrScale: float = 0.5, fastPyramids: bool = False, winSize: int = 13,
                 numIters: int = 10, polyN: int = 5, polySigma: float = 1.1, flags: int = 0,
                 ctx: Context | None = None):
        self.p = _lib.FarnebackParams(int(numLevels), float(pyrScale), int(bool(fastPyramids)), int(winSize),
                                      int(numIters), int(polyN), float(polySigma), int(flags))
        self.ctx = ctx

    @staticmethod
    def create(numLevels: int = 5, pyrScale: float = 0.5, fastPyramids: bool = False, winSize: int = 13,
               numIters: int = 10, polyN: int = 5, polySigma: float = 1.1, flags: int = 0, **kw):
        return FarnebackOpticalFlow(numLevels, pyrScale, fastPyramids, winSize, numIters, polyN, polySigma, flags,
                                    **kw)

    # getters / setters of cudaoptflow.hpp:218-240
    def getNumLevels(self): return self.p.num_levels
    def setNumLevels(self, v): self.p.num_levels = int(v)
    def getPyrScale(self): return self.p.pyr_scale
    def setPyrScale(self, v): self.p.pyr_scale = float(v)
    def getFastPyramids(self): return bool(self.p.fast_pyramids)
    def setFastPyramids(self, v): self.p.fast_pyramids = int(bool(v))
    def getWinSize(self): return self.p.win_size
    def setWinSize(self, v): self.p.win_size = int(v)
    def getNumIters(self): return self.p.num_iters
    def setNumIters(self, v): self.p.num_iters = int(v)
    def getPolyN(self): return self.p.poly_n
    def setPolyN(self, v): self.p.poly_n = int(v)
    def getPolySigma(self): return self.p.poly_sigma
    def setPolySigma(self, v): self.p.poly_sigma = float(v)
    def getFlags(self): return self.p.flags
    def setFlags(self, v): self.p.flags = int(v)

    def levels(self, width: int, height: int) -> list[tuple[int, int]]:
        """(width, height) of every pyramid level calc uses, finest first."""
        lib = _lib.load()
        n = C.c_int()
        sizes = (C.c_int32 * (2 * (max(self.p.num_levels, 0) + 1)))()
        _lib.check(lib.tbdk_farneback_levels(int(width), int(height), C.byref(self.p), C.byref(n), sizes),
                   "tbdk_farneback_levels")
        return [(sizes[2 * i], sizes[2 * i + 1]) for i in range(n.value)]

    def calc(self, I0: torch.Tensor, I1: torch.Tensor, flow: torch.Tensor | None = None, stream=None) -> torch.Tensor:
        if I0.dim() != 2 or I0.shape != I1.shape or I0.dtype != torch.uint8 or I1.dtype != torch.uint8:
            raise _lib.TbdkError("FarnebackOpticalFlow.calc: I0, I1 must be same-size 2-D uint8 (CV_8UC1)")
        if I0.stride(1) != 1 or I1.stride(1) != 1 or I0.stride(0) != I1.stride(0):
            raise _lib.TbdkError("FarnebackOpticalFlow.calc: frames need unit column stride and a common pitch")
        h, w = I0.shape
        if flow is None and self.p.flags & OPTFLOW_USE_INITIAL_FLOW:
            # CV_Assert(_flow0.size() == prev0.size() && ...) (optflowgf.cpp:1117-1119)
            raise _lib.TbdkError("FarnebackOpticalFlow.calc: OPTFLOW_USE_INITIAL_FLOW needs the initial flow")
        if flow is None:
            flow = torch.empty((h, w, 2), dtype=torch.float32, device=I0.device)
        if flow.shape != (h, w, 2) or flow.dtype != torch.float32 or not flow.is_contiguous():
            raise _lib.TbdkError("FarnebackOpticalFlow.calc: flow must be a contiguous (H, W, 2) float32 tensor")
        ctx = self.ctx or Context.get(I0.device.index or 0)
        _lib.check(ctx.lib.tbdk_farneback(ctx.handle, C.c_void_p(I0.data_ptr()), C.c_void_p(I1.data_ptr()), w, h,
                                          I0.stride(0), C.c_void_p(flow.data_ptr()), 8 * w, C.byref(self.p),
                                          _stream_ptr(stream)), "tbdk_farneback")
        return flow


def calc_optical_flow_farneback(prev: torch.Tensor, nxt: torch.Tensor, flow: torch.Tensor | None = None,
                                pyr_scale: float = 0.5, levels: int = 5, winsize: int = 13, iterations: int = 10,
                                poly_n: int = 5, poly_sigma: float = 1.1, flags: int = 0,
                                ctx: Context | None = None, stream=None) -> torch.Tensor:
    """cv::calcOpticalFlowFarneback's argument order (video/src/optflowgf.cpp:1192-1200)."""
    fb = FarnebackOpticalFlow(levels, pyr_scale, False, winsize, iterations, poly_n, poly_sigma, flags, ctx=ctx)
    return fb.calc(prev, nxt, flow, stream)


def level_image(img: torch.Tensor, size, smooth_size: int, sigma: float, ctx: Context | None = None,
                stream=None) -> torch.Tensor:
    """Stage hook: resize(GaussianBlur(float(img)), size, INTER_LINEAR) as calc builds a level."""
    h, w = img.shape
    dw, dh = size
    out = torch.empty((dh, dw), dtype=torch.float32, device=img.device)
    ctx = ctx or Context.get(img.device.index or 0)
    _lib.check(ctx.lib.tbdk_fb_level_image(ctx.handle, C.c_void_p(img.data_ptr()), w, h, img.stride(0), dw, dh,
                                           int(smooth_size), float(sigma), C.c_void_p(out.data_ptr()), 4 * dw,
                                           _stream_ptr(stream)), "tbdk_fb_level_image")
    return out


def poly_exp(src: torch.Tensor, poly_n: int, poly_sigma: float, ctx: Context | None = None,
             stream=None) -> torch.Tensor:
    """Stage hook: FarnebackPolyExp -> (H, W, 5) float32 (the reference's CV_32FC5)."""
    src = src.contiguous()
    h, w = src.shape
    planes = torch.empty((5, h, w), dtype=torch.float32, device=src.device)
    ctx = ctx or Context.get(src.device.index or 0)
    _lib.check(ctx.lib.tbdk_fb_poly_exp(ctx.handle, C.c_void_p(src.data_ptr()), w, h, 4 * w, int(poly_n),
                                        float(poly_sigma), C.c_void_p(planes.data_ptr()), 4 * w,
                                        _stream_ptr(stream)), "tbdk_fb_poly_exp")
    return planes.permute(1, 2, 0)
