"""GPU parity of the role-split floating-point pyramid build (klt_pyr_fp.hip,
ctx option pyr_fuse >= 1, the default) against the oracle
(oracle/klt16_oracle.c: orc16_pyr_down / orc16_scharr and the fp32 twins) and
against the one-launch-per-plane build (pyr_fuse=0), at 1 / 2 / 4 rows per
thread (ctx option pyr_rows), with and without the XCD row bands (pyr_xcd): fp16 levels from u8 and
fp16 frames, fp32 levels from u8, u16 and fp32 frames; padded levels (reflect-101
frames) and derivative planes bit-exact.  Layouts: dense frames, frames whose
last byte ends their allocation (the dword fast path's last-row rule), and
frames with an odd pitch and an element-offset start (no 4-byte alignment: the
per-element path everywhere); sizes down to levels of 1-3 pixels."""
import numpy as np
import pytest
import torch

import _oracle as O

pytestmark = pytest.mark.gpu

TT = {"u8": torch.uint8, "u16": torch.int16, "f16": torch.float16, "f32": torch.float32}


def _img(kind, h, w, seed):
    rng = np.random.default_rng(seed)
    if kind == "u8":
        return rng.integers(0, 256, (h, w), dtype=np.uint8)
    if kind == "u16":
        return rng.integers(0, 65536, (h, w), dtype=np.uint16)
    a = rng.uniform(0, 255, (h, w)) + rng.uniform(0, 1, (h, w))
    if kind == "f16":
        a = a.astype(np.float16)
        a[:2, :3] = np.float16(3e-7)  # subnormals
        return a
    return a.astype(np.float32)


def _place(img, kind, layout):
    """device view of img in the requested layout"""
    h, w = img.shape
    raw = torch.from_numpy(img.view(np.int16) if kind == "u16" else img)
    fix = (lambda t: t.view(torch.uint16)) if kind == "u16" else (lambda t: t)
    if layout == "dense":
        return fix(raw.cuda())
    if layout == "end":
        n = h * w + 4096
        buf = torch.empty(n, dtype=TT[kind], device="cuda")
        v = buf[n - h * w:].view(h, w)
        v.copy_(raw.cuda())
        return fix(v)
    pitch = w + 3  # odd pitch, start one element in
    buf = torch.zeros(1 + h * pitch, dtype=TT[kind], device="cuda")
    v = buf[1:].as_strided((h, w), (pitch, 1))
    v.copy_(raw.cuda())
    return fix(v)


def _build(ctx, dev, kind, store, win, maxlev):
    from opencv_amd import klt

    h, w = dev.shape
    P = klt.Pyramid(ctx, w, h, maxlev, win, torch.float16 if store == "f16" else torch.float32)
    return P.build(dev)


CASES = [("f16", "u8"), ("f16", "f16"), ("f32", "u8"), ("f32", "u16"), ("f32", "f32")]


@pytest.mark.parametrize("store,kind", CASES)
@pytest.mark.parametrize("layout", ["dense", "end", "odd"])
@pytest.mark.parametrize("shape,maxlev,win", [((217, 333), 3, 21), ((1081, 1920), 2, 21), ((97, 131), 3, 7),
                                             ((6, 11), 3, 21), ((2160, 3840), 2, 21)])
def test_pyr_fp_bit_exact(gpu, store, kind, layout, shape, maxlev, win):
    if shape == (2160, 3840) and layout != "dense":
        pytest.skip("4K: dense layout only")
    h, w = shape
    img = _img(kind, h, w, h * 7 + w)
    dev = _place(img, kind, layout)
    R = O.Pyramid16(img, (win, win), maxlev, f32=store == "f32")
    view = np.uint16 if store == "f16" else np.uint32
    try:
        for mode, rows, xcd in ((1, 1, 1), (1, 1, 0), (1, 4, 1), (1, 2, 0), (0, 1, 1)):
            gpu.set_option("pyr_fuse", mode)
            gpu.set_option("pyr_rows", rows)  # rows per thread of the role-split build
            gpu.set_option("pyr_xcd", xcd)  # row bands per XCD
            P = _build(gpu, dev, kind, store, (win, win), maxlev)
            torch.cuda.synchronize()
            assert P.nlevels == R.nlevels
            for i in range(P.nlevels):
                ref = R.levels[i]
                hh, ww = ref.shape
                pad = P.pyr.lv[i].pad
                ry = [O.load().orc_reflect101(y - pad, hh) for y in range(hh + 2 * pad)]
                rx = [O.load().orc_reflect101(x - pad, ww) for x in range(ww + 2 * pad)]
                full = P.level(i, with_border=True)
                assert np.array_equal(full.view(view), ref[np.ix_(ry, rx)].view(view)), f"mode {mode}/{rows}/{xcd} level {i}"
                assert np.array_equal(P.deriv(i).view(view), R.derivs[i].view(view)), f"mode {mode}/{rows}/{xcd} deriv {i}"
    finally:
        gpu.set_option("pyr_fuse", 1)
        gpu.set_option("pyr_rows", 1)
        gpu.set_option("pyr_xcd", 1)
