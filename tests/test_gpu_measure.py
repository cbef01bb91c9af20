"""The measurement helper behind bench.py's HBM copy peak (tbdk_hbm_copy, a
hand-written 16-byte-per-lane stream copy): exact copies, argument checks."""
import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_hbm_copy_exact_and_checked(gpu):
    from opencv_amd import _lib, klt

    for n in (16, 4096 * 16 + 48, (1 << 24) + 16 * 1000):
        src = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
        dst = torch.zeros_like(src)
        klt.hbm_copy(dst, src, ctx=gpu)
        torch.cuda.synchronize()
        assert torch.equal(dst, src), n
    a = torch.zeros(64, dtype=torch.uint8, device="cuda")
    b = torch.zeros(64, dtype=torch.uint8, device="cuda")
    lib, h = gpu.lib, gpu.handle
    assert lib.tbdk_hbm_copy(h, C.c_void_p(a.data_ptr()), C.c_void_p(b.data_ptr()), 24, None) == -1  # not x16
    assert lib.tbdk_hbm_copy(h, C.c_void_p(a.data_ptr() + 4), C.c_void_p(b.data_ptr()), 16, None) == -1  # align
    assert lib.tbdk_hbm_copy(h, C.c_void_p(a.data_ptr() + 16), C.c_void_p(a.data_ptr()), 32, None) == -1  # overlap
    assert lib.tbdk_hbm_copy(h, C.c_void_p(a.data_ptr()), C.c_void_p(b.data_ptr()), 0, None) == 0
    with pytest.raises(ValueError):
        klt.hbm_copy(a[:32], b, ctx=gpu)
    del _lib
