"""opencv_amd — MI355X-native TBD/KLT hot path (pyramid, GFTT, sparse PyrLK, affine box
propagation) behind the reference's operator interfaces.  Compute runs in the HIP
kernels of opencv_amd/lib/libtbdk.so (C ABI: include/tbdk.h)."""
from . import _lib  # noqa: F401

__all__ = ["_lib"]
__version__ = "0.1.0"
