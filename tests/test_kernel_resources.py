"""The built library's kernels hold their intended resources (CPU only: reads
the gfx950 code objects' metadata, tools/kernel_resources.py): no scratch and
no VGPR spills anywhere; no LDS in the streaming kernels (a runtime-indexed
private array that the compiler moved to LDS serialized the two-role pyramid
build's loads in round 4); the loop's PyrLK kernel within 128 VGPRs (4 waves
per SIMD)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
LIB = os.path.join(ROOT, "opencv_amd", "lib", "libtbdk.so")

pytestmark = pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-readelf"),
                                reason="library or llvm-readelf missing")

NO_LDS = ("pyr_build_kernel", "pyr_fp_jobs_kernel", "pad_copy_kernel", "pyr_down_padded_kernel",
          "scharr_levels_kernel", "lk_multi_kernel", "hbm_copy_kernel", "synth_kernel", "warp_affine_kernel")


@pytest.fixture(scope="module")
def res():
    import kernel_resources

    r = kernel_resources.kernel_resources(LIB)
    assert len(r) > 100, "too few kernels found in the library"
    return r


def test_no_scratch_no_vgpr_spills(res):
    bad = {k: v for k, v in res.items() if v["private_segment_fixed_size"] or v["vgpr_spill_count"]}
    assert not bad, bad


def test_streaming_kernels_use_no_lds(res):
    for frag in NO_LDS:
        ks = [k for k in res if frag in k]
        assert ks, frag
        for k in ks:
            assert res[k]["group_segment_fixed_size"] == 0, (k, res[k])


def test_loop_pyrlk_fits_four_waves_per_simd(res):
    k = [k for k in res if "lk_multi_kernelILi21ELi21ELb1E" in k]
    assert len(k) == 1 and res[k[0]]["vgpr_count"] <= 128, res.get(k[0] if k else None)


def test_compact_gftt_eig_fits_beside_one_pyrlk_wave(res):
    """the loop's GFTT eigenvalue kernel (compact candidates) stays at <= 128
    VGPRs, so its waves fit a SIMD slot one ending PyrLK wave frees"""
    k = [k for k in res if "gftt_eig_kernelILb1E" in k]
    assert len(k) == 1 and res[k[0]]["vgpr_count"] <= 128, res.get(k[0] if k else None)
