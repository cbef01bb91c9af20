"""ctypes binding of libtbdk.so (the C ABI declared in include/tbdk.h).

The product path is the HIP library; there is no CPU fallback.  If the shared
object is missing the import fails loudly (`TbdkError`), and every call that
returns a negative status raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libtbdk.so")

TBDK_OK = 0
TBDK_EINVAL = -1
TBDK_EHIP = -2
TBDK_ENOMEM = -3
TBDK_ENODEV = -4
TBDK_MAX_LEVELS = 8
TBDK_ABI_VERSION = 2  # include/tbdk.h: the struct layouts below
OPTFLOW_USE_INITIAL_FLOW = 4
OPTFLOW_LK_GET_MIN_EIGENVALS = 8

_ERRNAMES = {
    TBDK_EINVAL: "TBDK_EINVAL (bad argument)",
    TBDK_EHIP: "TBDK_EHIP (HIP runtime error)",
    TBDK_ENOMEM: "TBDK_ENOMEM (device allocation failed)",
    TBDK_ENODEV: "TBDK_ENODEV (no such device)",
}


class TbdkError(RuntimeError):
    """Raised for a negative TBDK_* status (the reference throws cv::Exception)."""


class Level(C.Structure):
    _fields_ = [
        ("data", C.c_void_p),
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("pitch", C.c_int32),
        ("pad", C.c_int32),
    ]


class Pyr(C.Structure):
    _fields_ = [
        ("nlevels", C.c_int32),
        ("win_w", C.c_int32),
        ("win_h", C.c_int32),
        ("lv", Level * TBDK_MAX_LEVELS),
        ("dv", Level * TBDK_MAX_LEVELS),
        ("storage", C.c_void_p),
        ("depth", C.c_int32),
        ("flags", C.c_int32),
        ("cn", C.c_int32),
    ]


class LkParams(C.Structure):
    _fields_ = [
        ("win_w", C.c_int32),
        ("win_h", C.c_int32),
        ("max_level", C.c_int32),
        ("max_count", C.c_int32),
        ("epsilon", C.c_double),
        ("flags", C.c_int32),
        ("min_eig_threshold", C.c_float),
        ("impl", C.c_int32),
    ]


class Roi(C.Structure):
    _fields_ = [("x", C.c_int32), ("y", C.c_int32), ("width", C.c_int32), ("height", C.c_int32)]


class GfttParams(C.Structure):
    _fields_ = [
        ("max_corners", C.c_int32),
        ("quality_level", C.c_double),
        ("min_distance", C.c_double),
        ("block_size", C.c_int32),
        ("use_harris", C.c_int32),
        ("harris_k", C.c_double),
    ]


class TbdConfig(C.Structure):
    _fields_ = [
        ("width", C.c_int32), ("height", C.c_int32),
        ("win", C.c_int32), ("max_level", C.c_int32), ("lk_iters", C.c_int32),
        ("lk_epsilon", C.c_double), ("min_eig_threshold", C.c_float),
        ("max_corners", C.c_int32), ("quality_level", C.c_double), ("min_distance", C.c_double),
        ("redetect_every", C.c_int32), ("min_points", C.c_int32), ("min_fit_points", C.c_int32),
        ("cost_of_non_assignment", C.c_double),
        ("time_window_size", C.c_int32), ("track_age_threshold", C.c_int32),
        ("track_visibility_threshold", C.c_double), ("track_confidence_threshold", C.c_double),
        ("bounds_xmin", C.c_int32), ("bounds_xmax", C.c_int32), ("bounds_ymin", C.c_int32),
        ("bounds_ymax", C.c_int32),
        ("max_tracks", C.c_int32), ("use_klt", C.c_int32),
    ]


class Detection(C.Structure):
    _fields_ = [("id", C.c_int32), ("x", C.c_int32), ("y", C.c_int32), ("width", C.c_int32),
                ("height", C.c_int32), ("confidence", C.c_double)]


class FrameMetrics(C.Structure):
    _fields_ = [("tp", C.c_int32), ("fn", C.c_int32), ("fp", C.c_int32), ("gt", C.c_int32),
                ("matches", C.c_int32), ("bbox_overlap", C.c_double), ("ntracks", C.c_int32),
                ("lk_points", C.c_int32), ("klt_points", C.c_int32), ("klt_predicted", C.c_int32),
                ("redetected", C.c_int32), ("early_gftt", C.c_int32), ("lk_iters", C.c_int64),
                ("host_wait_us", C.c_float), ("host_tracker_us", C.c_float),
                ("host_step_us", C.c_float), ("host_launch_us", C.c_float)]


class TrackInfo(C.Structure):
    _fields_ = [("id", C.c_uint32), ("x", C.c_int32), ("y", C.c_int32), ("width", C.c_int32),
                ("height", C.c_int32), ("pred_x", C.c_int32), ("pred_y", C.c_int32), ("pred_w", C.c_int32),
                ("pred_h", C.c_int32), ("age", C.c_int32), ("total_visible", C.c_int32),
                ("npoints", C.c_int32), ("max_confidence", C.c_double), ("bbox_overlap", C.c_double)]


class BoxFit(C.Structure):
    _fields_ = [("m", C.c_double * 6), ("cx", C.c_double), ("cy", C.c_double), ("npoints", C.c_int32),
                ("valid", C.c_int32)]


class TrackerArgs(C.Structure):
    _fields_ = [("cost_of_non_assignment", C.c_double), ("time_window_size", C.c_int32),
                ("track_age_threshold", C.c_int32), ("track_visibility_threshold", C.c_double),
                ("track_confidence_threshold", C.c_double), ("bounds_xmin", C.c_int32), ("bounds_xmax", C.c_int32),
                ("bounds_ymin", C.c_int32), ("bounds_ymax", C.c_int32)]


class Prediction(C.Structure):
    _fields_ = [("track_id", C.c_uint32), ("valid", C.c_int32), ("cx", C.c_double), ("cy", C.c_double)]


class ScenarioMetrics(C.Structure):
    _fields_ = [("mt", C.c_int32), ("pt", C.c_int32), ("ml", C.c_int32), ("idsw", C.c_int32), ("fm", C.c_int32),
                ("frames", C.c_int32), ("mota", C.c_double), ("amota", C.c_double), ("motp", C.c_double)]


class AppArgs(C.Structure):
    _fields_ = [("pedestrian_bbox_filename", C.c_char_p), ("vehicle_bbox_filename", C.c_char_p),
                ("pedestrian_tracking_filepath", C.c_char_p), ("vehicle_tracking_filepath", C.c_char_p),
                ("history_distribution", C.c_char_p), ("write_tracking", C.c_int32),
                ("num_tracking_iters", C.c_int32), ("num_tracking_frames", C.c_int32), ("rand_seed", C.c_uint32),
                ("verbose", C.c_int32), ("tracker", TrackerArgs)]


class AppResult(C.Structure):
    _fields_ = [("frames", C.c_int64), ("detections", C.c_int64), ("scenario", ScenarioMetrics * 2)]


class FarnebackParams(C.Structure):
    _fields_ = [("num_levels", C.c_int32), ("pyr_scale", C.c_double), ("fast_pyramids", C.c_int32),
                ("win_size", C.c_int32), ("num_iters", C.c_int32), ("poly_n", C.c_int32),
                ("poly_sigma", C.c_double), ("flags", C.c_int32)]


OPTFLOW_FARNEBACK_GAUSSIAN = 256


class HogParams(C.Structure):
    _fields_ = [("win_w", C.c_int32), ("win_h", C.c_int32), ("block_w", C.c_int32), ("block_h", C.c_int32),
                ("block_stride_x", C.c_int32), ("block_stride_y", C.c_int32), ("cell_w", C.c_int32),
                ("cell_h", C.c_int32), ("nbins", C.c_int32), ("win_sigma", C.c_double),
                ("l2hys_threshold", C.c_double), ("gamma_correction", C.c_int32), ("signed_gradient", C.c_int32),
                ("nlevels", C.c_int32), ("hit_threshold", C.c_double), ("win_stride_x", C.c_int32),
                ("win_stride_y", C.c_int32), ("scale0", C.c_double), ("group_threshold", C.c_int32)]

_P = C.c_void_p
_PI = C.POINTER(C.c_int)

# name -> (restype, argtypes); every symbol include/tbdk.h declares
SIGNATURES = {
    "tbdk_version": (C.c_char_p, []),
    "tbdk_abi_version": (C.c_int, []),
    "tbdk_ctx_create": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "tbdk_ctx_destroy": (C.c_int, [C.c_void_p]),
    "tbdk_ctx_device": (C.c_int, [C.c_void_p]),
    "tbdk_timing_enable": (C.c_int, [C.c_void_p, C.c_int]),
    "tbdk_corner_min_eig_val": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                          C.c_void_p]),
    "tbdk_corner_response": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                       C.c_int, C.c_int, C.c_double, C.c_void_p]),
    "tbdk_ctx_set_option": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int64]),
    "tbdk_timing_select": (C.c_int, [C.c_void_p, C.c_char_p]),
    "tbdk_timing_query": (C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(C.c_int64), C.POINTER(C.c_double)]),
    "tbdk_timing_calls": (C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(C.c_int64)]),
    "tbdk_pyr_create": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(Pyr)]),
    "tbdk_pyr_create_f16": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(Pyr)]),
    "tbdk_pyr_create_f32": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(Pyr)]),
    "tbdk_pyr_create_f32_cn": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                         C.POINTER(Pyr)]),
    "tbdk_pyr_build_u16": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.POINTER(Pyr), C.c_void_p]),
    "tbdk_pyr_build_f32": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.POINTER(Pyr), C.c_void_p]),
    "tbdk_pyr_create_levels": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(Pyr)]),
    "tbdk_pyr_create_cn": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                     C.POINTER(Pyr)]),
    "tbdk_pyr_build_f16": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.POINTER(Pyr), C.c_void_p]),
    "tbdk_pyr_destroy": (C.c_int, [C.c_void_p, C.POINTER(Pyr)]),
    "tbdk_pyr_build": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.POINTER(Pyr), C.c_void_p]),
    "tbdk_pyr_build_borrowed": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.POINTER(Pyr), C.c_void_p]),
    "tbdk_pyr_download": (C.c_int, [C.c_void_p, C.POINTER(Pyr), C.c_int, C.c_void_p, C.c_int, C.c_int]),
    "tbdk_pyr_download_deriv": (C.c_int, [C.c_void_p, C.POINTER(Pyr), C.c_int, C.c_void_p, C.c_int]),
    "tbdk_pyr_down_u8": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                   C.c_void_p]),
    "tbdk_lk_sparse": (C.c_int, [C.c_void_p, C.POINTER(Pyr), C.POINTER(Pyr), C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_void_p, C.c_void_p, C.c_int, C.POINTER(LkParams), C.c_void_p]),
    "tbdk_gftt_rois": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(Roi), C.c_int,
                                 C.POINTER(GfttParams), C.c_void_p, C.c_void_p, C.c_void_p]),
    "tbdk_gftt_reserve": (C.c_int, [C.c_void_p, C.c_int, C.c_int64]),
    "tbdk_box_propagate": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                     C.c_int, C.c_void_p, C.c_void_p]),
    "tbdk_warp_affine_u8": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int,
                                      C.c_int, C.POINTER(C.c_double), C.c_int, C.c_int, C.c_int, C.c_void_p]),
    "tbdk_tracker_default_args": (C.c_int, [C.POINTER(TrackerArgs)]),
    "tbdk_tracker_create": (C.c_int, [C.POINTER(TrackerArgs), C.POINTER(C.c_void_p)]),
    "tbdk_tracker_destroy": (C.c_int, [C.c_void_p]),
    "tbdk_tracker_step": (C.c_int, [C.c_void_p, C.POINTER(Detection), C.c_int, C.c_int, C.POINTER(Prediction), C.c_int,
                                    C.POINTER(FrameMetrics)]),
    "tbdk_tracker_tracks": (C.c_int, [C.c_void_p, C.POINTER(TrackInfo), C.c_int, C.POINTER(C.c_int)]),
    "tbdk_tracker_reset": (C.c_int, [_P]),
    "tbdk_tracker_step_traj": (C.c_int, [_P, C.POINTER(Detection), C.c_int, C.c_int, C.POINTER(Prediction), C.c_int,
                                         _P, C.POINTER(FrameMetrics)]),
    "tbdk_rand_create": (C.c_int, [C.c_uint32, C.POINTER(_P)]),
    "tbdk_rand_destroy": (C.c_int, [_P]),
    "tbdk_rand_next": (C.c_int, [_P, C.POINTER(C.c_int32)]),
    "tbdk_tracker_set_rand": (C.c_int, [_P, _P]),
    "tbdk_parse_history_distribution": (C.c_int, [C.c_char_p, C.POINTER(C.c_float), C.c_int, _PI]),
    "tbdk_history_age": (C.c_int, [_P, C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_uint32)]),
    "tbdk_sequence_create": (C.c_int, [C.POINTER(_P)]),
    "tbdk_sequence_destroy": (C.c_int, [_P]),
    "tbdk_sequence_parse_bbox_file": (C.c_int, [_P, C.c_int, C.c_char_p, C.c_uint32]),
    "tbdk_sequence_error": (C.c_char_p, [_P]),
    "tbdk_sequence_info": (C.c_int, [_P, C.c_int, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                     C.POINTER(C.c_int32)]),
    "tbdk_sequence_history": (C.c_int, [_P, C.POINTER(C.c_uint32), C.c_int, _PI]),
    "tbdk_sequence_camera_pose": (C.c_int, [_P, C.c_int, C.POINTER(C.c_double), C.c_int, _PI]),
    "tbdk_sequence_detections": (C.c_int, [_P, C.c_int, C.c_int, _P, C.POINTER(Detection), C.c_int, _PI]),
    "tbdk_trajectories_create": (C.c_int, [C.POINTER(_P)]),
    "tbdk_trajectories_destroy": (C.c_int, [_P]),
    "tbdk_trajectories_add_position": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
    "tbdk_trajectories_count": (C.c_int, [_P, _PI]),
    "tbdk_track_buffer_create": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "tbdk_track_buffer_destroy": (C.c_int, [_P]),
    "tbdk_tracker_store_tracks": (C.c_int, [_P, _P, C.c_int]),
    "tbdk_tracker_load_tracks": (C.c_int, [_P, _P, C.c_int]),
    "tbdk_tracking_write": (C.c_int, [_P, C.POINTER(C.c_uint32), C.c_int, C.c_int, _P, C.c_char_p, C.c_int,
                                      C.POINTER(ScenarioMetrics)]),
    "tbdk_app_default_args": (C.c_int, [C.POINTER(AppArgs)]),
    "tbdk_app_run": (C.c_int, [C.POINTER(AppArgs), C.POINTER(AppResult)]),
    "tbdk_tbd_default_config": (C.c_int, [C.c_int, C.c_int, C.POINTER(TbdConfig)]),
    "tbdk_tbd_create": (C.c_int, [C.c_void_p, C.POINTER(TbdConfig), C.POINTER(C.c_void_p)]),
    "tbdk_tbd_destroy": (C.c_int, [C.c_void_p]),
    "tbdk_tbd_step": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.POINTER(Detection), C.c_int,
                                C.POINTER(FrameMetrics), C.c_void_p]),
    "tbdk_tbd_step_ahead": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.POINTER(Detection), C.c_int,
                                      C.c_void_p, C.c_int, C.POINTER(FrameMetrics), C.c_void_p]),
    "tbdk_tbd_run": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.c_int, C.c_int, C.POINTER(Detection),
                               C.POINTER(C.c_int32), C.c_int, C.POINTER(FrameMetrics), C.c_void_p]),
    "tbdk_tbd_run_host": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.c_int, C.c_int, C.POINTER(Detection),
                                    C.POINTER(C.c_int32), C.c_int, C.POINTER(FrameMetrics), C.c_void_p]),
    "tbdk_tbd_set_trajectories": (C.c_int, [_P, _P]),
    "tbdk_tbd_tracking_write": (C.c_int, [_P, C.POINTER(C.c_uint32), C.c_int, C.c_int, C.c_char_p, C.c_int,
                                          C.POINTER(ScenarioMetrics)]),
    "tbdk_tbd_tracks": (C.c_int, [C.c_void_p, C.POINTER(TrackInfo), C.c_int, C.POINTER(C.c_int)]),
    "tbdk_tbd_predictions": (C.c_int, [C.c_void_p, C.POINTER(Prediction), C.c_int, C.POINTER(C.c_int)]),
    "tbdk_hbm_copy": (C.c_int, [_P, _P, _P, C.c_int64, _P]),
    "tbdk_synth_render": (C.c_int, [C.c_void_p, C.c_uint32, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                    C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]),
    "tbdk_lk_dense": (C.c_int, [_P, C.POINTER(Pyr), C.POINTER(Pyr), _P, C.c_int, _P, C.c_int, C.POINTER(LkParams),
                                _P]),
    "tbdk_farneback_default_params": (C.c_int, [C.POINTER(FarnebackParams)]),
    "tbdk_farneback_levels": (C.c_int, [C.c_int, C.c_int, C.POINTER(FarnebackParams), _PI, C.POINTER(C.c_int32)]),
    "tbdk_hog_default_params": (C.c_int, [C.POINTER(HogParams)]),
    "tbdk_hog_descriptor_size": (C.c_int, [C.POINTER(HogParams), _PI]),
    "tbdk_hog_detect_multiscale": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(HogParams), _P,
                                             C.c_int, _P, _P, C.c_int, _PI, _P]),
    "tbdk_hog_detect": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(HogParams), _P, C.c_int, _P,
                                  _P, C.c_int, _PI, _P]),
    "tbdk_hog_resize": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, C.c_int, _P, C.c_int, C.c_int, C.c_int, _P]),
    "tbdk_hog_gradient": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(HogParams), _P, C.c_int,
                                    _P, C.c_int, _P]),
    "tbdk_hog_blocks": (C.c_int, [_P, _P, C.c_int, _P, C.c_int, C.c_int, C.c_int, C.POINTER(HogParams), _P, _P]),
    "tbdk_farneback": (C.c_int, [_P, _P, _P, C.c_int, C.c_int, C.c_int, _P, C.c_int, C.POINTER(FarnebackParams), _P]),
    "tbdk_fb_level_image": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, _P,
                                      C.c_int, _P]),
    "tbdk_fb_poly_exp": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, _P, C.c_int, _P]),
}

_lib = None


def load(path: str | None = None) -> C.CDLL:
    """Load libtbdk.so (once).  Raises TbdkError if it is absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("TBDK_LIB") or LIB_PATH  # TBDK_LIB: an alternative build (tuning runs)
    if not os.path.exists(p):
        raise TbdkError(
            f"libtbdk.so not found at {p}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the HIP path has no CPU fallback)")
    # TBDK_HOST_ONLY: TBDK_LIB is the host-only C++ build (tracker, sample
    # driver; make host-asan), which exports only the host entry points and
    # needs no HIP runtime (tests/test_host_sanitizers.py)
    host_only = os.environ.get("TBDK_HOST_ONLY") == "1"
    if not host_only:
        # torch carries its own libamdhip64.so.7 (same soname as /opt/rocm's): load it
        # first so the process holds ONE HIP runtime, whichever of the two is imported
        # first by the caller (two runtimes -> the second sees no device).
        import torch  # noqa: F401
    lib = C.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        if host_only and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(status: int, what: str = "tbdk call") -> None:
    if status != TBDK_OK:
        raise TbdkError(f"{what} failed: {_ERRNAMES.get(status, status)}")
