"""ctypes bindings of libpm.so (include/pm_hip.h, include/pm_host.h).

The library is built in-tree by ``make -C patternmatching_amd/csrc`` (or
``__graft_entry__.build()``).  Importing this module without it raises: the
package has no CPU fallback for the scan.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# PM_LIBPM: an alternative build of the same library, for side-by-side
# timing of kernel revisions in one process tree (scripts/ab_time.sh).
LIB_PATH = os.environ.get("PM_LIBPM") or os.path.join(_HERE, "libpm.so")
CLI_PATH = os.path.join(_HERE, "bin", "pm")

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_vp = ctypes.c_void_p


class PmPattern(ctypes.Structure):
    """struct PmPattern (include/pm_host.h)."""


PmPattern._fields_ = [
    ("file", ctypes.c_uint32),
    ("line", ctypes.c_uint32),
    ("len", ctypes.c_uint32),
    ("index", ctypes.c_uint32),
    ("parent", ctypes.POINTER(PmPattern)),
    ("bytes", c_u8p),
]


class PmDict(ctypes.Structure):
    """PmDict (include/pm_host.h)."""

    _fields_ = [
        ("pats", ctypes.POINTER(PmPattern)),
        ("n", ctypes.c_size_t),
        ("max_len", ctypes.c_size_t),
        ("lines_total", ctypes.c_size_t),
        ("lines_rejected", ctypes.c_size_t),
        ("cap", ctypes.c_size_t),
        ("slots", ctypes.c_void_p),
        ("nslots", ctypes.c_size_t),
    ]


PmDictP = ctypes.POINTER(PmDict)

# name -> (restype, argtypes)
SIGNATURES = {
    # host front end
    "pm_parse_line": (ctypes.c_size_t, [c_u8p, ctypes.c_size_t, c_u8p]),
    "pm_dict_load": (PmDictP, [ctypes.POINTER(ctypes.c_char_p), ctypes.c_size_t, ctypes.c_char_p,
                               ctypes.c_size_t]),
    "pm_dict_new": (PmDictP, []),
    "pm_dict_add": (ctypes.c_int, [PmDictP, c_u8p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32]),
    "pm_dict_finalize": (None, [PmDictP]),
    "pm_dict_feed": (None, [PmDictP, c_vp, c_vp]),
    "pm_dict_free": (None, [PmDictP]),
    "pm_pattern_is_suffix": (ctypes.c_int, [c_vp, c_vp]),
    "pm_pattern_code": (ctypes.c_uint32, [c_vp]),
    "pm_success_rate_add": (None, [c_vp, c_vp, c_vp, ctypes.c_size_t]),
    "pm_mps_table_setup": (None, []),
    "pm_parse_args": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), c_vp]),
    "pm_conf_free": (None, [c_vp]),
    "pm_measure_all": (ctypes.c_int, [c_vp, PmDictP, c_vp]),
    "pm_write_stats": (ctypes.c_int, [c_vp, c_vp]),
    # plugin ABI
    "pm_hip_rt_create": (c_vp, []),
    "pm_hip_ac_create": (c_vp, []),
    "pm_hip_auto_create": (c_vp, []),
    "pm_hip_add_pattern": (None, [c_vp, ctypes.c_char_p, ctypes.c_size_t, c_vp]),
    "pm_hip_compile": (None, [c_vp]),
    "pm_hip_read_char": (c_vp, [c_vp, ctypes.c_char]),
    "pm_hip_read_block": (None, [c_vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(c_vp)]),
    "pm_hip_total_mem": (ctypes.c_size_t, [c_vp]),
    "pm_hip_reset": (None, [c_vp]),
    "pm_hip_free": (None, [c_vp]),
    "pm_mps_hip_rt_register": (None, [c_vp]),
    "pm_mps_hip_ac_register": (None, [c_vp]),
    # batch / introspection
    "pm_hip_read_block_gid": (ctypes.c_int, [c_vp, c_u8p, ctypes.c_size_t, c_u32p]),
    "pm_hip_scan_device": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, c_vp,
                                          c_vp, c_vp]),
    "pm_hip_scan_device16": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, c_vp,
                                            c_vp, c_vp]),
    "pm_hip_score_device": (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_int64, c_vp, c_vp]),
    "pm_hip_parent_gid": (ctypes.c_uint32, [c_vp, ctypes.c_uint32]),
    "pm_hip_set_image_cache": (None, [c_vp, ctypes.c_char_p]),
    "pm_hip_image_cache_hit": (ctypes.c_int, [c_vp]),
    "pm_hip_serve_stats": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "pm_hip_compile_stats": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    "pm_hip_pattern_counts_device": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int64, c_vp, c_vp]),
    "pm_hip_gen_stream_device": (ctypes.c_int, [c_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                ctypes.c_int, c_vp]),
    "pm_gen_stream_host": (None, [c_u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int]),
    "pm_hip_gen_lines_device": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, ctypes.c_uint64, c_vp]),
    "pm_gen_lines_host": (None, [c_vp, c_u8p, ctypes.c_uint64, ctypes.c_uint64]),
    "pm_gen_lines_dict": (None, [PmDictP, c_u8p, ctypes.c_uint64, ctypes.c_uint64]),
    "pm_hip_n_patterns": (ctypes.c_uint32, [c_vp]),
    "pm_hip_max_pattern_len": (ctypes.c_uint32, [c_vp]),
    "pm_hip_gid_index": (ctypes.c_uint32, [c_vp, ctypes.c_uint32]),
    "pm_hip_kernel_kind": (ctypes.c_int, [c_vp]),
    "pm_hip_kernel_last": (ctypes.c_int, [c_vp]),
    "pm_hip_dfa_form_last": (ctypes.c_int, [c_vp]),
    "pm_hip_device_seconds": (ctypes.c_double, [c_vp]),
    "pm_hip_table_bytes": (ctypes.c_size_t, [c_vp]),
    "pm_hip_last_error": (ctypes.c_char_p, []),
    "pm_hip_device_count": (ctypes.c_int, []),
    "pm_hip_set_device": (ctypes.c_int, [ctypes.c_int]),
    "pm_hip_set_option": (ctypes.c_int, [c_vp, ctypes.c_char_p, ctypes.c_int64]),
    "pm_hip_streaming_floor_device": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int64, c_vp, ctypes.c_int, c_vp]),
    "pm_hip_gather_ceiling_device": (ctypes.c_int, [c_vp, ctypes.c_int, c_vp, c_vp]),
    "pm_hip_sparse_kernel_last": (ctypes.c_int, [c_vp]),
    # host-only table images
    "pm_flat_build": (c_vp, [ctypes.POINTER(ctypes.c_char_p), c_u32p, ctypes.c_size_t, ctypes.c_int]),
    "pm_flat_build_cached": (c_vp, [ctypes.POINTER(ctypes.c_char_p), c_u32p, ctypes.c_size_t, ctypes.c_int,
                                    ctypes.c_char_p]),
    "pm_flat_cache_hit": (ctypes.c_int, [c_vp]),
    "pm_flat_fits": (ctypes.c_int, [c_vp]),
    "pm_flat_dfa_sparse_rows": (ctypes.c_uint32, [c_vp]),
    "pm_flat_array": (ctypes.c_size_t, [c_vp, ctypes.c_char_p, ctypes.POINTER(c_vp),
                                        ctypes.POINTER(ctypes.c_size_t)]),
    "pm_flat_free": (None, [c_vp]),
    "pm_hip_last_out_width": (ctypes.c_int, [c_vp]),
    "pm_hip_hbm_peak_gbs": (ctypes.c_double, []),
    "pm_hip_hold_choice": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "pm_hip_prepare_capture": (ctypes.c_int, [c_vp]),
    "pm_hip_host_profile": (None, [ctypes.c_int, ctypes.POINTER(ctypes.c_double)]),
    "pm_hip_scratch_bytes": (ctypes.c_size_t, [c_vp]),
    "pm_flat_host_scan": (ctypes.c_int, [c_vp, c_u8p, ctypes.c_size_t, c_u32p, ctypes.c_int]),
}

_lib = None


def load():
    """Load libpm.so once; raise (never fall back) if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: PyTorch-ROCm bundles its own
    # libamdhip64.so (SONAME libamdhip64.so.7, NEEDED as "libamdhip64.so" by
    # libtorch_hip).  Loading torch first makes libpm.so's libamdhip64.so.7
    # resolve to that same runtime, so device pointers and streams are
    # shared; loading libpm.so first would pull /opt/rocm's copy and torch
    # would then load a second runtime and see no device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: run `make -C patternmatching_amd/csrc` "
                           "(or __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        if not hasattr(lib, name) and os.environ.get("PM_LIBPM"):
            continue  # an older build under A/B comparison (PM_LIBPM) may lack a newer entry point
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    lib.pm_mps_table_setup()
    _lib = lib
    return lib
