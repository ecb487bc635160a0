"""ctypes wrapper of the oracle (oracle/ac_oracle.c).  TEST INFRASTRUCTURE:
only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it."""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(REPO, "oracle", "_build", "liboracle.so")
REF_DRIVER = os.path.join(REPO, "oracle", "_ref", "ref_driver")
GOLDEN = os.path.join(REPO, "tests", "golden")
DATA = os.path.join(GOLDEN, "data")

DICTS = {"et": ["et.dict"], "snort": ["snort.dict"], "merged": ["snort.dict", "et.dict"]}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
        L = ctypes.CDLL(ORACLE_SO)
        vp = ctypes.c_void_p
        L.oracle_ac_build.restype = vp
        L.oracle_ac_build.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int]
        for f in ("oracle_ac_n_states", "oracle_ac_n_patterns", "oracle_ac_max_len"):
            getattr(L, f).restype = ctypes.c_size_t
            getattr(L, f).argtypes = [vp]
        L.oracle_ac_reset.argtypes = [vp]
        L.oracle_ac_scan.argtypes = [vp, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.oracle_ac_scan_idx.argtypes = [vp, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.oracle_ac_pattern.restype = ctypes.c_uint32
        L.oracle_ac_pattern.argtypes = [vp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32),
                                        ctypes.POINTER(ctypes.c_uint32), ctypes.c_char_p, ctypes.c_uint32]
        L.oracle_parse_line.restype = ctypes.c_size_t
        L.oracle_parse_line.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
        L.oracle_ac_time_scan.restype = ctypes.c_double
        L.oracle_ac_time_scan.argtypes = [vp, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_ac_free.argtypes = [vp]
        L.oracle_fnv1a64.restype = ctypes.c_uint64
        L.oracle_fnv1a64.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        _lib = L
    return _lib


def dict_paths(key):
    return [os.path.join(DATA, d) for d in DICTS[key]]


class Oracle:
    """The reference's AC restated in C (oracle/ac_oracle.c)."""

    def __init__(self, paths):
        L = lib()
        arr = (ctypes.c_char_p * len(paths))(*[p.encode() for p in paths])
        self.h = L.oracle_ac_build(arr, len(paths))
        if not self.h:
            raise OSError(f"oracle could not load {paths}")
        self.n_states = L.oracle_ac_n_states(self.h)
        self.n_patterns = L.oracle_ac_n_patterns(self.h)
        self.max_len = L.oracle_ac_max_len(self.h)

    def reset(self):
        lib().oracle_ac_reset(self.h)

    def scan_codes(self, data):
        a = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data,
                                 dtype=np.uint8)
        out = np.empty(len(a), np.uint32)
        lib().oracle_ac_scan(self.h, a.ctypes.data, len(a), out.ctypes.data)
        return out

    def pattern(self, i):
        f, l = ctypes.c_uint32(), ctypes.c_uint32()
        buf = ctypes.create_string_buffer(4096)
        n = lib().oracle_ac_pattern(self.h, i, ctypes.byref(f), ctypes.byref(l), buf, 4096)
        return f.value, l.value, buf.raw[:n]

    def patterns(self):
        return [self.pattern(i) for i in range(self.n_patterns)]

    def time_scan(self, data, threads=1):
        a = np.ascontiguousarray(data, dtype=np.uint8)
        nn = ctypes.c_uint64()
        s = lib().oracle_ac_time_scan(self.h, a.ctypes.data, len(a), threads, ctypes.byref(nn))
        return s, nn.value

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_ac_free(self.h)
            self.h = None


def parse_line(line: bytes):
    out = ctypes.create_string_buffer(max(len(line), 1))
    n = lib().oracle_parse_line(line, len(line), out)
    return out.raw[:n] if n else None


_cache = {}


def oracle_for(key):
    if key not in _cache:
        _cache[key] = Oracle(dict_paths(key))
    return _cache[key]


def fnv1a64_codes(codes: np.ndarray) -> str:
    """FNV-1a-64 over the little-endian bytes of the u32 codes (ref_driver digest)."""
    b = np.ascontiguousarray(codes, dtype="<u4")
    return f"{lib().oracle_fnv1a64(b.ctypes.data, b.nbytes):016x}"
