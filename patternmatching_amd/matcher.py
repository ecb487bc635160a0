"""Python mirror of the plugin interface (include/pm_mps.h) over libpm.so.

Names and argument meaning follow the reference's MpsElem
(Core/src/mps.h:71-80) so tests read like the reference's own call order:

    d = Dictionary(["et.dict"])              # PatternsTree.c:260-312
    m = HipMatcher("rt")                     # mps_table[...].create()
    m.add_dictionary(d)                      # add_pattern per unique pattern
    m.compile()                              # flatten + upload to HBM
    codes = m.read_block_codes(stream_bytes) # == read_char per byte
    m.reset()                                # new stream file

Every scan goes through the HIP kernels; without a GPU, ``HipMatcher``
creation fails (the library exits, as the reference's FatalExit would).
"""
import ctypes

import numpy as np

from ._lib import load, PmPattern

KIND_RT = 1
KIND_AC = 2
KIND_AUTO = 3


def parse_line(line: bytes):
    """parser.c:63-99 via the library.  Returns the pattern bytes, or None
    when the line is rejected or empty."""
    lib = load()
    n = len(line)
    src = (ctypes.c_uint8 * max(n, 1)).from_buffer_copy(line or b"\0")
    dst = (ctypes.c_uint8 * max(n, 1))()
    k = lib.pm_parse_line(src, n, dst)
    return bytes(dst[:k]) if k else None


class Dictionary:
    """Unique patterns of the -d files, first occurrence wins."""

    def __init__(self, paths=None, patterns=None):
        self.lib = load()
        if paths is not None:
            arr = (ctypes.c_char_p * len(paths))(*[p.encode() for p in paths])
            err = ctypes.create_string_buffer(512)
            self.ptr = self.lib.pm_dict_load(arr, len(paths), err, 512)
            if not self.ptr:
                raise OSError(err.value.decode())
        else:
            self.ptr = self.lib.pm_dict_new()
            for k, p in enumerate(patterns or []):
                b = (ctypes.c_uint8 * max(len(p), 1)).from_buffer_copy(p or b"\0")
                self.lib.pm_dict_add(self.ptr, b, len(p), 0, k + 1)
            self.lib.pm_dict_finalize(self.ptr)
        d = self.ptr.contents
        self.n = d.n
        self.max_len = d.max_len
        self.lines_total = d.lines_total
        self.lines_rejected = d.lines_rejected

    def pattern(self, i):
        p = self.ptr.contents.pats[i]
        return p.file, p.line, ctypes.string_at(p.bytes, p.len)

    def pattern_ptr(self, i):
        """The pm_pattern_id_t of pattern i (address of its PmPattern)."""
        return ctypes.addressof(self.ptr.contents.pats[i])

    def patterns(self):
        return [self.pattern(i)[2] for i in range(self.n)]

    def codes(self):
        """u32 (file << 24 | line) per pattern index."""
        out = np.empty(self.n, dtype=np.uint32)
        pats = self.ptr.contents.pats
        for i in range(self.n):
            out[i] = (pats[i].file << 24) | pats[i].line
        return out

    def parents(self):
        """Index of the longest proper suffix that is a pattern, -1 if none."""
        base = ctypes.addressof(self.ptr.contents.pats[0]) if self.n else 0
        size = ctypes.sizeof(PmPattern)
        out = np.full(self.n, -1, dtype=np.int64)
        pats = self.ptr.contents.pats
        for i in range(self.n):
            par = pats[i].parent
            if par:
                out[i] = (ctypes.addressof(par.contents) - base) // size
        return out

    def gen_lines(self, n, seed) -> np.ndarray:
        """The lines stream of these patterns (pm_gen_lines_dict; the same
        bytes as HipMatcher.gen_lines of a matcher fed this dictionary)."""
        buf = np.empty(n, np.uint8)
        self.lib.pm_gen_lines_dict(self.ptr, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), n, seed)
        return buf

    def __del__(self):
        ptr = getattr(self, "ptr", None)
        if ptr:
            self.lib.pm_dict_free(ptr)
            self.ptr = None


def gen_stream(n, seed, mode=0, offset=0):
    """Synthetic stream, host implementation."""
    lib = load()
    buf = np.empty(n, dtype=np.uint8)
    lib.pm_gen_stream_host(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), offset, n, seed, mode)
    return buf


class HipMatcher:
    """One GPU matcher instance ("rt" = reverse-trie kernel, "ac" = AC DFA,
    "auto" = both, picked per launch)."""

    def __init__(self, kind="rt"):
        self.lib = load()
        self.kind_name = kind
        self.obj = getattr(self.lib, {"rt": "pm_hip_rt_create", "ac": "pm_hip_ac_create",
                                      "auto": "pm_hip_auto_create"}[kind])()
        self._codes = None
        self._dict = None

    # --- MpsElem -------------------------------------------------------
    def add_pattern(self, pat: bytes, pattern_id=None):
        self.lib.pm_hip_add_pattern(self.obj, pat, len(pat), pattern_id)

    def add_dictionary(self, d: Dictionary):
        fn = ctypes.cast(self.lib.pm_hip_add_pattern, ctypes.c_void_p)
        self.lib.pm_dict_feed(d.ptr, self.obj, fn)
        self._dict = d

    def compile(self):
        self.lib.pm_hip_compile(self.obj)
        if self._dict is not None:
            self._codes = self.gid_codes(self._dict.codes())

    def compile_stats(self):
        """Start-up cost of the last compile(): {"compile_ms", "upload_ms",
        "image_bytes", "image_cache_hit"} (pm_hip_compile_stats)."""
        c, u = ctypes.c_double(), ctypes.c_double()
        if self.lib.pm_hip_compile_stats(self.obj, ctypes.byref(c), ctypes.byref(u)) != 0:
            raise RuntimeError("compile_stats before compile()")
        return {"compile_ms": round(c.value, 2), "upload_ms": round(u.value, 2),
                "image_bytes": int(self.lib.pm_hip_table_bytes(self.obj)),
                "image_cache_hit": bool(self.lib.pm_hip_image_cache_hit(self.obj))}

    def serve_stats(self):
        """The resident small-call server of an rt object ("host_serve"):
        {"launches": grids launched, "calls": requests served}
        (pm_hip_serve_stats)."""
        la, ca = ctypes.c_uint64(), ctypes.c_uint64()
        self.lib.pm_hip_serve_stats(self.obj, ctypes.byref(la), ctypes.byref(ca))
        return {"launches": la.value, "calls": ca.value}

    def set_image_cache(self, directory: str):
        self.lib.pm_hip_set_image_cache(self.obj, directory.encode())

    def read_char(self, c: int):
        return self.lib.pm_hip_read_char(self.obj, bytes([c]))

    def read_block_ids(self, data: bytes):
        """pm_pattern_id_t per position (ints; 0 = null)."""
        n = len(data)
        out = (ctypes.c_void_p * max(n, 1))()
        self.lib.pm_hip_read_block(self.obj, data, n, out)
        return [x or 0 for x in out[:n]]

    def read_block_id_array(self, data) -> np.ndarray:
        """pm_hip_read_block into a numpy uintp array (pattern id per position)."""
        arr = np.ascontiguousarray(np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray)
                                   else data, dtype=np.uint8)
        out = np.empty(max(len(arr), 1), dtype=np.uintp)
        self.lib.pm_hip_read_block(self.obj, arr.ctypes.data_as(ctypes.c_char_p), len(arr),
                                   out.ctypes.data_as(ctypes.POINTER(ctypes.c_void_p)))
        return out[:len(arr)]

    def total_mem(self):
        return self.lib.pm_hip_total_mem(self.obj)

    def reset(self):
        self.lib.pm_hip_reset(self.obj)

    def free(self):
        if self.obj:
            self.lib.pm_hip_free(self.obj)
            self.obj = None

    def set_option(self, name: str, value: int) -> int:
        """pm_hip_set_option: a per-object option (include/pm_hip.h lists
        them); 0 on success, -1 for an unknown name or value."""
        return self.lib.pm_hip_set_option(self.obj, name.encode(), int(value))

    # --- batch ---------------------------------------------------------
    def read_block_gids(self, data) -> np.ndarray:
        arr = np.ascontiguousarray(np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray)
                                   else data, dtype=np.uint8)
        out = np.empty(len(arr), dtype=np.uint32)
        self.lib.pm_hip_read_block_gid(self.obj, arr.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), len(arr),
                                       out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
        return out

    def gid_codes(self, index_codes: np.ndarray) -> np.ndarray:
        """Table gid -> value, given a value per pattern index (add order)."""
        P = self.lib.pm_hip_n_patterns(self.obj)
        tab = np.zeros(P + 1, dtype=index_codes.dtype)
        for g in range(1, P + 1):
            tab[g] = index_codes[self.lib.pm_hip_gid_index(self.obj, g)]
        return tab

    def read_block_codes(self, data) -> np.ndarray:
        """(file << 24 | line) per position, the golden-fixture format."""
        return self._codes[self.read_block_gids(data)]

    def scan_device(self, d_text_ptr, stream_start, pos0, n, d_out_ptr, d_count_ptr, stream_ptr, out_width=4):
        """Device-resident scan (pm_hip_scan_device / _scan_device16): ids of
        out_width bytes (4 = u32, 2 = u16) to d_out_ptr, or count only."""
        fn = {4: self.lib.pm_hip_scan_device, 2: self.lib.pm_hip_scan_device16}[out_width]
        rc = fn(self.obj, d_text_ptr, stream_start, pos0, n, d_out_ptr, d_count_ptr, stream_ptr)
        if rc != 0:
            raise RuntimeError(self.lib.pm_hip_last_error().decode())

    def gen_lines_device(self, d_dst_ptr, n, seed, stream_ptr):
        """pm_hip_gen_lines_device: the lines stream (random dictionary
        patterns back to back, '\\n' after each) of this object's patterns."""
        rc = self.lib.pm_hip_gen_lines_device(self.obj, d_dst_ptr, n, seed, stream_ptr)
        if rc != 0:
            raise RuntimeError(self.lib.pm_hip_last_error().decode())

    def gen_lines(self, n, seed) -> np.ndarray:
        """The same bytes on the host (pm_gen_lines_host)."""
        buf = np.empty(n, np.uint8)
        self.lib.pm_gen_lines_host(self.obj, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), n, seed)
        return buf

    def score_device(self, d_algo_ptr, d_real_ptr, n, d_counts_ptr, stream_ptr):
        """pm_hip_score_device: d_counts (5 u64) += success, partial,
        false_neg, false_pos, all_matches of algo ids against real ids."""
        rc = self.lib.pm_hip_score_device(self.obj, d_algo_ptr, d_real_ptr, n, d_counts_ptr, stream_ptr)
        if rc != 0:
            raise RuntimeError(self.lib.pm_hip_last_error().decode())

    def pattern_counts_device(self, d_ids_ptr, n, d_hist_ptr, stream_ptr):
        """pm_hip_pattern_counts_device: d_hist (u64[n_patterns + 1], by gid)
        += occurrences of every pattern (suffix chains of the dense ids)."""
        rc = self.lib.pm_hip_pattern_counts_device(self.obj, d_ids_ptr, n, d_hist_ptr, stream_ptr)
        if rc != 0:
            raise RuntimeError(self.lib.pm_hip_last_error().decode())

    def hold_choice(self, launches):
        """pm_hip_hold_choice: keep the picked kernel for `launches` more
        scan_device launches (1 RT, 2 AC dense rows, 3 AC rows + records;
        0 = nothing to pick; -1 = still measuring)."""
        return self.lib.pm_hip_hold_choice(self.obj, launches)

    def prepare_capture(self):
        """pm_hip_prepare_capture: the scratch captured scan_device launches
        need, allocated before any stream capture begins."""
        if self.lib.pm_hip_prepare_capture(self.obj) != 0:
            raise RuntimeError(self.lib.pm_hip_last_error().decode())

    @property
    def scratch_bytes(self):
        return self.lib.pm_hip_scratch_bytes(self.obj)

    def parent_gid(self, gid):
        return self.lib.pm_hip_parent_gid(self.obj, gid)

    @property
    def kernel_kind(self):
        return self.lib.pm_hip_kernel_kind(self.obj)

    @property
    def dfa_form_last(self):
        """1 = dense rows, 2 = rows + records (pm_flatten.h), 0 = RT ran."""
        return self.lib.pm_hip_dfa_form_last(self.obj)

    @property
    def sparse_kernel_last(self):
        """The sparse form's kernel of the last launch that ran it
        ("sparse_kernel" numbering, 0 before any)."""
        return self.lib.pm_hip_sparse_kernel_last(self.obj)

    @property
    def kernel_last(self):
        """Kernel of the last launch: 1 = reverse trie, 2 = AC DFA."""
        return self.lib.pm_hip_kernel_last(self.obj)

    @property
    def max_pattern_len(self):
        return self.lib.pm_hip_max_pattern_len(self.obj)

    @property
    def table_bytes(self):
        return self.lib.pm_hip_table_bytes(self.obj)

    @property
    def device_seconds(self):
        """Device seconds of read_block's scans since reset(), or None when
        some of them were untimed (small calls with the "host_events" option
        off, its default: pm_hip_device_seconds returns -1)."""
        v = self.lib.pm_hip_device_seconds(self.obj)
        return None if v < 0 else v

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
