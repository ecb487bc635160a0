"""TEST-ONLY numpy emulation of the two scan kernels over the flattened
images (pm_flat_build), so the CPU suite can check the flattener byte for
byte before any GPU time.  Mirrors csrc/pm_kernels.hip's rt_one/rt_deep and
dfa_scan_kernel; never used by the product."""
import ctypes

import numpy as np

import patternmatching_amd as pm


class FlatImage:
    def __init__(self, patterns, kind):
        self.lib = pm.load()
        n = len(patterns)
        arr = (ctypes.c_char_p * n)(*patterns)
        lens = (ctypes.c_uint32 * n)(*[len(p) for p in patterns])
        self.h = self.lib.pm_flat_build(arr, lens, n, kind)
        self.kind = kind

    def fits(self):
        return bool(self.lib.pm_flat_fits(self.h))

    def array(self, name):
        data = ctypes.c_void_p()
        es = ctypes.c_size_t()
        n = self.lib.pm_flat_array(self.h, name.encode(), ctypes.byref(data), ctypes.byref(es))
        dt = {2: np.uint16, 4: np.uint32}[es.value] if es.value else np.uint32
        if n == 0:
            return np.zeros(0, dt)
        buf = (ctypes.c_char * (n * es.value)).from_address(data.value)
        return np.frombuffer(buf, dtype=dt).copy()

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.pm_flat_free(self.h)


def rt_scan(img, text, stream_start=0):
    """gids for every position of text (stream begins at stream_start)."""
    t12 = img.array("t12").astype(np.uint32)
    t3 = img.array("t3")
    b2 = img.array("b2")
    rec = img.array("rec").reshape(-1, 12)
    text = np.asarray(text, dtype=np.uint8)
    n = len(text)
    i = np.arange(n, dtype=np.int64)
    avail = i - stream_start + 1
    c0 = text.astype(np.uint32)
    c1 = np.concatenate([[0], text[:-1]]).astype(np.uint32)
    c2 = np.concatenate([[0, 0], text[:-2]]).astype(np.uint32)
    v = t12[(c0 << 8) | c1]
    out = v.copy()
    out[avail == 1] = t12[65536 + c0[avail == 1]]
    cont = (v & 0x8000) != 0
    m2 = cont & (avail == 2)
    out[m2] = b2[v[m2] & 0x7FFF]
    m3 = cont & (avail >= 3)
    r = t3[(v[m3] & 0x7FFF).astype(np.int64) * 256 + c2[m3]]
    out[m3] = r
    deep_pos = i[m3][(r & 0x80000000) != 0]
    for p in deep_pos:
        node = int(out[p]) & 0x7FFFFFFF
        d = 3
        while True:
            R = rec[node]
            if d >= avail[p]:
                out[p] = R[9]
                break
            c = int(text[p - d])
            w, bit = c >> 5, c & 31
            if not (int(R[w]) >> bit) & 1:
                out[p] = R[9]
                break
            pre = (int(R[10 + (w >> 2)]) >> (8 * (w & 3))) & 0xFF
            node = int(R[8]) + pre + bin(int(R[w]) & ((1 << bit) - 1)).count("1")
            d += 1
    return out


def dfa_scan(img, text):
    nxt = img.array("next")
    outt = img.array("out")
    s = 0
    res = np.empty(len(text), np.uint32)
    for j, c in enumerate(np.asarray(text, dtype=np.uint8).tolist()):
        s = int(nxt[s * 256 + c])
        res[j] = outt[s]
    return res


def gid_to_code(img, dictionary):
    idx = img.array("index_of_gid")
    codes = dictionary.codes()
    tab = np.zeros(len(idx), np.uint32)
    tab[1:] = codes[idx[1:]]
    return tab
