"""TEST-ONLY numpy emulation of the two scan kernels over the flattened
images (pm_flat_build), so the CPU suite can check the flattener byte for
byte before any GPU time.  Mirrors csrc/pm_kernels.hip's rt_one/rt_deep and
dfa_scan_kernel; never used by the product."""
import ctypes

import numpy as np

import patternmatching_amd as pm


class FlatImage:
    def __init__(self, patterns, kind, cache_dir=None):
        self.lib = pm.load()
        n = len(patterns)
        arr = (ctypes.c_char_p * n)(*patterns)
        lens = (ctypes.c_uint32 * n)(*[len(p) for p in patterns])
        if cache_dir is None:
            self.h = self.lib.pm_flat_build(arr, lens, n, kind)
        else:
            self.h = self.lib.pm_flat_build_cached(arr, lens, n, kind, str(cache_dir).encode())
        self.kind = kind
        self.cache_hit = bool(self.lib.pm_flat_cache_hit(self.h))

    def fits(self):
        return bool(self.lib.pm_flat_fits(self.h))

    def array(self, name):
        data = ctypes.c_void_p()
        es = ctypes.c_size_t()
        n = self.lib.pm_flat_array(self.h, name.encode(), ctypes.byref(data), ctypes.byref(es))
        dt = {2: np.uint16, 4: np.uint32, 8: np.uint64}[es.value] if es.value else np.uint32
        if n == 0:
            return np.zeros(0, dt)
        buf = (ctypes.c_char * (n * es.value)).from_address(data.value)
        return np.frombuffer(buf, dtype=dt).copy()

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.pm_flat_free(self.h)


FILTER_WORDS = 4096


def rt_hash(k):
    """pm_rt_hash: key24 * 0x9E3779B1 mod 2^32 (t3h slots)."""
    return (np.asarray(k).astype(np.uint64) * np.uint64(0x9E3779B1)) & np.uint64(0xFFFFFFFF)


def filter_maybe(filt, key24):
    """pm_rt_fhash / pm_rt_filter_word / pm_rt_filter_mask: 3 bits per key."""
    f = (np.asarray(key24).astype(np.uint64) * np.uint64(0x9E3779)) & np.uint64(0xFFFFFFFF)
    w = filt[(f >> np.uint64(20)).astype(np.int64)].astype(np.uint64)
    m = np.zeros_like(f)
    for sh in (0, 8, 16):
        m |= np.uint64(1) << ((f >> np.uint64(sh)) & np.uint64(31))
    return (w & m) == m


def _bits(w, g):
    ok = np.ones(len(g), bool)
    for sh in (0, 8, 16):
        ok &= ((w >> ((g >> np.uint64(sh)) & np.uint64(31))) & np.uint64(1)) == 1
    return ok


def filter2_maybe(filt, key24, c3):
    """Stage 2 (pm_rt_p3hash / pm_rt_s4hash): a 3-byte pattern, or a depth-4
    suffix text[i-3..i]."""
    M = np.uint64(0xFFFFFFFF)
    f2 = filt[FILTER_WORDS:].astype(np.uint64)
    k = np.asarray(key24).astype(np.uint64)
    g3 = (k * np.uint64(0x85EBCA)) & M
    hit3 = _bits(f2[(g3 >> np.uint64(24)).astype(np.int64)], g3)
    k32 = (k << np.uint64(8)) | np.asarray(c3).astype(np.uint64)
    g4 = (k32 * np.uint64(0x9E3779B1)) & M
    w4 = f2[(256 + (((g4 >> np.uint64(20)) * np.uint64(7)) >> np.uint64(4))).astype(np.int64)]
    return hit3 | _bits(w4, g4)


def t3h_lookup(t3h, bits, key24):
    """The 4-word entry of key24 (cuckoo: slot1 or slot2), or None."""
    s1 = int(rt_hash(np.array([key24], np.uint32))[0]) >> (32 - bits)
    s2 = ((key24 * 0x85EBCA77) & 0xFFFFFFFF) >> (32 - bits)
    for slot in (s1, s2):
        e = t3h[4 * slot:4 * slot + 4]
        if int(e[0]) & 0x1FFFFFF == (1 << 24) | key24:
            return [int(x) for x in e]
    return None


def rec_walk(rec, wide, text, p, avail, node, d):
    """16-B node records (pm_flatten.h): leaf / one child and its run (chain)
    / up to 8 inline children / wide (4 quarters {word 2q, word 2q+1, first
    child index, best})."""
    while True:
        x, best, z, w = (int(v) for v in rec[node])
        if d >= avail:
            return best
        kind, cnt, first = x >> 30, (x >> 24) & 63, x & 0xFFFFFF
        c = int(text[p - d])
        if kind == 0:
            return best
        if kind == 2:  # chain: the run's bytes at once (pm_flatten.h)
            P = (w << 32) | z
            m = 0
            while m < cnt and d + m < avail and int(text[p - d - m]) == (P >> (8 * (7 - m))) & 0xFF:
                m += 1
            if m < cnt:
                return best  # stopped inside the run (or before it): no pattern there
            node, d = first + m - 1, d + m
            continue
        if kind == 1:
            kids = [((z | (w << 32)) >> (8 * j)) & 0xFF for j in range(cnt)]
            if c not in kids:
                return best
            node = first + kids.index(c)
        else:
            Q = [int(v) for v in wide[z][4 * (c >> 6):4 * (c >> 6) + 4]]  # {word 2q, word 2q+1, index, best}
            w = (c >> 5) & 1
            word = Q[w]
            if not (word >> (c & 31)) & 1:
                return Q[3]
            node = Q[2] + (bin(Q[0]).count("1") if w else 0) + bin(word & ((1 << (c & 31)) - 1)).count("1")
        d += 1


def rt_scan(img, text, stream_start=0, use_filter=True):
    """gids for every position of text (stream begins at stream_start)."""
    t12 = img.array("t12").astype(np.uint32)
    filt = img.array("filt")
    t3h = img.array("t3h")
    bits = int(len(t3h) // 4).bit_length() - 1
    rec = img.array("rec").reshape(-1, 4)
    wide = img.array("wide").reshape(-1, 16)
    text = np.asarray(text, dtype=np.uint8)
    n = len(text)
    i = np.arange(n, dtype=np.int64)
    avail = i - stream_start + 1
    c0 = text.astype(np.uint32)
    c1 = np.concatenate([[0], text[:-1]]).astype(np.uint32)
    c2 = np.concatenate([[0, 0], text[:-2]]).astype(np.uint32)
    v = t12[(c0 << 8) | c1]
    out = v & 0x7FFF
    out[avail == 1] = t12[65536 + c0[avail == 1]]
    key24 = c2 | (c1 << 8) | (c0 << 16)
    cont = ((v & 0x8000) != 0) & (avail >= 3)
    if use_filter:
        c3 = np.concatenate([[0, 0, 0], text[:-3]]).astype(np.uint32)
        cont &= filter_maybe(filt, key24) & filter2_maybe(filt, key24, c3)
    for p in i[cont]:
        e = t3h_lookup(t3h, bits, int(key24[p]))
        if e is None:
            continue  # best2 stays
        kind = e[0] >> 25
        if kind == 0 or avail[p] < 4:
            out[p] = e[1]
        elif kind == 1:
            nch = e[2] >> 24
            kids = [(e[2] >> (8 * k)) & 0xFF for k in range(nch)]
            c3 = int(text[p - 3])
            if c3 not in kids:
                out[p] = e[1]
            elif nch > 1:
                out[p] = rec_walk(rec, wide, text, p, avail[p], e[3] + kids.index(c3), 4)
            elif not e[3] & 0x80000000:
                out[p] = e[3]
            else:
                out[p] = rec_walk(rec, wide, text, p, avail[p], e[3] & 0x7FFFFFFF, 4)
        else:
            out[p] = rec_walk(rec, wide, text, p, avail[p], e[3] & 0x7FFFFFFF, 3)
    return out


def dfa_scan(img, text):
    """dfa_scan_kernel / dfa_coded_kernel: below 2^20 states a transition
    word is target | min(out[target], 4095) << 20 (pm_flatten.h); the code
    is checked against out[] at every step."""
    nxt = img.array("next")
    outt = img.array("out")
    coded = len(outt) <= 0xFFFFF
    s = 0
    res = np.empty(len(text), np.uint32)
    for j, c in enumerate(np.asarray(text, dtype=np.uint8).tolist()):
        x = int(nxt[s * 256 + c])
        s = x & 0xFFFFF if coded else x
        if coded:
            code = x >> 20
            assert code == min(int(outt[s]), 4095)
            res[j] = code if code != 4095 else outt[s]
        else:
            res[j] = outt[s]
    return res


def sdfa_scan(img, text):
    """dfa_sparse_kernel over the sparse form (pm_flatten.h): states below
    F have full rows; a record {x = (c0|0x100) | (c1|0x100) << 16, y, z,
    w = fallback} answers its two bytes and defers every other byte to row
    w.  The codes are checked against sout at every step."""
    F = int(img.lib.pm_flat_dfa_sparse_rows(img.h))
    blk = img.array("sblock")
    sout = img.array("sout")
    assert F >= 1 and len(blk) == F * 256 + (len(sout) - F) * 4
    rows = blk[: F * 256]
    rec = blk[F * 256:].reshape(-1, 4)
    s = 0
    res = np.empty(len(text), np.uint32)
    for j, c in enumerate(np.asarray(text, dtype=np.uint8).tolist()):
        if s < F:
            x = int(rows[s * 256 + c])
        else:
            R = rec[s - F]
            key = c | 0x100
            if int(R[0]) & 0x1FF == key:
                x = int(R[1])
            elif (int(R[0]) >> 16) & 0x1FF == key:
                x = int(R[2])
            else:
                assert int(R[3]) < F
                x = int(rows[int(R[3]) * 256 + c])
        s = x & 0xFFFFF
        code = x >> 20
        assert code == min(int(sout[s]), 4095)
        res[j] = code if code != 4095 else sout[s]
    return res


def sdfa8_scan(img, text):
    """dfa_sparse_lds_kernel<..., RB = 8> over the 8-B record units
    (pm_pack_sparse8, pm_flatten.h): rows as in the 16-B form; state F + u
    is the record at unit u -- {y, x0 | w << 9} with one or no slot, or
    {y, x | 1 << 31}, {z, w} with two, never straddling an aligned block of
    4 units (32 B; so neither one of 8).  Codes checked against sout8 at
    every step."""
    F = int(img.lib.pm_flat_dfa_sparse_rows(img.h))
    blk = img.array("sblock8")
    sout = img.array("sout8")
    assert F >= 1 and len(blk) == F * 256 + (len(sout) - F) * 2
    rows = blk[: F * 256]
    units = blk[F * 256:].reshape(-1, 2)
    s = 0
    res = np.empty(len(text), np.uint32)
    for j, c in enumerate(np.asarray(text, dtype=np.uint8).tolist()):
        if s < F:
            x = int(rows[s * 256 + c])
        else:
            u = s - F
            y, xw = int(units[u][0]), int(units[u][1])
            key = c | 0x100
            if xw & 0x1FF == key:
                x = y
            elif xw >> 31 and (xw >> 16) & 0x1FF == key:
                assert u % 4 != 3  # both units in one 32-B block
                x = int(units[u + 1][0])
            else:
                if xw >> 31:
                    assert u % 4 != 3
                    w = int(units[u + 1][1])
                else:
                    w = (xw >> 9) & 0x3FFFFF
                assert w < F
                x = int(rows[w * 256 + c])
        s = x & 0xFFFFF
        code = x >> 20
        assert code == min(int(sout[s]), 4095)
        res[j] = code if code != 4095 else sout[s]
    return res


def gid_to_code(img, dictionary):
    idx = img.array("index_of_gid")
    codes = dictionary.codes()
    tab = np.zeros(len(idx), np.uint32)
    tab[1:] = codes[idx[1:]]
    return tab
