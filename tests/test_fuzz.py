"""Randomized dictionaries and streams against the oracle (the reference's
AC restated in C, pinned by the golden vectors): small alphabets for deep
walks and shared suffixes, pattern suffixes and extensions for nesting,
byte fans for wide trie nodes, duplicate and rejected lines for the parser,
every byte value.  CPU: the flattened images through the numpy emulation of
both kernels.  GPU: all three plugin kinds through read_block and the
device entry, bit-exact."""
import os

import numpy as np
import pytest

import patternmatching_amd as pm
from oracle_lib import Oracle

ALPHABETS = (2, 3, 4, 16, 95, 256)


def fuzz_case(seed, stream_bytes):
    rng = np.random.default_rng(1000 + seed)
    a = ALPHABETS[seed % len(ALPHABETS)]
    alphabet = rng.choice(256, size=a, replace=False).astype(np.uint8)
    n = (30, 300, 3000)[seed % 3]
    pats = []
    for _ in range(n):
        r = rng.random()
        if pats and r < 0.2:  # a suffix of an earlier pattern (nesting)
            p = pats[rng.integers(len(pats))]
            p = p[rng.integers(0, len(p)):]
        elif pats and r < 0.35:  # an extension (deep chains)
            p = pats[rng.integers(len(pats))] + bytes(rng.choice(alphabet, 1 + rng.geometric(0.3)))
        else:
            p = bytes(rng.choice(alphabet, min(1 + rng.geometric(0.12), 200)))
        pats.append(p[:200])
    if a >= 16:  # a wide reversed-trie node: many bytes before one suffix
        tail = bytes(rng.choice(alphabet, 3))
        pats += [bytes([c]) + tail for c in alphabet[:40]]
    lines = [b"|" + b" ".join(b"%02x" % c for c in p) + b"|" for p in pats if p]
    # the parser's rejections and skips (parser.c:63-99): they only shift line numbers
    for bad in (b"|41 |", b"|4|", b"|41", b""):
        lines.insert(int(rng.integers(len(lines) + 1)), bad)
    # the stream: runs of alphabet bytes and copies of patterns
    parts, size = [], 0
    while size < stream_bytes:
        if rng.random() < 0.5:
            q = pats[rng.integers(len(pats))]
        else:
            q = bytes(rng.choice(alphabet, int(rng.integers(1, 64))))
        parts.append(q)
        size += len(q)
    text = np.frombuffer(b"".join(parts)[:stream_bytes], np.uint8).copy()
    return b"\n".join(lines) + b"\n", text


def write_dict(tmp_path, seed, data):
    path = os.path.join(str(tmp_path), f"fuzz{seed}.dict")
    with open(path, "wb") as f:
        f.write(data)
    return path


@pytest.mark.parametrize("seed", range(12))
def test_fuzz_images_cpu(tmp_path, seed):
    """The RT image and both forms of the DFA image (emulated on the CPU)
    equal the oracle."""
    from table_emulator import FlatImage, dfa_scan, gid_to_code, rt_scan, sdfa_scan
    data, text = fuzz_case(seed, 6000)
    path = write_dict(tmp_path, seed, data)
    o = Oracle([path])
    o.reset()
    exp = o.scan_codes(text)
    d = pm.Dictionary([path])
    for kind in (pm.KIND_RT, pm.KIND_AC):
        img = FlatImage(d.patterns(), kind)
        if kind == pm.KIND_RT and not img.fits():
            continue
        tab = gid_to_code(img, d)
        got = tab[rt_scan(img, text)] if kind == pm.KIND_RT else tab[dfa_scan(img, text)]
        assert np.array_equal(got, exp), (seed, kind)
        if kind == pm.KIND_AC:
            assert np.array_equal(tab[sdfa_scan(img, text)], exp), (seed, "sparse")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(36))
def test_fuzz_gpu_all_kinds(tmp_path, seed):
    """read_block (in uneven calls) and scan_device of every plugin kind equal
    the oracle on 256 KiB streams."""
    import torch
    data, text = fuzz_case(seed, 256 << 10)
    path = write_dict(tmp_path, seed, data)
    o = Oracle([path])
    o.reset()
    exp = o.scan_codes(text)
    d = pm.Dictionary([path])
    for kind in ("rt", "ac", "auto"):
        m = pm.HipMatcher(kind)
        m.add_dictionary(d)
        m.compile()
        cuts = [0, 1, 777, 70001, len(text)]
        got = np.concatenate([m.read_block_codes(text[a:b]) for a, b in zip(cuts, cuts[1:])])
        assert np.array_equal(got, exp), (seed, kind, "read_block")
        s = torch.cuda.current_stream().cuda_stream
        dt = torch.from_numpy(np.concatenate([text, np.zeros(64, np.uint8)])).cuda()
        ids = torch.empty(len(text), dtype=torch.int32, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        m.scan_device(dt.data_ptr(), 0, 0, len(text), ids.data_ptr(), cnt.data_ptr(), s)
        torch.cuda.synchronize()
        assert np.array_equal(m._codes[ids.cpu().numpy().view(np.uint32)], exp), (seed, kind, "scan_device")
        assert int(cnt.item()) == int((exp != 0).sum())
        ids16 = torch.empty(len(text), dtype=torch.int16, device="cuda")
        m.scan_device(dt.data_ptr(), 0, 0, len(text), ids16.data_ptr(), None, s, out_width=2)
        cnt.zero_()
        m.scan_device(dt.data_ptr(), 0, 0, len(text), None, cnt.data_ptr(), s)  # count only
        torch.cuda.synchronize()
        assert torch.equal(ids16.to(torch.int32) & 0xFFFF, ids), (seed, kind, "u16")
        assert int(cnt.item()) == int((exp != 0).sum()), (seed, kind, "count only")
        m.free()
