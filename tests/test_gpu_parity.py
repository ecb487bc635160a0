"""GPU parity: both HIP kernels, through the C-ABI, against the oracle and
the reference's golden vectors.  Bit-exact (integer ids per position)."""
import json
import os

import numpy as np
import pytest

import patternmatching_amd as pm
from oracle_lib import DATA, GOLDEN, dict_paths, fnv1a64_codes, oracle_for

pytestmark = pytest.mark.gpu

MANIFEST = json.load(open(os.path.join(GOLDEN, "manifest.json")))
SHIP = np.fromfile(os.path.join(DATA, "dictionaries_generated.stream"), dtype=np.uint8)
KINDS = ["rt", "ac", "auto"]
KIND_OF = {"rt": pm.KIND_RT, "ac": pm.KIND_AC, "auto": pm.KIND_AUTO}

_m = {}


def fresh_matcher(key, kind):
    """A new compiled object (never launched), not the cached one."""
    m = pm.HipMatcher(kind)
    m.add_dictionary(pm.Dictionary(dict_paths(key)))
    m.compile()
    return m


def matcher(key, kind):
    if (key, kind) not in _m:
        d = pm.Dictionary(dict_paths(key))
        m = pm.HipMatcher(kind)
        m.add_dictionary(d)
        m.compile()
        assert m.kernel_kind == KIND_OF[kind]
        _m[(key, kind)] = m
    m = _m[(key, kind)]
    m.reset()
    m.set_option("rt_small_max", _RT_SMALL[0])
    return m


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("key", ["et", "snort", "merged"])
def test_ship_stream_golden(key, kind):
    gold = np.fromfile(os.path.join(GOLDEN, f"ship_{key}.u32"), dtype="<u4")
    got = matcher(key, kind).read_block_codes(SHIP)
    bad = np.nonzero(got != gold)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at {bad[:5]}"


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("case", MANIFEST["digests"], ids=lambda d: f"{d['dict']}-s{d['seed']}-m{d['mode']}-n{d['n']}")
def test_seeded_digests(case, kind):
    m = matcher(case["dict"], kind)
    codes = m.read_block_codes(pm.gen_stream(case["n"], case["seed"], case["mode"]))
    assert int(np.count_nonzero(codes)) == case["nonnull"]
    nz = np.nonzero(codes)[0][:len(case["first"])]
    assert [[int(i), int(codes[i])] for i in nz] == case["first"]
    assert fnv1a64_codes(codes) == case["fnv1a64"]


@pytest.mark.parametrize("kind", KINDS)
def test_ship_x64_merged(kind):
    import hashlib
    codes = matcher("merged", kind).read_block_codes(np.tile(SHIP, 64))
    g = MANIFEST["ship_x64_merged"]
    assert int(np.count_nonzero(codes)) == g["nonnull"]
    assert hashlib.sha256(codes.astype("<u4").tobytes()).hexdigest() == g["sha256"]


@pytest.mark.parametrize("kind", KINDS)
def test_state_carries_across_read_block_calls(kind):
    """read_block == n read_char calls, state carried across calls
    (mps.h:41-42; measure.c:281-304 never resets between chunks)."""
    m = matcher("merged", kind)
    text = np.tile(SHIP, 4)
    whole = m.read_block_codes(text)
    m.reset()
    rng = np.random.default_rng(3)
    cuts = np.sort(rng.choice(np.arange(1, len(text)), size=40, replace=False))
    cuts = np.concatenate([[0], [1, 2, 3, 17, 346, 347, 348], cuts, [len(text)]])
    cuts = np.unique(cuts)
    parts = [m.read_block_codes(text[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
    assert np.array_equal(np.concatenate(parts), whole)


@pytest.mark.parametrize("kind", KINDS)
def test_read_block_pipeline_blocks(kind):
    """The host path pipelines 8 Mi-position blocks over two slots
    (pm_plugin.hip scan_host): a 20 MiB stream read in one call, and in calls
    cut around the block edges, equals one device-resident scan of it; the
    pattern-id form is the gid's add_pattern id."""
    import ctypes
    torch = _torch()
    m = matcher("merged", kind)
    n = (20 << 20) + 12345
    text = pm.gen_stream(n, 5, 0)
    dev = torch.from_numpy(np.concatenate([text, np.zeros(64, np.uint8)])).cuda()
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    m.scan_device(dev.data_ptr(), 0, 0, n, out.data_ptr(), cnt.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    exp = out.cpu().numpy().view(np.uint32)
    m.reset()
    assert np.array_equal(m.read_block_gids(text), exp)
    B = 8 << 20
    cuts = [0, 1, 7, B - 3, B + 5, 2 * B, 2 * B + 1, 2 * B + 100000, n - 2, n]
    m.reset()
    parts = [m.read_block_gids(text[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
    assert np.array_equal(np.concatenate(parts), exp)
    d = m._dict
    size = ctypes.sizeof(pm._lib.PmPattern)
    P = m.lib.pm_hip_n_patterns(m.obj)
    pid = m.gid_codes(np.uint64(d.pattern_ptr(0)) + np.arange(P, dtype=np.uint64) * np.uint64(size))
    m.reset()
    ids = m.read_block_id_array(text)
    assert np.array_equal(ids.astype(np.uint64), pid[exp])


@pytest.mark.parametrize("key", ["et", "merged"])
@pytest.mark.parametrize("kind", KINDS)
def test_read_char_per_byte(kind, key):
    """read_char (the host step over the object's images, pm_hoststep.h)
    over all 10,240 shipped bytes, interleaved with read_block calls of
    uneven sizes: the state carries both ways (mps.h:41-42), every position
    equals the reference's golden vector."""
    m = matcher(key, kind)
    gold = np.fromfile(os.path.join(GOLDEN, f"ship_{key}.u32"), dtype="<u4")
    got = np.zeros(len(SHIP), np.uint32)
    rng = np.random.default_rng(11)
    i = 0
    per_byte = 0
    while i < len(SHIP):
        if rng.random() < 0.5:  # a run of read_char calls
            k = min(len(SHIP) - i, int(rng.integers(1, 700)))
            for j in range(i, i + k):
                got[j] = m.lib.pm_pattern_code(m.read_char(int(SHIP[j])))
            per_byte += k
        else:  # a read_block of 0..900 bytes
            k = min(len(SHIP) - i, int(rng.integers(0, 900)))
            got[i:i + k] = m.read_block_codes(SHIP[i:i + k])
        i += k
    assert per_byte > len(SHIP) // 4
    bad = np.nonzero(got != gold)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at {bad[:5]}"
    m.reset()  # and after a reset, per byte from the stream start
    codes = [m.lib.pm_pattern_code(m.read_char(int(c))) for c in SHIP[:2000].tolist()]
    assert codes == gold[:2000].tolist()


@pytest.mark.parametrize("kind", KINDS)
def test_read_block_returns_pattern_ids(kind):
    """The ids handed to add_pattern come back verbatim (mps.h:35-37)."""
    m = matcher("et", kind)
    ids = m.read_block_ids(SHIP[:2000].tobytes())
    d = m._dict
    base = d.pattern_ptr(0)
    import ctypes
    size = ctypes.sizeof(pm._lib.PmPattern)
    gold = np.fromfile(os.path.join(GOLDEN, "ship_et.u32"), dtype="<u4")[:2000]
    codes = d.codes()
    for j, pid in enumerate(ids):
        if pid == 0:
            assert gold[j] == 0
        else:
            assert (pid - base) % size == 0
            assert codes[(pid - base) // size] == gold[j]


@pytest.mark.parametrize("kind", KINDS)
def test_duplicate_add_pattern_last_id_wins(kind):
    """add_pattern with a byte string already added: the later id is the one
    returned, as ac_add_pattern overwrites `cur->id` (mpac.c:272)."""
    m = pm.HipMatcher(kind)
    m.add_pattern(b"abc", 0x1000)
    m.add_pattern(b"bc", 0x2000)
    m.add_pattern(b"abc", 0x3000)
    m.compile()
    assert m.read_block_ids(b"xxabcxbc") == [0, 0, 0, 0, 0x3000, 0, 0, 0x2000]
    m.free()


_RT_SMALL = [-1]  # the "rt_small_max" option matcher() applies


@pytest.fixture(params=["chunked", "small"])
def rt_small(request):
    """RT launches of small sizes through the chunked kernel or the
    one-thread-per-position kernel (the per-object "rt_small_max" option:
    0 = never, 2^40 = every launch); all exact.  Yields the option value for
    matchers a test makes itself; matcher() applies it to the cached ones."""
    _RT_SMALL[0] = 0 if request.param == "chunked" else 1 << 40
    yield _RT_SMALL[0]
    _RT_SMALL[0] = -1
    for m in _m.values():
        m.set_option("rt_small_max", -1)


@pytest.mark.parametrize("kind", KINDS)
def test_empty_and_ragged_inputs(kind, rt_small):
    m = matcher("snort", kind)
    assert m.read_block_codes(b"").size == 0
    o = oracle_for("snort")
    text = pm.gen_stream(5000, seed=21, mode=0)
    o.reset()
    exp = o.scan_codes(text)
    for n in (1, 2, 3, 15, 16, 17, 31, 33, 1000, 4999):
        m.reset()
        assert np.array_equal(m.read_block_codes(text[:n]), exp[:n]), n


@pytest.mark.parametrize("kind", KINDS)
def test_kmp_kat(kind, rt_small):
    """Core/src/kmprt.c:303-326: AAAAAAAAAAAAAAAAAB matches at 17 and 42."""
    d = pm.Dictionary([os.path.join(DATA, "kmp_kat.dict")])
    m = pm.HipMatcher(kind)
    m.add_dictionary(d)
    m.compile()
    m.set_option("rt_small_max", rt_small)
    codes = m.read_block_codes(np.fromfile(os.path.join(DATA, "kmp_kat.stream"), dtype=np.uint8))
    assert list(np.nonzero(codes)[0]) == [17, 42]
    m.free()


EDGE_DICTS = {
    "one_byte": [b"a"],
    "nul_high": [b"\x00", b"\xff\x00", b"\x00\x00\x00", b"\x80\x81\x82\x83"],
    "nested": [b"abcdef", b"cdef", b"ef", b"f", b"zzzzzzzzzz", b"zz"],
    "dense_short": [bytes([i]) for i in range(256)] + [bytes([i, j]) for i in range(0, 256, 7) for j in range(0, 256, 5)],
    "long": [bytes(range(40, 240)), bytes(range(40, 240))[100:], b"x" * 300, b"x" * 299 + b"y"],
    # the RT image's limit (max_len <= 511, pm_flatten.cpp) and one past it
    # (the RT and auto kinds then run the AC-DFA kernel alone)
    "max_len_511": [b"ab" * 255 + b"a", b"ba" * 100, b"q"],
    "max_len_600": [b"ab" * 300, b"ba" * 100, b"q"],
}


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("name", list(EDGE_DICTS))
def test_edge_dictionaries_brute_force(name, kind, rt_small):
    pats = EDGE_DICTS[name]
    d = pm.Dictionary(patterns=pats)
    m = pm.HipMatcher(kind)
    m.add_dictionary(d)
    m.compile()
    m.set_option("rt_small_max", rt_small)
    rng = np.random.default_rng(9)
    alphabet = np.unique(np.frombuffer(b"".join(pats), np.uint8))
    text = rng.choice(alphabet, size=20000).astype(np.uint8)
    if name.startswith("max_len"):
        for k in range(2000, 18000, 1500):  # long alternating runs: the whole patterns occur
            text[k:k + 700] = np.frombuffer(b"ab" * 350, np.uint8)
    if name == "long":
        text[5000:5200] = np.frombuffer(bytes(range(40, 240)), np.uint8)
        text[8000:8300] = ord("x")
        text[9000:9299] = ord("x")
        text[9299] = ord("y")
    codes = {}
    for i in range(d.n):
        f, l, b = d.pattern(i)
        codes[b] = (f << 24) | l
    L = max(map(len, pats))
    tb = text.tobytes()
    exp = np.zeros(len(tb), np.uint32)
    for i in range(len(tb)):
        for k in range(min(L, i + 1), 0, -1):
            c = codes.get(tb[i + 1 - k:i + 1])
            if c is not None:
                exp[i] = c
                break
    got = m.read_block_codes(text)
    assert np.array_equal(got, exp)
    m.free()


def _torch():
    torch = pytest.importorskip("torch")
    assert torch.cuda.is_available()
    return torch


@pytest.mark.parametrize("kind", KINDS)
def test_device_generator_matches_host(kind):
    torch = _torch()
    n = (1 << 20) + 13
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    lib = pm.load()
    assert lib.pm_hip_gen_stream_device(d.data_ptr(), 12345, n, 77, 0 if kind == "rt" else 1,
                                        torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), pm.gen_stream(n, 77, 0 if kind == "rt" else 1, offset=12345))


@pytest.mark.parametrize("kind", KINDS)
def test_scan_device_shards_with_context(kind, rt_small):
    """Shard exactness: a shard scanned with max_len-1 bytes of context equals
    the same positions of one whole-stream scan."""
    torch = _torch()
    m = matcher("merged", kind)
    text = np.tile(SHIP, 40)  # adversarial: deep states everywhere
    whole = m.read_block_gids(text)
    W = m.max_pattern_len - 1
    dt = torch.from_numpy(np.concatenate([text, np.zeros(64, np.uint8)])).cuda()
    s = torch.cuda.current_stream().cuda_stream
    for a, b in ((0, 10240), (4096, 50000), (10240 * 7 + 16 * 5, 10240 * 39), (len(text) - 4000, len(text))):
        a16 = a - a % 16
        out = torch.zeros(b - a16, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        m.scan_device(dt.data_ptr(), max(0, a16 - W), a16, b - a16, out.data_ptr(), cnt.data_ptr(), s)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        assert np.array_equal(got, whole[a16:b]), (a, b)
        assert int(cnt.item()) == int(np.count_nonzero(whole[a16:b]))
    # too little context is detectably wrong on this adversarial stream (W = 346 matters)
    wrong = 0
    for a in range(10240, 10240 * 30, 10240 + 32):
        a -= a % 16
        out = torch.zeros(512, dtype=torch.int32, device="cuda")
        m.scan_device(dt.data_ptr(), a, a, 512, out.data_ptr(), None, s)
        torch.cuda.synchronize()
        wrong += int(np.count_nonzero(out.cpu().numpy().view(np.uint32) != whole[a:a + 512]))
    assert wrong > 0


@pytest.mark.parametrize("kind", KINDS)
def test_count_only_mode(kind):
    torch = _torch()
    m = matcher("snort", kind)
    n = 3_000_017
    dt = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    pm.load().pm_hip_gen_stream_device(dt.data_ptr(), 0, n + 64, 5, 0, s)
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    c1 = torch.zeros(1, dtype=torch.int64, device="cuda")
    c2 = torch.zeros(1, dtype=torch.int64, device="cuda")
    m.scan_device(dt.data_ptr(), 0, 0, n, out.data_ptr(), c1.data_ptr(), s)
    m.scan_device(dt.data_ptr(), 0, 0, n, None, c2.data_ptr(), s)
    torch.cuda.synchronize()
    assert int(c1.item()) == int(c2.item()) == int((out != 0).sum().item())
    o = oracle_for("snort")
    o.reset()
    exp = o.scan_codes(dt[:n].cpu().numpy())
    assert np.array_equal(m._codes[out.cpu().numpy().view(np.uint32)], exp)


@pytest.mark.parametrize("kind", KINDS)
def test_u16_ids_equal_u32_ids(kind):
    """pm_hip_scan_device16: the compact id stream is the u32 one, narrowed,
    on random text and on the adversarial tiling (deep walks, dense queue),
    including unaligned tails and context-only heads."""
    torch = _torch()
    s = torch.cuda.current_stream().cuda_stream
    m = matcher("merged", kind)
    rnd = pm.gen_stream(3_000_017, 9, 0)
    adv = np.tile(SHIP, 30)
    for text in (rnd, adv):
        n = len(text)
        dt = torch.from_numpy(np.concatenate([text, np.zeros(64, np.uint8)])).cuda()
        for pos0, ss in ((0, 0), (4096, 4096 - (m.max_pattern_len - 1)), (4096, 4096)):
            ss = max(ss, 0)
            w = n - pos0
            a = torch.zeros(w, dtype=torch.int32, device="cuda")
            b = torch.full((w + 8,), 0x7777, dtype=torch.int16, device="cuda")
            ca = torch.zeros(1, dtype=torch.int64, device="cuda")
            cb = torch.zeros(1, dtype=torch.int64, device="cuda")
            m.scan_device(dt.data_ptr(), ss, pos0, w, a.data_ptr(), ca.data_ptr(), s)
            m.scan_device(dt.data_ptr(), ss, pos0, w, b.data_ptr(), cb.data_ptr(), s, out_width=2)
            torch.cuda.synchronize()
            a32 = a.cpu().numpy().view(np.uint32)
            b16 = b.cpu().numpy().view(np.uint16)
            assert a32.max() < 65536
            assert np.array_equal(b16[:w].astype(np.uint32), a32), (n, pos0, ss)
            assert np.all(b16[w:] == 0x7777)  # nothing written past n
            assert int(ca.item()) == int(cb.item()) == int(np.count_nonzero(a32))
    o = oracle_for("merged")
    o.reset()
    exp = o.scan_codes(rnd[:1 << 20])
    b = torch.zeros(1 << 20, dtype=torch.int16, device="cuda")
    dt = torch.from_numpy(np.concatenate([rnd, np.zeros(64, np.uint8)])).cuda()
    m.scan_device(dt.data_ptr(), 0, 0, 1 << 20, b.data_ptr(), None, s, out_width=2)
    torch.cuda.synchronize()
    assert np.array_equal(m._codes[b.cpu().numpy().view(np.uint16).astype(np.uint32)], exp)


def test_image_cache_compile_scans_identically(tmp_path):
    """compile() through the image cache: the second object loads the file
    and its scan is identical."""
    torch = _torch()
    s = torch.cuda.current_stream().cuda_stream
    d = pm.Dictionary(dict_paths("snort"))
    outs = []
    for k in range(2):
        m = pm.HipMatcher("rt")
        m.lib.pm_hip_set_image_cache(m.obj, str(tmp_path).encode())
        m.add_dictionary(d)
        m.compile()
        assert m.lib.pm_hip_image_cache_hit(m.obj) == k
        text = np.tile(SHIP, 8)
        outs.append(m.read_block_gids(text))
    assert np.array_equal(outs[0], outs[1])


def test_u16_ids_refused_for_large_dictionaries():
    torch = _torch()
    pats = [b"%05dxq" % k for k in range(70000)]
    m = pm.HipMatcher("rt")
    m.add_dictionary(pm.Dictionary(patterns=pats))
    m.compile()
    dt = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    b = torch.zeros(4096, dtype=torch.int16, device="cuda")
    with pytest.raises(RuntimeError, match="65536"):
        m.scan_device(dt.data_ptr(), 0, 0, 4096, b.data_ptr(), None, torch.cuda.current_stream().cuda_stream,
                      out_width=2)


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("key", ["snort", "70k"])
def test_small_gid_calls_u16_and_u32(kind, key):
    """Small read_block_gid calls (<= 256 Ki positions) bring u16 gids over
    the link and widen them on the host when every gid fits, u32 otherwise
    (a 70,000-pattern dictionary), with or without the per-call timing
    events (the "host_gid16" / "host_events" options), their results
    copied / mapped on the host pool or by the caller alone ("host_pool"):
    every form equals one large call, for gids and pattern ids."""
    if key == "snort":
        m = matcher("snort", kind)
        text = np.tile(SHIP, 1 + (600 << 10) // len(SHIP))[:600 << 10]
    else:
        pats = [b"%05dxq" % k for k in range(70000)]
        m = pm.HipMatcher(kind)
        m.add_dictionary(pm.Dictionary(patterns=pats))
        m.compile()
        rng = np.random.default_rng(3)
        text = np.frombuffer(b"".join(pats[k] for k in rng.integers(0, 70000, size=90000)), np.uint8).copy()
    m.reset()
    whole = m.read_block_gids(text)  # > 256 Ki positions: u32 straight into the caller's array
    if key == "70k":
        assert whole.max() >= 65536
    m.reset()
    whole_ids = m.read_block_id_array(text)
    try:
        for gid16, ev, pool in ((1, 0, -1), (0, 0, -1), (1, 1, -1), (0, 1, 0), (1, 0, 0)):
            assert m.set_option("host_gid16", gid16) == 0 and m.set_option("host_events", ev) == 0
            assert m.set_option("host_pool", pool) == 0  # the result copy / id map on the host pool, or not
            m.reset()
            parts = [m.read_block_gids(text[o:o + (100 << 10)]) for o in range(0, len(text), 100 << 10)]
            assert np.array_equal(np.concatenate(parts), whole), (gid16, ev, pool)
            m.reset()
            ids = [m.read_block_id_array(text[o:o + (100 << 10)]) for o in range(0, len(text), 100 << 10)]
            assert np.array_equal(np.concatenate(ids), whole_ids), (gid16, ev, pool)
    finally:
        for k in ("host_gid16", "host_events", "host_pool"):
            m.set_option(k, -1)
    if key == "70k":
        m.free()


@pytest.mark.parametrize("kind", KINDS)
def test_small_calls_changing_sizes(kind):
    """Small read_block calls of repeated, changing and returning sizes --
    ragged ends, 1-byte calls, 255 Ki calls -- with and without the
    per-call timing events ("host_events"; pm_hip_device_seconds is -1
    after an untimed call and a total after timed ones) give the ids of one
    large call, for gids and pattern ids; an option set between calls
    changes which kernel the next launches take, not their ids."""
    m = matcher("snort", kind)
    sizes = [100 << 10] * 6 + [37 << 10] * 3 + [100 << 10] * 3 + [1, 1, 255 << 10, 255 << 10, 5000]
    text = np.tile(SHIP, 1 + sum(sizes) // len(SHIP))[:sum(sizes)]
    offs = np.cumsum([0] + sizes)
    m.reset()
    whole = m.read_block_gids(text)
    m.reset()
    whole_ids = m.read_block_id_array(text)
    try:
        for ev in (1, 0):
            assert m.set_option("host_events", ev) == 0
            m.reset()
            parts = [m.read_block_gids(text[a:b]) for a, b in zip(offs[:-1], offs[1:])]
            assert np.array_equal(np.concatenate(parts), whole), ev
            assert (m.device_seconds > 0) if ev else (m.device_seconds is None and m.lib.pm_hip_device_seconds(m.obj) == -1.0)
            m.reset()
            ids = [m.read_block_id_array(text[a:b]) for a, b in zip(offs[:-1], offs[1:])]
            assert np.array_equal(np.concatenate(ids), whole_ids), ev
        m.reset()
        parts = [m.read_block_gids(text[a:b]) for a, b in zip(offs[:7], offs[1:8])]
        if kind == "rt":
            assert m.set_option("rt_small_max", 0) == 0  # the chunked RT kernel from here on
        else:
            assert m.set_option("dfa_form", 2) == 0 and m.set_option("sparse_kernel", 2) == 0
        parts += [m.read_block_gids(text[a:b]) for a, b in zip(offs[7:-1], offs[8:])]
        assert np.array_equal(np.concatenate(parts), whole)
        if kind == "ac":
            assert m.sparse_kernel_last == 2
    finally:
        for k, v in (("host_events", -1), ("rt_small_max", -1), ("dfa_form", 0), ("sparse_kernel", 0)):
            m.set_option(k, v)


def _score_host(algo, real, parent, depth):
    """measure_success_rate (Core/src/measure.c:174-190) + all-matches, numpy."""
    algo = algo.astype(np.int64)
    real = real.astype(np.int64)
    eq = algo == real
    fn = ~eq & (algo == 0)
    part = 0
    for i in np.nonzero(~eq & (algo != 0))[0]:
        cur = real[i]
        while cur and cur != algo[i]:
            cur = parent[cur]
        part += cur != 0
    fp = int(np.count_nonzero(~eq & (algo != 0))) - part
    return [int(eq.sum()), part, int(fn.sum()), fp, int(depth[real].sum())]


@pytest.mark.parametrize("key", ["snort", "merged"])
def test_score_device_matches_measure_success_rate(key):
    """pm_hip_score_device == the reference's scoring (numpy restatement over
    the patterns-tree parents) on RT vs AC ids (all success) and on ids with
    injected partial / false-negative / false-positive answers."""
    torch = _torch()
    s = torch.cuda.current_stream().cuda_stream
    rt, ac = matcher(key, "rt"), matcher(key, "ac")
    n = (4 << 20) + 12
    dt = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    pm.load().pm_hip_gen_stream_device(dt.data_ptr(), 0, n + 64, 21, 0, s)
    a = torch.empty(n + 4, dtype=torch.int32, device="cuda")
    b = torch.empty(n + 4, dtype=torch.int32, device="cuda")
    rt.scan_device(dt.data_ptr(), 0, 0, n, a.data_ptr(), None, s)
    ac.scan_device(dt.data_ptr(), 0, 0, n, b.data_ptr(), None, s)
    torch.cuda.synchronize()
    P = rt.lib.pm_hip_n_patterns(rt.obj)
    parent = np.array([rt.parent_gid(g) for g in range(P + 1)], np.int64)
    depth = np.zeros(P + 1, np.int64)
    for g in range(1, P + 1):  # patterns on g's suffix chain, g included
        c, k = g, 0
        while c:
            c, k = parent[c], k + 1
        depth[g] = k
    real = b[:n].cpu().numpy().view(np.uint32)
    cnt = torch.zeros(5, dtype=torch.int64, device="cuda")
    rt.score_device(a.data_ptr(), b.data_ptr(), n, cnt.data_ptr(), s)
    torch.cuda.synchronize()
    exp = _score_host(a[:n].cpu().numpy().view(np.uint32), real, parent, depth)
    assert cnt.cpu().tolist() == exp and exp[0] == n
    # injected errors: partial (a proper suffix pattern), false negatives, false positives
    algo = real.copy()
    rng = np.random.default_rng(3)
    withpar = np.nonzero(parent[real] > 0)[0]
    sel = rng.choice(withpar, 5000, replace=False)
    algo[sel] = parent[real[sel]]
    nz = np.nonzero(real)[0]
    algo[rng.choice(nz, 4000, replace=False)] = 0
    fpi = rng.choice(n, 3000, replace=False)
    algo[fpi] = rng.integers(1, P + 1, 3000)
    ad = torch.from_numpy(np.concatenate([algo, np.zeros(4, np.uint32)]).view(np.int32)).cuda()
    cnt.zero_()
    rt.score_device(ad.data_ptr(), b.data_ptr(), n, cnt.data_ptr(), s)
    torch.cuda.synchronize()
    exp = _score_host(algo, real, parent, depth)
    got = cnt.cpu().tolist()
    assert got == exp, (got, exp)
    assert exp[1] > 1000 and exp[2] > 1000 and exp[3] > 1000


@pytest.mark.parametrize("key", ["snort", "merged"])
def test_pattern_counts_device(key):
    """pm_hip_pattern_counts_device == numpy all-matches expansion over the
    parent chains (merged needs two LDS windows of gids)."""
    torch = _torch()
    s = torch.cuda.current_stream().cuda_stream
    rt = matcher(key, "rt")
    n = (2 << 20) + 7
    dt = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    pm.load().pm_hip_gen_stream_device(dt.data_ptr(), 0, n + 64, 23, 0, s)
    ids = torch.empty(n + 4, dtype=torch.int32, device="cuda")
    rt.scan_device(dt.data_ptr(), 0, 0, n, ids.data_ptr(), None, s)
    P = rt.lib.pm_hip_n_patterns(rt.obj)
    hist = torch.zeros(P + 1, dtype=torch.int64, device="cuda")
    rt.pattern_counts_device(ids.data_ptr(), n, hist.data_ptr(), s)
    torch.cuda.synchronize()
    parent = np.array([rt.parent_gid(g) for g in range(P + 1)], np.int64)
    exp = np.zeros(P + 1, np.int64)
    cur = ids[:n].cpu().numpy().view(np.uint32).astype(np.int64)
    while cur.any():
        cur = cur[cur > 0]
        np.add.at(exp, cur, 1)
        cur = parent[cur]
    got = hist.cpu().numpy()
    assert np.array_equal(got, exp)
    assert got.sum() > n // 2 and (got > 0).sum() > 1000


@pytest.mark.slow
def test_full_size_snort_1gib_kernels_agree():
    """BASELINE config 3 size (snort, 1 GiB): the two independent kernels agree
    position by position, and sampled windows match the oracle."""
    torch = _torch()
    rt, ac = matcher("snort", "rt"), matcher("snort", "ac")
    n = 1 << 30
    s = torch.cuda.current_stream().cuda_stream
    dt = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    pm.load().pm_hip_gen_stream_device(dt.data_ptr(), 0, n + 64, 1, 0, s)
    a = torch.empty(n, dtype=torch.int32, device="cuda")
    b = torch.empty(n, dtype=torch.int32, device="cuda")
    ca = torch.zeros(1, dtype=torch.int64, device="cuda")
    cb = torch.zeros(1, dtype=torch.int64, device="cuda")
    rt.scan_device(dt.data_ptr(), 0, 0, n, a.data_ptr(), ca.data_ptr(), s)
    ac.scan_device(dt.data_ptr(), 0, 0, n, b.data_ptr(), cb.data_ptr(), s)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert int(ca.item()) == int(cb.item()) == int((a != 0).sum().item())
    c = torch.empty(n, dtype=torch.int16, device="cuda")  # the bench's compact id stream
    rt.scan_device(dt.data_ptr(), 0, 0, n, c.data_ptr(), None, s, out_width=2)
    torch.cuda.synchronize()
    assert torch.equal(c.to(torch.int32) & 0xFFFF, a)
    del c
    o = oracle_for("snort")
    W = o.max_len - 1
    rng = np.random.default_rng(0)
    for off in rng.integers(W, n - 100000, size=6).tolist() + [n - 70000]:
        o.reset()
        seg = dt[off - W:off + 65536].cpu().numpy()
        exp = o.scan_codes(seg)[W:]
        got = rt._codes[a[off:off + 65536].cpu().numpy().view(np.uint32)]
        assert np.array_equal(got, exp), off
    del a, b, dt
    torch.cuda.empty_cache()


@pytest.mark.slow
def test_full_size_merged_4gib_kernels_agree():
    """BASELINE config 5 size (snort + et merged, 4 GiB: four 1 GiB launches
    of the RT kernel, pm_kernels.hip launch_rt_impl): the two independent
    kernels agree at every position, and oracle windows (each with max_len-1
    bytes of context) match at the 2^30-position seams between the launches
    -- where the shipped stream is pasted in, so deep walks cross them --
    at random offsets and at both ends."""
    torch = _torch()
    rt, ac = matcher("merged", "rt"), matcher("merged", "ac")
    n = 4 << 30
    s = torch.cuda.current_stream().cuda_stream
    dt = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    pm.load().pm_hip_gen_stream_device(dt.data_ptr(), 0, n + 64, 5, 0, s)
    ship = torch.from_numpy(np.tile(SHIP, 2)).cuda()
    seams = [k << 30 for k in (1, 2, 3)]
    for sm in seams:  # deep matches straddling each launch seam
        dt[sm - 10000:sm - 10000 + ship.numel()] = ship
    a = torch.empty(n, dtype=torch.int32, device="cuda")
    b = torch.empty(n, dtype=torch.int32, device="cuda")
    ca = torch.zeros(1, dtype=torch.int64, device="cuda")
    cb = torch.zeros(1, dtype=torch.int64, device="cuda")
    rt.scan_device(dt.data_ptr(), 0, 0, n, a.data_ptr(), ca.data_ptr(), s)
    ac.scan_device(dt.data_ptr(), 0, 0, n, b.data_ptr(), cb.data_ptr(), s)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert int(ca.item()) == int(cb.item())
    assert int(ca.item()) > 0.95 * n  # merged: ~99 % of ASCII positions match something
    del b
    o = oracle_for("merged")
    W = o.max_len - 1
    rng = np.random.default_rng(1)
    windows = [sm - 32768 for sm in seams] + rng.integers(W, n - 100000, size=4).tolist() + [0, n - 65536]
    for off in windows:
        lo = max(0, off - W)
        o.reset()
        seg = dt[lo:off + 65536].cpu().numpy()
        exp = o.scan_codes(seg)[off - lo:]
        got = rt._codes[a[off:off + 65536].cpu().numpy().view(np.uint32)]
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, (off, bad[:5])
    del a, dt
    torch.cuda.empty_cache()


@pytest.mark.slow
@pytest.mark.parametrize("stream", ["lines", "ship"])
def test_full_size_merged_deep_auto_oracle_windows(stream):
    """The reference's published dictionary (snort + et merged, results.csv:
    2-4) on deep input at 1 GiB through the auto kind -- the bench's
    merged_lines_auto and merged_ship_auto legs, seed 1: once the pick holds
    (the measured RT launch, then the DFA trials) the held kernel's ids equal
    the RT kernel's at every position, its count is the nonzero ids', and
    oracle windows (each with max_len-1 bytes of context) match at random
    offsets, at the held DFA kernel's segment starts (4 KiB apart at this
    size: warm-ups from the last synchronizing 3-gram) and at both ends."""
    torch = _torch()
    rt, au = matcher("merged", "rt"), matcher("merged", "auto")
    n = 1 << 30
    s = torch.cuda.current_stream().cuda_stream
    dt = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    if stream == "lines":
        au.gen_lines_device(dt.data_ptr(), n + 64, 1, s)
    else:
        dt.copy_(torch.from_numpy(np.tile(SHIP, (n + 64) // len(SHIP) + 1)[: n + 64]).cuda())
    ref = torch.empty(n, dtype=torch.int32, device="cuda")
    rt.scan_device(dt.data_ptr(), 0, 0, n, ref.data_ptr(), None, s)
    a = torch.empty(n, dtype=torch.int32, device="cuda")
    c = torch.zeros(1, dtype=torch.int64, device="cuda")
    held = au.hold_choice(0)
    for _ in range(16):  # the pick: launches synchronized one by one until it holds
        if held != -1:
            break
        au.scan_device(dt.data_ptr(), 0, 0, n, a.data_ptr(), None, s)
        torch.cuda.synchronize()
        held = au.hold_choice(0)
    held = au.hold_choice(2)
    assert held in (1, 2, 3, 4, 5, 6)
    a.zero_()
    au.scan_device(dt.data_ptr(), 0, 0, n, a.data_ptr(), c.data_ptr(), s)
    torch.cuda.synchronize()
    assert torch.equal(a, ref), held
    assert int(c.item()) == int((ref != 0).sum().item())
    if stream == "lines":  # deep, no period: a DFA form holds
        assert au.kernel_last == 2, held
    del ref
    o = oracle_for("merged")
    W = o.max_len - 1
    rng = np.random.default_rng(2)
    windows = (rng.integers(W, n - 100000, size=4).tolist() + [k * 4096 - 96 for k in (1, 4097, 131073, 262000)]
               + [0, n - 65536])
    for off in windows:
        lo = max(0, off - W)
        o.reset()
        seg = dt[lo:off + 65536].cpu().numpy()
        exp = o.scan_codes(seg)[off - lo:]
        got = au._codes[a[off:off + 65536].cpu().numpy().view(np.uint32)]
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, (off, held, bad[:5])
    del a, dt
    torch.cuda.empty_cache()


@pytest.mark.slow
@pytest.mark.parametrize("stream", ["bytes", "ship"])
def test_full_size_binary_and_deep_streams_kernels_agree(stream):
    """1 GiB of uniform bytes (every byte value, snort's binary patterns) and
    the shipped adversarial stream tiled to 1 GiB (26% of positions spill to
    the deep-walk tail): RT, AC and the auto kind agree at every position."""
    torch = _torch()
    rt, ac, au = matcher("snort", "rt"), matcher("snort", "ac"), matcher("snort", "auto")
    n = 1 << 30
    s = torch.cuda.current_stream().cuda_stream
    dt = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    if stream == "bytes":
        pm.load().pm_hip_gen_stream_device(dt.data_ptr(), 0, n + 64, 7, 1, s)
    else:
        ship = torch.from_numpy(SHIP).cuda()
        dt.copy_(ship.repeat((n + 64) // len(SHIP) + 1)[: n + 64])
    a = torch.empty(n, dtype=torch.int32, device="cuda")
    b = torch.empty(n, dtype=torch.int32, device="cuda")
    ca = torch.zeros(1, dtype=torch.int64, device="cuda")
    cb = torch.zeros(1, dtype=torch.int64, device="cuda")
    rt.scan_device(dt.data_ptr(), 0, 0, n, a.data_ptr(), ca.data_ptr(), s)
    ac.scan_device(dt.data_ptr(), 0, 0, n, b.data_ptr(), cb.data_ptr(), s)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert int(ca.item()) == int(cb.item()) == int((a != 0).sum().item())
    try:  # both DFA forms at full size
        for form in (1, 2):
            ac.set_option("dfa_form", form)
            b.zero_()
            ac.scan_device(dt.data_ptr(), 0, 0, n, b.data_ptr(), None, s)
            torch.cuda.synchronize()
            assert ac.dfa_form_last == form and torch.equal(a, b), form
    finally:
        ac.set_option("dfa_form", 0)
    for _ in range(2):  # auto: an RT launch, then (deep stream) the DFA
        b.zero_()
        au.scan_device(dt.data_ptr(), 0, 0, n, b.data_ptr(), None, s)
        torch.cuda.synchronize()
        assert torch.equal(a, b)
    del a, b, dt
    torch.cuda.empty_cache()


@pytest.mark.slow
def test_large_automaton_uses_the_uncoded_dfa():
    """A dictionary of more than 2^20 automaton states: the DFA image keeps
    plain transitions (the coded word has 20 state bits, pm_flatten.h) and
    runs dfa_scan_kernel; it must still equal the RT kernel and a brute
    force on a stream that contains the patterns."""
    import torch
    rng = np.random.default_rng(21)
    pats = [bytes(rng.integers(0x20, 0x7F, size=int(L), dtype=np.uint8)) for L in rng.integers(20, 40, size=40000)]
    d = pm.Dictionary(patterns=pats)
    ac, rt = pm.HipMatcher("ac"), pm.HipMatcher("rt")
    for m in (ac, rt):
        m.add_dictionary(d)
        m.compile()
    n = 1 << 20
    text = np.frombuffer(b"".join(pats[int(k)] for k in rng.integers(0, len(pats), size=n // 20)), np.uint8)[:n]
    a = ac.read_block_codes(text)
    b = rt.read_block_codes(text)
    assert np.array_equal(a, b)
    codes = {}
    for i in range(d.n):
        f, l, by = d.pattern(i)
        codes[by] = (f << 24) | l
    tb = text[:20000].tobytes()
    for i in range(len(tb)):
        exp = 0
        for k in range(min(40, i + 1), 0, -1):
            c = codes.get(tb[i + 1 - k:i + 1])
            if c is not None:
                exp = c
                break
        assert a[i] == exp, i
    ac.free()
    rt.free()


def test_lines_stream_generator_and_kernels():
    """The lines stream (random dictionary patterns back to back): device
    bytes == host bytes; on 64 MiB of it RT, AC and auto agree at every
    position, and a window matches the oracle."""
    import torch
    n = 64 << 20
    rt, ac, au = matcher("snort", "rt"), matcher("snort", "ac"), matcher("snort", "auto")
    s = torch.cuda.current_stream().cuda_stream
    dt = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    rt.gen_lines_device(dt.data_ptr(), n + 64, 3, s)
    torch.cuda.synchronize()
    host = rt.gen_lines(1 << 20, 3)
    assert np.array_equal(dt[: 1 << 20].cpu().numpy(), host)
    assert np.array_equal(ac.gen_lines(1 << 20, 3), host)  # the same patterns in the same order
    a = torch.empty(n, dtype=torch.int32, device="cuda")
    b = torch.empty(n, dtype=torch.int32, device="cuda")
    rt.scan_device(dt.data_ptr(), 0, 0, n, a.data_ptr(), None, s)
    ac.scan_device(dt.data_ptr(), 0, 0, n, b.data_ptr(), None, s)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert int((a != 0).sum().item()) > 0.9 * n  # deep: nearly every position inside a pattern
    au.scan_device(dt.data_ptr(), 0, 0, n, b.data_ptr(), None, s)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    o = oracle_for("snort")
    o.reset()
    assert np.array_equal(o.scan_codes(host), rt._codes[a[: 1 << 20].cpu().numpy().view(np.uint32)])


@pytest.mark.parametrize("key,stream", [("snort", "ascii"), ("snort", "lines"), ("snort", "ship"),
                                        ("et", "lines"), ("merged", "lines"), ("merged", "ship")])
def test_sparse_dfa_equals_dense_dfa(key, stream):
    """The AC kind's two forms of the output-coded automaton -- dense rows
    (dfa_coded_kernel) and rows + default-transition records
    (dfa_sparse_kernel, pm_flatten.h) -- give the same u32 / u16 ids and
    counts at every position, at launch sizes from one segment with its
    warm-up to 64 MiB, under both warm-up rules (max_len - 1 bytes back, or
    from the last synchronizing 3-gram), and equal the RT kernel."""
    torch = _torch()
    lib = pm.load()
    rt, ac = matcher(key, "rt"), matcher(key, "ac")
    n = (64 if key == "snort" else 16) << 20
    s = torch.cuda.current_stream().cuda_stream
    dt = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    if stream == "ascii":
        lib.pm_hip_gen_stream_device(dt.data_ptr(), 0, n + 64, 5, 0, s)
    elif stream == "lines":
        rt.gen_lines_device(dt.data_ptr(), n + 64, 9, s)
    else:
        dt.copy_(torch.from_numpy(np.tile(SHIP, (n + 64) // len(SHIP) + 1)[: n + 64]).cuda())
    ref = torch.empty(n, dtype=torch.int32, device="cuda")
    rt.scan_device(dt.data_ptr(), 0, 0, n, ref.data_ptr(), None, s)
    try:
        for size, start in ((n, 0), (1000, 5000), (100 << 10, 12345), (3 << 20, 1 << 20)):
            start &= ~15
            got = {}
            for form, sync in [(x, y) for x in (1, 2) for y in (0, 1)]:
                ac.set_option("dfa_form", form)
                ac.set_option("dfa_sync", sync)
                a = torch.zeros(size, dtype=torch.int32, device="cuda")
                h = torch.zeros(size, dtype=torch.int16, device="cuda")
                c = torch.zeros(3, dtype=torch.int64, device="cuda")
                ac.scan_device(dt.data_ptr(), 0, start, size, a.data_ptr(), c[0:1].data_ptr(), s)
                ac.scan_device(dt.data_ptr(), 0, start, size, h.data_ptr(), c[1:2].data_ptr(), s, out_width=2)
                ac.scan_device(dt.data_ptr(), 0, start, size, 0, c[2:3].data_ptr(), s)
                torch.cuda.synchronize()
                got[(form, sync)] = (a, h, c)
            a0, h0, c0 = got[(1, 0)]
            for key in list(got)[1:]:
                a1, h1, c1 = got[key]
                assert torch.equal(a0, a1) and torch.equal(h0, h1) and torch.equal(c0, c1), key
            assert torch.equal(a1, ref[start:start + size])
            assert int(c1[0].item()) == int(c1[2].item()) == int((a1 != 0).sum().item())
            assert torch.equal(h1.to(torch.int32) & 0xFFFF, a1)
    finally:
        ac.set_option("dfa_form", 0)
        ac.set_option("dfa_sync", 1)


# the sparse form's kernels ("sparse_kernel": 1 fallback-linked, 2 lock-step
# 8-B units, 3 lock-step 16-B records) and the widths each writes
SPARSE_KERNELS = {1: (4, 2, 0), 2: (4, 2, 0), 3: (4, 2, 0)}


@pytest.mark.parametrize("key", ["et", "merged"])
def test_fl_kernel_every_width(key):
    """The fallback-linked kernel (sparse_kernel 1) on et and the merged
    dictionaries, 8 MiB of each one's lines stream plus the shipped stream,
    with each record-load policy ("fl_hold": 16-B halves, deep records'
    32-B and 64-B blocks) and with two chains per lane ("fl_chains" 2,
    dfa_fl2_kernel, 16-B halves and 32-B blocks): u32 ids, u16 ids and the
    count equal the reverse-trie kernel's."""
    torch = _torch()
    rt, ac = matcher(key, "rt"), matcher(key, "ac")
    n = 8 << 20
    s = torch.cuda.current_stream().cuda_stream
    dt = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    try:
        assert ac.set_option("dfa_form", 2) == 0 and ac.set_option("sparse_kernel", 1) == 0
        assert ac.set_option("fl_hold", 3) == -1 and ac.set_option("fl_chains", 3) == -1
        for stream in ("lines", "ship"):
            if stream == "lines":
                rt.gen_lines_device(dt.data_ptr(), n + 64, 21, s)
            else:
                dt.copy_(torch.from_numpy(np.tile(SHIP, (n + 64) // len(SHIP) + 1)[: n + 64]).cuda())
            ref = torch.empty(n, dtype=torch.int32, device="cuda")
            rt.scan_device(dt.data_ptr(), 0, 0, n, ref.data_ptr(), None, s)
            nz = int((ref != 0).sum().item())
            for hold, chains in ((1, 1), (2, 1), (4, 1), (1, 2), (2, 2)):
                assert ac.set_option("fl_hold", hold) == 0 and ac.set_option("fl_chains", chains) == 0
                a = torch.zeros(n, dtype=torch.int32, device="cuda")
                h = torch.zeros(n, dtype=torch.int16, device="cuda")
                c = torch.zeros(2, dtype=torch.int64, device="cuda")
                ac.scan_device(dt.data_ptr(), 0, 0, n, a.data_ptr(), c[0:1].data_ptr(), s)
                assert ac.sparse_kernel_last == 1
                ac.scan_device(dt.data_ptr(), 0, 0, n, h.data_ptr(), None, s, out_width=2)
                assert ac.sparse_kernel_last == 1
                ac.scan_device(dt.data_ptr(), 0, 0, n, 0, c[1:2].data_ptr(), s)
                assert ac.sparse_kernel_last == 1
                torch.cuda.synchronize()
                assert torch.equal(a, ref), (stream, hold, chains)
                assert torch.equal(h.to(torch.int32) & 0xFFFF, ref), (stream, hold, chains)
                assert int(c[0].item()) == nz and int(c[1].item()) == nz, (stream, hold, chains)
    finally:
        ac.set_option("fl_hold", 0)
        ac.set_option("fl_chains", 0)
        ac.set_option("sparse_kernel", 0)
        ac.set_option("dfa_form", 0)


def test_gather_ceiling_probe():
    """pm_hip_gather_ceiling_device (bench.py's live bound for the DFA legs):
    runs over an ac object's own FL image and finishes; an rt object, which
    has no such image, gets -2 and launches nothing."""
    torch = _torch()
    lib = pm.load()
    s = torch.cuda.current_stream()
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    assert lib.pm_hip_gather_ceiling_device(matcher("snort", "ac").obj, 64, sink.data_ptr(), s.cuda_stream) == 0
    torch.cuda.synchronize()
    assert int(sink.item()) == 0
    assert lib.pm_hip_gather_ceiling_device(matcher("snort", "rt").obj, 64, sink.data_ptr(), s.cuda_stream) == -2


def test_sparse_form_without_8b_units():
    """An automaton inside the coded range whose 8-B record units do not fit
    the coded word (F + units > 2^20: 200,000 random 8-byte patterns over
    20 letters, 916,050 states -- larger than merged's) has the sparse form
    but neither the 8-B nor the fallback-linked layout (gids past u16): its
    u32 scans and its count take the lock-step kernel over the 16-B records
    (sparse_kernel 3) and equal the dense rows' (no 8-B-unit
    kernel may run on the missing image)."""
    torch = _torch()
    rng = np.random.default_rng(7)
    pats = list({bytes(r) for r in (rng.integers(0, 20, size=(200000, 8)).astype(np.uint8) + ord("a"))})
    m = pm.HipMatcher("ac")
    m.add_dictionary(pm.Dictionary(patterns=pats))
    m.compile()
    n = 2 << 20
    order = rng.integers(0, len(pats), size=n // 8 + 1)
    text = np.frombuffer(b"".join(pats[k] for k in order), np.uint8)[:n].copy()
    text[::97] = ord("z")  # breaks between pattern runs
    s = torch.cuda.current_stream().cuda_stream
    dt = torch.from_numpy(np.concatenate([text, np.zeros(64, np.uint8)])).cuda()
    try:
        out = {}
        for form in (1, 2):
            assert m.set_option("dfa_form", form) == 0
            a = torch.zeros(n, dtype=torch.int32, device="cuda")
            c = torch.zeros(1, dtype=torch.int64, device="cuda")
            m.scan_device(dt.data_ptr(), 0, 0, n, a.data_ptr(), c.data_ptr(), s)
            torch.cuda.synchronize()
            if form == 2:
                assert m.sparse_kernel_last == 3
            cc = torch.zeros(1, dtype=torch.int64, device="cuda")
            m.scan_device(dt.data_ptr(), 0, 0, n, 0, cc.data_ptr(), s)
            torch.cuda.synchronize()
            out[form] = (a, int(c.item()), int(cc.item()))
        assert torch.equal(out[1][0], out[2][0])
        assert out[1][1] == out[2][1] == out[1][2] == out[2][2] == int((out[1][0] != 0).sum().item())
        assert out[1][1] > 0
    finally:
        m.set_option("dfa_form", 0)
        m.free()


@pytest.mark.parametrize("stream", ["lines", "ship"])
def test_sparse_dfa_kernel_variants_agree(stream):
    """Every kernel of the sparse form ("sparse_kernel" 1-3: the
    fallback-linked form, the lock-step kernels over 8-B units and 16-B
    records), under both warm-up
    rules, gives the RT kernel's u32 / u16 ids and the same count, at sizes
    from one warm-up segment to 32 MiB (snort); a width a kernel does not
    write runs the product choice, and pm_hip_sparse_kernel_last says which
    ran."""
    torch = _torch()
    rt, ac = matcher("snort", "rt"), matcher("snort", "ac")
    n = 32 << 20
    s = torch.cuda.current_stream().cuda_stream
    dt = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    if stream == "lines":
        rt.gen_lines_device(dt.data_ptr(), n + 64, 11, s)
    else:
        dt.copy_(torch.from_numpy(np.tile(SHIP, (n + 64) // len(SHIP) + 1)[: n + 64]).cuda())
    ref = torch.empty(n, dtype=torch.int32, device="cuda")
    rt.scan_device(dt.data_ptr(), 0, 0, n, ref.data_ptr(), None, s)
    ac.set_option("dfa_form", 2)
    try:
        # (2,567: 41 segments of 64, a wave with chains past 32 active, not all)
        for size, start in ((n, 0), (777, 4096), (2567, 8208), (100 << 10, 12345 & ~15), (5 << 20, 3 << 20)):
            for sk, sync, chains in [(k, y, 1) for k in SPARSE_KERNELS for y in (0, 1)] + [(1, 0, 2), (1, 1, 2)]:
                assert ac.set_option("sparse_kernel", sk) == 0 and ac.set_option("dfa_sync", sync) == 0
                assert ac.set_option("fl_chains", chains) == 0
                a = torch.zeros(size, dtype=torch.int32, device="cuda")
                h = torch.zeros(size, dtype=torch.int16, device="cuda")
                c = torch.zeros(2, dtype=torch.int64, device="cuda")
                tag = (size, sk, sync, chains)
                ac.scan_device(dt.data_ptr(), 0, start, size, a.data_ptr(), c[0:1].data_ptr(), s)
                assert ac.sparse_kernel_last == sk, tag
                ac.scan_device(dt.data_ptr(), 0, start, size, h.data_ptr(), None, s, out_width=2)
                assert (ac.sparse_kernel_last == sk) == (2 in SPARSE_KERNELS[sk]), tag
                ac.scan_device(dt.data_ptr(), 0, start, size, 0, c[1:2].data_ptr(), s)
                assert (ac.sparse_kernel_last == sk) == (0 in SPARSE_KERNELS[sk]), tag
                torch.cuda.synchronize()
                assert torch.equal(a, ref[start:start + size]), tag
                assert torch.equal(h.to(torch.int32) & 0xFFFF, a), tag
                assert int(c[0].item()) == int(c[1].item()) == int((a != 0).sum().item()), tag
    finally:
        ac.set_option("sparse_kernel", 0)
        ac.set_option("fl_chains", 0)
        ac.set_option("dfa_sync", 1)
        ac.set_option("dfa_form", 0)


@pytest.mark.parametrize("stream", ["lines", "ship"])
def test_dfa_warmups_stop_at_stream_start(stream):
    """Bytes before stream_start are not the stream: the DFA warm-ups (from
    max_len - 1 bytes back, or from the last synchronizing 3-gram,
    dfa_sync_lo) must not look at them.  The bytes before stream_start are
    pattern-dense text of another seed, stream_start is not aligned, and the
    first positions lie within max_len of it; every DFA form (dense rows;
    every kernel of the sparse form) under both warm-up rules gives the RT
    kernel's u32 / u16 ids and count."""
    torch = _torch()
    rt, ac = matcher("snort", "rt"), matcher("snort", "ac")
    n = 4 << 20
    s = torch.cuda.current_stream().cuda_stream
    dt = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    if stream == "lines":
        rt.gen_lines_device(dt.data_ptr(), n + 64, 13, s)
    else:
        dt.copy_(torch.from_numpy(np.tile(SHIP, (n + 64) // len(SHIP) + 1)[: n + 64]).cuda())
    garbage = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    rt.gen_lines_device(garbage.data_ptr(), n + 64, 99, s)
    try:
        for stream_start, pos0, size in ((4099, 4112, 1 << 20), (77, 80, 3000), (1000, 1040, 2 << 20),
                                         (12345, 12352 + 4096, 1 << 20)):
            buf = garbage.clone()
            buf[stream_start:] = dt[: n + 64 - stream_start]
            ref = torch.empty(size, dtype=torch.int32, device="cuda")
            rt.scan_device(buf.data_ptr(), stream_start, pos0, size, ref.data_ptr(), None, s)
            forms = [(1, 0, y, 1) for y in (0, 1)] + [(2, k, y, 1) for k in [0] + list(SPARSE_KERNELS) for y in (0, 1)]
            forms += [(2, 1, y, 2) for y in (0, 1)]  # two chains per lane
            for form, sk, sync, chains in forms:
                ac.set_option("dfa_form", form)
                ac.set_option("sparse_kernel", sk)
                ac.set_option("dfa_sync", sync)
                ac.set_option("fl_chains", chains)
                a = torch.zeros(size, dtype=torch.int32, device="cuda")
                h = torch.zeros(size, dtype=torch.int16, device="cuda")
                c = torch.zeros(1, dtype=torch.int64, device="cuda")
                ac.scan_device(buf.data_ptr(), stream_start, pos0, size, a.data_ptr(), None, s)
                ac.scan_device(buf.data_ptr(), stream_start, pos0, size, h.data_ptr(), None, s, out_width=2)
                ac.scan_device(buf.data_ptr(), stream_start, pos0, size, 0, c.data_ptr(), s)
                torch.cuda.synchronize()
                tag = (stream_start, pos0, form, sk, sync, chains)
                assert torch.equal(a, ref), tag
                assert torch.equal(h.to(torch.int32) & 0xFFFF, a), tag
                assert int(c.item()) == int((a != 0).sum().item()), tag
    finally:
        ac.set_option("sparse_kernel", 0)
        ac.set_option("fl_chains", 0)
        ac.set_option("dfa_sync", 1)
        ac.set_option("dfa_form", 0)


def test_adversarial_stream_large_rt_equals_ac():
    """A 32 MiB tiling of the shipped adversarial stream queues far more
    positions than the worklist holds, so the scan kernel's in-kernel
    fallback runs; RT must still equal the independent AC-DFA kernel and the
    oracle."""
    torch = _torch()
    rt, ac = matcher("merged", "rt"), matcher("merged", "ac")
    n = 32 << 20
    text = np.tile(SHIP, n // len(SHIP) + 1)[:n]
    s = torch.cuda.current_stream().cuda_stream
    dt = torch.from_numpy(np.concatenate([text, np.zeros(64, np.uint8)])).cuda()
    a = torch.empty(n, dtype=torch.int32, device="cuda")
    b = torch.empty(n, dtype=torch.int32, device="cuda")
    ca = torch.zeros(1, dtype=torch.int64, device="cuda")
    cb = torch.zeros(1, dtype=torch.int64, device="cuda")
    rt.scan_device(dt.data_ptr(), 0, 0, n, a.data_ptr(), ca.data_ptr(), s)
    ac.scan_device(dt.data_ptr(), 0, 0, n, b.data_ptr(), cb.data_ptr(), s)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert int(ca.item()) == int(cb.item()) == int((a != 0).sum().item())
    o = oracle_for("merged")
    o.reset()
    exp = o.scan_codes(text[:1 << 20])
    assert np.array_equal(rt._codes[a[:1 << 20].cpu().numpy().view(np.uint32)], exp)


@pytest.mark.parametrize("n", [1, 3, 4, 5, 17, 4099, (1 << 18) * 4 + 13])
def test_score_and_counts_ragged_lengths(n):
    """Both A12 kernels load several 16-B id vectors per thread (HIST_V,
    SCORE_V in csrc/pm_kernels.hip) and score the n % 4 tail separately; tiny
    and ragged lengths against the numpy restatement (measure.c:174-190)."""
    torch = _torch()
    s = torch.cuda.current_stream().cuda_stream
    rt = matcher("snort", "rt")
    P = rt.lib.pm_hip_n_patterns(rt.obj)
    parent = np.array([rt.parent_gid(g) for g in range(P + 1)], np.int64)
    depth = np.zeros(P + 1, np.int64)
    for g in range(1, P + 1):
        c, k = g, 0
        while c:
            c, k = parent[c], k + 1
        depth[g] = k
    rng = np.random.default_rng(n)
    real = rng.integers(0, P + 1, n).astype(np.uint32)
    real[rng.random(n) < 0.3] = 0
    algo = real.copy()
    m = rng.random(n)
    algo[m < 0.1] = 0
    algo[(m >= 0.1) & (m < 0.2)] = parent[real[(m >= 0.1) & (m < 0.2)]].astype(np.uint32)
    algo[m >= 0.9] = rng.integers(1, P + 1, int((m >= 0.9).sum()))
    pad = np.zeros(4, np.uint32)
    ad = torch.from_numpy(np.concatenate([algo, pad]).view(np.int32)).cuda()
    rd = torch.from_numpy(np.concatenate([real, pad]).view(np.int32)).cuda()
    cnt = torch.zeros(5, dtype=torch.int64, device="cuda")
    rt.score_device(ad.data_ptr(), rd.data_ptr(), n, cnt.data_ptr(), s)
    hist = torch.zeros(P + 1, dtype=torch.int64, device="cuda")
    rt.pattern_counts_device(rd.data_ptr(), n, hist.data_ptr(), s)
    torch.cuda.synchronize()
    assert cnt.cpu().tolist() == _score_host(algo, real, parent, depth)
    exp = np.zeros(P + 1, np.int64)
    cur = real.astype(np.int64)
    while cur.any():
        cur = cur[cur > 0]
        np.add.at(exp, cur, 1)
        cur = parent[cur]
    assert np.array_equal(hist.cpu().numpy(), exp)


def _tiled_ship(n):
    return np.tile(SHIP, n // len(SHIP) + 1)[:n]


def test_auto_switches_to_the_dfa_on_dense_deep_matches():
    """The auto kind runs RT first; on the reference's shipped stream (dense
    deep matches: the RT kernel spills > 10 % of positions) the next launch
    is a timed AC-DFA trial, then the faster of the two holds; every launch
    is exact."""
    import torch
    n = 16 << 20
    text = _tiled_ship(n)
    s = torch.cuda.current_stream()
    dt = torch.from_numpy(np.concatenate([text, np.zeros(64, np.uint8)])).cuda()
    ref = matcher("et", "ac")
    want = torch.empty(n, dtype=torch.int32, device="cuda")
    ref.scan_device(dt.data_ptr(), 0, 0, n, want.data_ptr(), None, s.cuda_stream)
    m = matcher("et", "auto")
    kernels, forms = [], []
    for _ in range(15):
        got = torch.empty(n, dtype=torch.int32, device="cuda")
        m.scan_device(dt.data_ptr(), 0, 0, n, got.data_ptr(), None, s.cuda_stream)
        torch.cuda.synchronize()
        kernels.append(m.kernel_last)
        forms.append(m.dfa_form_last)
        assert torch.equal(got, want)
    # RT first (measured: it spills), then two trial launches of each DFA
    # candidate (dense rows; rows + records with 16-B halves, two chains per
    # lane, 64-B deep blocks; the second of each timed); the fastest per
    # position holds
    assert kernels[:9] == [pm.KIND_RT] + [pm.KIND_AC] * 8, kernels
    assert forms[:9] == [0, 1, 1] + [2] * 6, forms
    assert len(set(zip(kernels[9:], forms[9:]))) == 1, (kernels, forms)


@pytest.mark.parametrize("cap", [1, 2])
def test_bounded_spill_region_resolves_many_times(cap):
    """The RT spill region is bounded per wave (pm_kernels.hip, resolved in
    the push's ring-full branch when a chunk could overflow it).  With the
    bound at 1-2 chunks, 32 MiB of the shipped stream (deep matches: a
    quarter of the positions spill) resolves full regions dozens of times
    per wave; ids (u32, u16) and counts equal the AC-DFA's."""
    import torch
    lib = pm.load()
    n = 32 << 20
    text = _tiled_ship(n)
    dt = torch.from_numpy(np.concatenate([text, np.zeros(64, np.uint8)])).cuda()
    s = torch.cuda.current_stream().cuda_stream
    want = torch.empty(n, dtype=torch.int32, device="cuda")
    matcher("merged", "ac").scan_device(dt.data_ptr(), 0, 0, n, want.data_ptr(), None, s)
    rt = matcher("merged", "rt")
    rt.set_option("spill_cap_chunks", cap)
    try:
        got = torch.empty(n, dtype=torch.int32, device="cuda")
        got16 = torch.empty(n, dtype=torch.int16, device="cuda")
        c = torch.zeros(3, dtype=torch.int64, device="cuda")
        rt.scan_device(dt.data_ptr(), 0, 0, n, got.data_ptr(), c[0:].data_ptr(), s)
        rt.scan_device(dt.data_ptr(), 0, 0, n, got16.data_ptr(), c[1:].data_ptr(), s, out_width=2)
        rt.scan_device(dt.data_ptr(), 0, 0, n, None, c[2:].data_ptr(), s)
        torch.cuda.synchronize()
    finally:
        rt.set_option("spill_cap_chunks", 0)
    assert torch.equal(got, want)
    assert torch.equal(got16.to(torch.int32) & 0xFFFF, want)
    nz = int((want != 0).sum().item())
    assert c.tolist() == [nz, nz, nz]


def test_rt_scan_device_concurrent_streams_spill():
    """Launches of one RT object on different streams may run at once; each
    stream has its own spill scratch (pm_plugin.hip stream_spill), and past
    four streams the least recently used one is handed over behind an event
    wait.  Deep input with the region bounded at two chunks per wave makes
    every launch use its scratch; six streams, launched with no host
    synchronization, must all be exact."""
    import torch
    n = 6 << 20
    text = _tiled_ship(n)
    dt = torch.from_numpy(np.concatenate([text, np.zeros(64, np.uint8)])).cuda()
    ref = matcher("et", "ac")
    want = torch.empty(n, dtype=torch.int32, device="cuda")
    ref.scan_device(dt.data_ptr(), 0, 0, n, want.data_ptr(), None, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    m = matcher("et", "rt")
    m.set_option("spill_cap_chunks", 2)
    try:
        streams = [torch.cuda.Stream() for _ in range(6)]
        outs = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(18)]
        for k, o in enumerate(outs):
            m.scan_device(dt.data_ptr(), 0, 0, n, o.data_ptr(), None, streams[k % 6].cuda_stream)
        torch.cuda.synchronize()
    finally:
        m.set_option("spill_cap_chunks", 0)
    for o in outs:
        assert torch.equal(o, want)


def test_auto_scan_device_across_two_streams_and_hold():
    """The auto kind's pick is polled, never waited for (pm_plugin.hip
    launch): launches alternating between two streams with no host
    synchronization are all exact; once they have landed the pick resolves
    and pm_hip_hold_choice pins it."""
    import torch
    n = 8 << 20
    text = _tiled_ship(n)
    dt = torch.from_numpy(np.concatenate([text, np.zeros(64, np.uint8)])).cuda()
    ref = matcher("et", "ac")
    want = torch.empty(n, dtype=torch.int32, device="cuda")
    ref.scan_device(dt.data_ptr(), 0, 0, n, want.data_ptr(), None, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    m = matcher("et", "auto")
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(12)]
    for k, o in enumerate(outs):
        m.scan_device(dt.data_ptr(), 0, 0, n, o.data_ptr(), None, streams[k & 1].cuda_stream)
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, want)
    held = m.hold_choice(0)
    for _ in range(16):
        if held > 0:
            break
        o = outs[0]
        m.scan_device(dt.data_ptr(), 0, 0, n, o.data_ptr(), None, streams[0].cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(o, want)
        held = m.hold_choice(0)
    assert held in (1, 2, 3, 4, 5, 6), held
    assert m.hold_choice(100) == held  # pinned for the next 100 launches
    for _ in range(3):
        m.scan_device(dt.data_ptr(), 0, 0, n, outs[1].data_ptr(), None, streams[1].cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(outs[1], want)
        assert m.hold_choice(0) == held
    assert matcher("et", "rt").hold_choice(5) == 0  # the rt kind has nothing to pick


def test_auto_scan_device_under_graph_capture():
    """scan_device of the auto kind inside a HIP graph capture (torch CUDA
    graph): nothing is measured under capture (no events, no copies), the
    current choice is captured, and a replay gives the eager ids."""
    import torch
    n = 4 << 20
    text = _tiled_ship(n)
    dt = torch.from_numpy(np.concatenate([text, np.zeros(64, np.uint8)])).cuda()
    m = matcher("et", "auto")
    m.prepare_capture()
    s = torch.cuda.Stream()
    want = torch.empty(n, dtype=torch.int32, device="cuda")
    got = torch.zeros(n, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    with torch.cuda.stream(s):
        m.scan_device(dt.data_ptr(), 0, 0, n, want.data_ptr(), None, s.cuda_stream)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        m.scan_device(dt.data_ptr(), 0, 0, n, got.data_ptr(), cnt.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    for _ in range(2):
        cnt.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(got, want)
        assert int(cnt.item()) == int((want != 0).sum().item())


@pytest.mark.parametrize("kind", ["auto", "ac", "rt"])
def test_first_scan_device_inside_graph_capture(kind):
    """The very first scan_device of a new object inside a capture: with
    pm_hip_prepare_capture before it the launch is captured and a replay
    gives the RT kernel's eager ids; without it (rt / auto, whose scratch
    cannot be allocated under capture) scan_device fails with an error,
    launches nothing, and the capture ends cleanly.  Nothing is allocated
    under capture either way (pm_plugin.hip init_pick)."""
    import torch
    n = 4 << 20
    dt = torch.from_numpy(np.concatenate([_tiled_ship(n), np.zeros(64, np.uint8)])).cuda()
    want = torch.empty(n, dtype=torch.int32, device="cuda")
    matcher("et", "rt").scan_device(dt.data_ptr(), 0, 0, n, want.data_ptr(), None,
                                    torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    if kind != "ac":
        bare = fresh_matcher("et", kind)
        got = torch.zeros(n, dtype=torch.int32, device="cuda")
        g = torch.cuda.CUDAGraph()
        with pytest.raises(RuntimeError, match="prepare_capture"):
            with torch.cuda.graph(g, stream=s):
                bare.scan_device(dt.data_ptr(), 0, 0, n, got.data_ptr(), None, s.cuda_stream)
        torch.cuda.synchronize()
        # a launch the one-thread-per-position kernel takes (<= 256 Ki
        # positions) needs no scratch, so no prepare_capture
        small = 100 << 10
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2, stream=s):
            bare.scan_device(dt.data_ptr(), 0, 0, small, got.data_ptr(), None, s.cuda_stream)
        got.zero_()
        g2.replay()
        torch.cuda.synchronize()
        assert torch.equal(got[:small], want[:small])
    m = fresh_matcher("et", kind)
    m.prepare_capture()
    assert m.scratch_bytes >= (0 if kind == "ac" else 1 << 20)
    got = torch.zeros(n, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        m.scan_device(dt.data_ptr(), 0, 0, n, got.data_ptr(), cnt.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    for _ in range(2):
        cnt.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(got, want)
        assert int(cnt.item()) == int((want != 0).sum().item())


def test_spill_cap_raised_after_prepare():
    """A spill cap raised after the capture scratch was sized (the
    "spill_cap_chunks" option: 2 chunks when prepare_capture sized the
    scratch, the default 16 at the captured launch) clamps the captured
    launch's regions to the scratch instead of failing it; the ids stay
    exact."""
    import torch
    n = 128 << 20  # 32 chunks per wave: past the default 16-chunk regions
    dt = torch.from_numpy(np.concatenate([_tiled_ship(n), np.zeros(64, np.uint8)])).cuda()
    want = torch.empty(n, dtype=torch.int32, device="cuda")
    matcher("et", "ac").scan_device(dt.data_ptr(), 0, 0, n, want.data_ptr(), None,
                                    torch.cuda.current_stream().cuda_stream)
    m = fresh_matcher("et", "rt")
    m.set_option("spill_cap_chunks", 2)
    m.prepare_capture()
    m.set_option("spill_cap_chunks", 0)
    s = torch.cuda.Stream()
    got = torch.zeros(n, dtype=torch.int32, device="cuda")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        m.scan_device(dt.data_ptr(), 0, 0, n, got.data_ptr(), None, s.cuda_stream)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(got, want)


@pytest.mark.parametrize("stream", ["ship", "lines"])
def test_ac_kind_times_both_dfa_forms(stream):
    """The AC kind tries its forms (dense rows, rows + records, the latter
    with each record-load policy and with two chains per lane; two launches
    each, the second timed) and holds the fastest; every launch equals the
    RT kernel."""
    import torch
    n = 16 << 20
    s = torch.cuda.current_stream()
    rt, ac = matcher("snort", "rt"), matcher("snort", "ac")
    dt = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    if stream == "ship":
        dt.copy_(torch.from_numpy(np.concatenate([_tiled_ship(n), np.zeros(64, np.uint8)])).cuda())
    else:
        rt.gen_lines_device(dt.data_ptr(), n + 64, 4, s.cuda_stream)
    want = torch.empty(n, dtype=torch.int32, device="cuda")
    rt.scan_device(dt.data_ptr(), 0, 0, n, want.data_ptr(), None, s.cuda_stream)
    forms = []
    for _ in range(13):
        got = torch.empty(n, dtype=torch.int32, device="cuda")
        ac.scan_device(dt.data_ptr(), 0, 0, n, got.data_ptr(), None, s.cuda_stream)
        torch.cuda.synchronize()
        assert ac.kernel_last == pm.KIND_AC
        forms.append(ac.dfa_form_last)
        assert torch.equal(got, want)
    # dense rows, then rows + records with 16-B halves, the same with two
    # chains per lane, and with 64-B deep blocks: two launches each, then
    # the fastest holds
    assert forms[:8] == [1, 1] + [2] * 6 and forms[8] == forms[9] == forms[10] in (1, 2), forms
    ac.reset()  # a new stream: the forms are timed again
    ac.scan_device(dt.data_ptr(), 0, 0, n, got.data_ptr(), None, s.cuda_stream)
    torch.cuda.synchronize()
    assert ac.dfa_form_last == 1 and torch.equal(got, want)


def test_auto_count_only_follows_deep_walks():
    """Count-only RT launches spill every candidate, so the auto kind's
    signal there is the positions the tail walked; random ASCII keeps it on
    RT; the counts are exact on the shipped stream and random ASCII."""
    import torch
    n = 16 << 20
    s = torch.cuda.current_stream()
    deep = torch.from_numpy(np.concatenate([_tiled_ship(n), np.zeros(64, np.uint8)])).cuda()
    sparse = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    assert pm.load().pm_hip_gen_stream_device(sparse.data_ptr(), 0, n + 64, 5, 0, s.cuda_stream) == 0
    ref = matcher("snort", "ac")
    for text, want_kernel in ((sparse, pm.KIND_RT), (deep, pm.KIND_AC)):
        want = torch.zeros(1, dtype=torch.int64, device="cuda")
        ref.scan_device(text.data_ptr(), 0, 0, n, None, want.data_ptr(), s.cuda_stream)
        m = matcher("snort", "auto")
        kernels = []
        for _ in range(3):
            got = torch.zeros(1, dtype=torch.int64, device="cuda")
            m.scan_device(text.data_ptr(), 0, 0, n, None, got.data_ptr(), s.cuda_stream)
            torch.cuda.synchronize()
            kernels.append(m.kernel_last)
            assert int(got.item()) == int(want.item())
        # sparse: RT throughout.  (Deep: count-only walks only positions
        # whose depth-2 answer is 0, so the walk signal rarely fires there
        # either; whichever kernel runs, the count is exact.)
        assert kernels[0] == pm.KIND_RT, kernels
        if want_kernel == pm.KIND_RT:
            assert kernels == [pm.KIND_RT] * 3, kernels


def test_auto_hold_doubles_when_confirmed():
    """The auto kind re-measures (an RT launch, then the DFA trials) after
    its hold; a choice the next measurement confirms is held twice as long
    (pm_plugin.hip AUTO_STREAK_MAX), so on a deep stream the RT launches
    come further apart; every launch stays exact."""
    import torch
    n = 16 << 20  # the tiled shipped stream: a DFA form holds, so each RT launch is a measurement
    s = torch.cuda.current_stream()
    rt, au = matcher("et", "rt"), matcher("et", "auto")
    dt = torch.from_numpy(np.concatenate([_tiled_ship(n), np.zeros(64, np.uint8)])).cuda()
    want = torch.empty(n, dtype=torch.int32, device="cuda")
    rt.scan_device(dt.data_ptr(), 0, 0, n, want.data_ptr(), None, s.cuda_stream)
    au.reset()
    kinds = []
    got = torch.empty(n, dtype=torch.int32, device="cuda")
    for k in range(260):
        au.scan_device(dt.data_ptr(), 0, 0, n, got.data_ptr(), None, s.cuda_stream)
        torch.cuda.synchronize()
        kinds.append(au.kernel_last)
        if k % 37 == 0:
            assert torch.equal(got, want), k
    rts = [k for k, v in enumerate(kinds) if v == pm.KIND_RT]
    assert rts[0] == 0 and len(rts) >= 3 and kinds[10] == pm.KIND_AC, (rts, kinds[:12])
    gaps = [b - a for a, b in zip(rts, rts[1:])]
    assert gaps[1] > gaps[0] + 32, (rts, gaps)
    au.reset()


def test_auto_stays_on_rt_for_sparse_matches():
    import torch
    n = 16 << 20
    s = torch.cuda.current_stream()
    lib = pm.load()
    dt = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    assert lib.pm_hip_gen_stream_device(dt.data_ptr(), 0, n + 64, 5, 0, s.cuda_stream) == 0
    m = matcher("snort", "auto")
    ref = matcher("snort", "rt")
    want = torch.empty(n, dtype=torch.int32, device="cuda")
    ref.scan_device(dt.data_ptr(), 0, 0, n, want.data_ptr(), None, s.cuda_stream)
    for _ in range(4):
        got = torch.empty(n, dtype=torch.int32, device="cuda")
        m.scan_device(dt.data_ptr(), 0, 0, n, got.data_ptr(), None, s.cuda_stream)
        torch.cuda.synchronize()
        assert m.kernel_last == pm.KIND_RT
        assert torch.equal(got, want)
    # small launches (<= 256 Ki positions: rt_small_kernel, whose deep
    # signal counts only filter-passing candidates, as the chunked kernel's
    # does): the reference's 100 KiB read_block chunks stay on RT too
    text = dt[:4 << 20].cpu().numpy()
    ref.reset()
    want_ids = ref.read_block_gids(text)
    m.reset()
    got = []
    for k in range(0, len(text), 100 << 10):
        got.append(m.read_block_gids(text[k:k + (100 << 10)]))
        assert m.kernel_last == pm.KIND_RT, k
    assert np.array_equal(np.concatenate(got), want_ids)


def test_auto_read_block_over_deep_then_sparse_blocks():
    """read_block through the auto kind: 64 MiB of the shipped stream then
    random ASCII, in 8 MiB calls (blocks switch kernels), equal to the AC
    kind's codes everywhere."""
    text = np.concatenate([_tiled_ship(40 << 20), pm.gen_stream(24 << 20, seed=9, mode=0)])
    a = matcher("et", "auto")
    r = matcher("et", "ac")
    for k in range(0, len(text), 8 << 20):
        assert np.array_equal(a.read_block_codes(text[k:k + (8 << 20)]), r.read_block_codes(text[k:k + (8 << 20)])), k


@pytest.mark.parametrize("kind", ["rt", "auto"])
def test_resident_server_small_calls(kind):
    """Small read_block calls of an rt object -- and of an auto object while
    its pick holds the reverse trie (shallow text) -- go to its resident
    server grid (rt_serve_kernel, the "host_serve" option; measure.c:77, 284):
    gids and pattern ids equal one large call's and the launch-per-call
    path's.  A grid that exits when idle ("serve_idle_us") is launched again
    by the next call -- also when it ends while a call waits for it (idle
    times about as long as the gaps between calls) -- a scan_device launch
    between calls stops it, and free() waits for it."""
    import time
    torch = _torch()
    m = fresh_matcher("snort", kind)
    sizes = [100 << 10] * 8 + [1, 17, 255 << 10, 5000, 3, 100 << 10]
    if kind == "rt":
        text = np.tile(SHIP, 1 + sum(sizes) // len(SHIP))[:sum(sizes)]
    else:  # shallow: the auto pick holds RT
        text = pm.gen_stream(sum(sizes), 9, 0)
    offs = np.cumsum([0] + sizes)
    pieces = list(zip(offs[:-1], offs[1:]))
    m.reset()
    whole = m.read_block_gids(text)  # > 256 Ki positions: the pipeline, not the server
    m.reset()
    whole_ids = m.read_block_id_array(text)
    s0 = m.serve_stats()
    m.reset()
    assert np.array_equal(np.concatenate([m.read_block_gids(text[a:b]) for a, b in pieces]), whole)
    m.reset()
    assert np.array_equal(np.concatenate([m.read_block_id_array(text[a:b]) for a, b in pieces]), whole_ids)
    s1 = m.serve_stats()
    if kind == "rt":
        assert s1["calls"] - s0["calls"] == 2 * len(sizes) and s1["launches"] >= 1
    else:  # the first call of each pass measures (a launch); the hold serves
        assert s1["calls"] - s0["calls"] >= len(sizes) and s1["launches"] >= 1
    assert m.set_option("host_serve", 0) == 0
    m.reset()
    assert np.array_equal(np.concatenate([m.read_block_gids(text[a:b]) for a, b in pieces]), whole)
    assert m.serve_stats() == s1  # launches per call
    assert m.set_option("host_serve", 1) == 0
    assert m.set_option("serve_idle_us", 9) == -1
    # idle exits between calls: every call launches a grid again
    assert m.set_option("serve_idle_us", 50) == 0
    m.reset()
    parts = []
    for a, b in pieces:
        time.sleep(0.003)
        parts.append(m.read_block_gids(text[a:b]))
    assert np.array_equal(np.concatenate(parts), whole)
    s2 = m.serve_stats()
    assert s2["launches"] - s1["launches"] >= len(sizes) // (2 if kind == "rt" else 4)
    # gaps about the idle time: grids end around the requests
    rng = np.random.default_rng(5)
    for idle in (10, 40, 200):
        assert m.set_option("serve_idle_us", idle) == 0
        m.reset()
        parts = []
        for a, b in pieces:
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < rng.uniform(0, 2.5 * idle) * 1e-6:
                pass
            parts.append(m.read_block_gids(text[a:b]))
        assert np.array_equal(np.concatenate(parts), whole), idle
    # a scan_device launch between calls
    assert m.set_option("serve_idle_us", -1) == 0
    n = 1 << 20
    dev = torch.from_numpy(np.concatenate([pm.gen_stream(n, 2, 0), np.zeros(64, np.uint8)])).cuda()
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    m.reset()
    parts = []
    for k, (a, b) in enumerate(pieces):
        parts.append(m.read_block_gids(text[a:b]))
        if k % 3 == 0:
            m.scan_device(dev.data_ptr(), 0, 0, n, out.data_ptr(), None, s)
    torch.cuda.synchronize()
    assert np.array_equal(np.concatenate(parts), whole)
    m.free()


def test_resident_servers_of_two_objects_interleaved():
    """Two rt objects in one process, each with its own resident server grid,
    their small read_block calls interleaved (the reference's loop keeps
    several slots; measure.c:324-332): each object's ids equal its own
    large call's; freeing one leaves the other serving."""
    a, b = fresh_matcher("snort", "rt"), fresh_matcher("et", "rt")
    text = pm.gen_stream(24 * (100 << 10), 4, 0)
    chunks = [(o, o + (100 << 10)) for o in range(0, len(text), 100 << 10)]
    whole = {}
    for m in (a, b):
        m.reset()
        whole[id(m)] = m.read_block_gids(text)
        m.reset()
    parts = {id(a): [], id(b): []}
    for k, (lo, hi) in enumerate(chunks):
        for m in ((a, b) if k % 2 else (b, a)):
            parts[id(m)].append(m.read_block_gids(text[lo:hi]))
    for m in (a, b):
        assert np.array_equal(np.concatenate(parts[id(m)]), whole[id(m)])
        assert m.serve_stats()["calls"] >= len(chunks)
    a.free()
    b.reset()
    assert np.array_equal(np.concatenate([b.read_block_gids(text[lo:hi]) for lo, hi in chunks]), whole[id(b)])
    b.free()


def test_resident_server_process_exit_without_free():
    """A process that ends right after a served small call, its object never
    freed, exits cleanly: the exit handler stops the live grid and waits
    for it (no grid outlives its process)."""
    import subprocess
    import sys
    import time
    code = (
        "import sys, numpy as np\n"
        f"sys.path.insert(0, {os.path.dirname(os.path.dirname(os.path.abspath(__file__)))!r})\n"
        "import patternmatching_amd as pm\n"
        f"m = pm.HipMatcher('rt'); m.add_dictionary(pm.Dictionary([{os.path.join(DATA, 'snort.dict')!r}])); m.compile()\n"
        "g = m.read_block_gids(pm.gen_stream(100 << 10, 3, 0))\n"
        "assert m.serve_stats()['calls'] == 1, m.serve_stats()\n"
        "print('served', int(np.count_nonzero(g)))\n")
    t0 = time.time()
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "served" in r.stdout
    assert time.time() - t0 < 90
