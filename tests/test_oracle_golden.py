"""Pin the oracle (oracle/ac_oracle.c) against the reference's own outputs
(tests/golden/, produced by tests/golden/gen_golden.py from the reference
compiled by oracle/Makefile)."""
import json
import os

import numpy as np
import pytest

from oracle_lib import DATA, GOLDEN, Oracle, dict_paths, fnv1a64_codes, oracle_for, parse_line
import oracle_lib

MANIFEST = json.load(open(os.path.join(GOLDEN, "manifest.json")))
SHIP = np.fromfile(os.path.join(DATA, "dictionaries_generated.stream"), dtype=np.uint8)


@pytest.mark.parametrize("key", ["et", "snort", "merged"])
def test_stats(key):
    st = MANIFEST["stats"][key]
    o = oracle_for(key)
    assert o.n_patterns == st["unique"]
    assert o.n_states == st["ac_states"]
    assert o.max_len == st["max_len"]


def test_results_csv_memory():
    # results.csv:2: AC "Total Memory Used" 1,485,093,592 B = 716,744 states x 2072 B + 24 B
    assert MANIFEST["stats"]["merged"]["ac_total_mem"] == 1485093592
    assert oracle_for("merged").n_states * 2072 + 24 == 1485093592


@pytest.mark.parametrize("key", ["et", "snort", "merged"])
def test_ship_stream_dense(key):
    gold = np.fromfile(os.path.join(GOLDEN, f"ship_{key}.u32"), dtype="<u4")
    o = oracle_for(key)
    o.reset()
    got = o.scan_codes(SHIP)
    assert got.shape == gold.shape
    bad = np.nonzero(got != gold)[0]
    assert bad.size == 0, f"first mismatch at {bad[:5]}"


@pytest.mark.parametrize("case", [d for d in MANIFEST["digests"] if d["n"] <= (1 << 20)],
                         ids=lambda d: f"{d['dict']}-s{d['seed']}-m{d['mode']}")
def test_seeded_digest(case):
    from patternmatching_amd import gen_stream
    o = oracle_for(case["dict"])
    o.reset()
    codes = o.scan_codes(gen_stream(case["n"], case["seed"], case["mode"]))
    assert int(np.count_nonzero(codes)) == case["nonnull"]
    nz = np.nonzero(codes)[0][:len(case["first"])]
    assert [[int(i), int(codes[i])] for i in nz] == case["first"]
    assert fnv1a64_codes(codes) == case["fnv1a64"]


def test_seeded_digest_64mib_et():
    """BASELINE config 2's stream (et, 64 MiB ASCII) through the oracle."""
    from patternmatching_amd import gen_stream
    case = [d for d in MANIFEST["digests"] if d["n"] == 64 << 20][0]
    o = oracle_for("et")
    o.reset()
    codes = o.scan_codes(gen_stream(case["n"], case["seed"], case["mode"]))
    assert int(np.count_nonzero(codes)) == case["nonnull"]
    assert fnv1a64_codes(codes) == case["fnv1a64"]


def test_ship_x64_merged():
    import hashlib
    o = oracle_for("merged")
    o.reset()
    codes = o.scan_codes(np.tile(SHIP, 64))
    g = MANIFEST["ship_x64_merged"]
    assert int(np.count_nonzero(codes)) == g["nonnull"]
    assert hashlib.sha256(codes.astype("<u4").tobytes()).hexdigest() == g["sha256"]


def test_kmp_kat():
    """Core/src/kmprt.c:303-326: matches at 17 and 42."""
    o = Oracle([os.path.join(DATA, "kmp_kat.dict")])
    codes = o.scan_codes(np.fromfile(os.path.join(DATA, "kmp_kat.stream"), dtype=np.uint8))
    assert list(np.nonzero(codes)[0]) == MANIFEST["kmp_kat"] == [17, 42]


def test_parser_kat():
    lines = open(os.path.join(DATA, "parser_kat.dict"), "rb").read().split(b"\n")[:-1]
    gold = MANIFEST["parser"]["parser_kat.dict"]
    for i, line in enumerate(lines, 1):
        got = parse_line(line)
        exp = gold.get(str(i))
        assert (got.hex() if got else None) == exp, (i, line)


def test_state_carries_across_calls():
    o = oracle_for("merged")
    o.reset()
    whole = o.scan_codes(SHIP)
    o.reset()
    parts = np.concatenate([o.scan_codes(SHIP[a:b]) for a, b in ((0, 1), (1, 4000), (4000, 4001), (4001, 10240))])
    assert np.array_equal(whole, parts)
