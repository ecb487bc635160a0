"""The patterns tree pinned to the reference's own (A12):
tests/golden/tree_<key>.u32.gz holds each pattern's PatternsTreeNode->parent
(PatternsTree.h:90-94) as dumped by oracle/_ref/ref_driver from the
reference's objects, and suffix_<key>.u32 holds is_pattern_suffix
(PatternsTree.c:485-494) on sampled pairs (tests/golden/gen_golden.py).
Checked here against the host tree (pm_dict_finalize, the CLI's scoring)
and the gid-space parent[] / depth[] the device scoring kernels read
(pm_build_parents).  CPU only."""
import ctypes
import gzip
import json
import os

import numpy as np
import pytest

import patternmatching_amd as pm
from oracle_lib import GOLDEN, dict_paths
from table_emulator import FlatImage

MANIFEST = json.load(open(os.path.join(GOLDEN, "manifest.json")))
_d = {}


def tree(key):
    if key not in _d:
        with gzip.open(os.path.join(GOLDEN, f"tree_{key}.u32.gz"), "rb") as f:
            pairs = np.frombuffer(f.read(), "<u4").reshape(-1, 2)
        d = pm.Dictionary(dict_paths(key))
        code_to_index = {int(c): i for i, c in enumerate(d.codes())}
        _d[key] = (d, pairs, code_to_index)
    return _d[key]


@pytest.mark.parametrize("key", ["et", "snort", "merged"])
def test_fixture_matches_manifest(key):
    import hashlib
    with gzip.open(os.path.join(GOLDEN, f"tree_{key}.u32.gz"), "rb") as f:
        blob = f.read()
    m = MANIFEST["tree"][key]
    assert hashlib.sha256(blob).hexdigest() == m["parents_sha256"]
    assert len(blob) // 8 == m["patterns"] == MANIFEST["stats"][key]["unique"]


@pytest.mark.parametrize("key", ["et", "snort", "merged"])
def test_host_tree_parent_is_the_reference_parent(key):
    d, pairs, c2i = tree(key)
    assert d.n == len(pairs) and set(c2i) == set(int(c) for c in pairs[:, 0])
    host = d.parents()  # pattern index -> parent index, -1 = the root
    codes = d.codes()
    got = np.array([codes[host[c2i[int(c)]]] if host[c2i[int(c)]] >= 0 else 0 for c in pairs[:, 0]], np.uint32)
    assert np.array_equal(got, pairs[:, 1])
    assert (pairs[:, 1] != 0).sum() > 0.5 * len(pairs)  # most patterns have a proper suffix pattern


@pytest.mark.parametrize("key", ["et", "snort", "merged"])
def test_device_parent_and_depth_tables_are_the_reference_tree(key):
    """parent[] / depth[] in gid space (the score_kernel / hist_kernel
    inputs) follow the reference tree; depth = patterns on the chain."""
    d, pairs, c2i = tree(key)
    img = FlatImage(d.patterns(), pm.KIND_RT)
    idx = img.array("index_of_gid").astype(np.int64)
    parent = img.array("parent").astype(np.int64)
    depth = img.array("depth").astype(np.int64)
    codes = d.codes()
    gid_of_code = {int(codes[idx[g]]): g for g in range(1, len(idx))}
    ref_parent = {int(a): int(b) for a, b in pairs}
    for g in range(1, len(idx)):
        c = int(codes[idx[g]])
        pc = ref_parent[c]
        assert parent[g] == (gid_of_code[pc] if pc else 0), (g, c, pc)
    # depth: walk the reference chain
    ref_depth = {}

    def rdepth(c):
        if c == 0:
            return 0
        if c not in ref_depth:
            ref_depth[c] = 1 + rdepth(ref_parent[c])
        return ref_depth[c]

    import sys
    sys.setrecursionlimit(10000)
    for g in range(1, len(idx)):
        assert depth[g] == rdepth(int(codes[idx[g]]))


@pytest.mark.parametrize("key", ["et", "snort", "merged"])
def test_is_pattern_suffix_matches_the_reference(key):
    """pm_pattern_is_suffix (the host scoring's partial test) gives the
    reference's is_pattern_suffix on the sampled pairs."""
    d, pairs, c2i = tree(key)
    trip = np.fromfile(os.path.join(GOLDEN, f"suffix_{key}.u32"), "<u4").reshape(-1, 3)
    assert trip[:, 2].sum() > 0.3 * len(trip) and (trip[:, 0] == 0).sum() > 0
    lib = pm.load()

    def pid(code):
        return ctypes.c_void_p(d.pattern_ptr(c2i[int(code)])) if code else ctypes.c_void_p(0)

    for a, b, r in trip:
        assert lib.pm_pattern_is_suffix(pid(a), pid(b)) == int(r), (a, b, r)
