#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Run in the build container only (it needs /root/reference and
oracle/_ref/ref_driver, built by `make -C oracle ref` from the reference's
own C sources).  The outputs are data: inputs copied from the reference's
data directories plus the outputs the reference's own Aho-Corasick path
(Core/src/mpac.c via mps_table[MPS_AC]) produced for them.

    python tests/golden/gen_golden.py          # everything
    python tests/golden/gen_golden.py tree     # only the patterns-tree fixtures
"""
import hashlib
import json
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
DRIVER = os.path.join(REPO, "oracle", "_ref", "ref_driver")
DATA = os.path.join(HERE, "data")

DICTS = {
    "et": ["et.dict"],
    "snort": ["snort.dict"],
    "merged": ["snort.dict", "et.dict"],  # results.csv's configuration
}

# Parser known-answer lines (SURVEY §8a, A11 rules).  Each entry is one line
# of a synthetic dictionary; the reference parser decides what it becomes.
PARSER_LINES = [
    b"plain",
    b"|41 42|",
    b"|41 |",            # space before closing bar -> rejected
    b"|4142|x",
    b"| 4 1 42|",
    b"|414|",            # odd nibble count -> rejected
    b"|41",              # unterminated -> rejected
    b"a||b",             # empty hex block
    b"| |",              # rejected
    b"",                 # empty line, counted
    b"cr\r",             # \r is kept
    b"nul\x00byte",      # NUL inside a literal
    b"|00 ff 7F|",
    b"|0g|",             # non-hex -> rejected
    b"plain",            # duplicate of line 1 (dedup is not the parser's job)
    b"x|20|y|7c|z",
    b"||",               # empty result -> skipped
    b"|4 1|",
    b"   ",
    b"|41|\xff\xfe",
]


def run(args, **kw):
    return subprocess.run(args, check=True, capture_output=True, **kw).stdout


def sha256(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def gen_tree(manifest):
    """(6) The reference's patterns tree (PatternsTree.h:90-94): each pattern's
    PatternsTreeNode->parent as codes (tree_<key>.u32.gz: u32 pairs in add
    order, 0 = the root), and is_pattern_suffix (PatternsTree.c:485-494) on
    2048 sampled pairs (suffix_<key>.u32: u32 triples first, second, result)."""
    import gzip
    manifest["tree"] = {}
    for key in DICTS:
        dp = [os.path.join(DATA, d) for d in DICTS[key]]
        raw = os.path.join("/tmp", f"tree_{key}.u32")
        run([DRIVER, "parents", raw] + dp)
        with open(raw, "rb") as f:
            blob = f.read()
        out = os.path.join(HERE, f"tree_{key}.u32.gz")
        with gzip.GzipFile(out, "wb", mtime=0) as f:
            f.write(blob)
        suf = os.path.join(HERE, f"suffix_{key}.u32")
        run([DRIVER, "suffix", suf, "7", "2048"] + dp)
        manifest["tree"][key] = {"parents": os.path.basename(out), "parents_sha256": hashlib.sha256(blob).hexdigest(),
                                 "patterns": len(blob) // 8, "suffix": os.path.basename(suf),
                                 "suffix_sha256": sha256(suf)}


def main():
    if not os.path.exists(DRIVER):
        sys.exit("build the reference driver first: make -C oracle ref")
    if sys.argv[1:] == ["tree"]:  # only section (6), into the existing manifest
        path = os.path.join(HERE, "manifest.json")
        with open(path) as f:
            manifest = json.load(f)
        gen_tree(manifest)
        with open(path, "w") as f:
            json.dump(manifest, f, indent=1, sort_keys=True)
        return
    os.makedirs(DATA, exist_ok=True)
    for name in ("et.dict", "snort.dict"):
        shutil.copyfile(os.path.join(REF, "Dictionaries", name), os.path.join(DATA, name))
    shutil.copyfile(os.path.join(REF, "Streams", "dictionaries_generated.stream"),
                    os.path.join(DATA, "dictionaries_generated.stream"))
    ship = os.path.join(DATA, "dictionaries_generated.stream")
    manifest = {"source": "reference Core/src compiled by oracle/Makefile; driver oracle/ref_driver.c",
                "files": {}, "stats": {}, "ship": {}, "digests": [], "parser": {}}
    for name in ("et.dict", "snort.dict", "dictionaries_generated.stream"):
        manifest["files"][name] = sha256(os.path.join(DATA, name))

    def dpaths(key):
        return [os.path.join(DATA, d) for d in DICTS[key]]

    # (1) aggregate cross-checks
    for key in DICTS:
        st = json.loads(run([DRIVER, "stats"] + dpaths(key)))
        st["ac_states"] = (st["ac_total_mem"] - 24) // 2072  # mpac.c:328-332
        manifest["stats"][key] = st

    # (2) dense per-position codes on the shipped adversarial stream
    for key in DICTS:
        out = os.path.join(HERE, f"ship_{key}.u32")
        run([DRIVER, "dense", out, ship] + dpaths(key))
        manifest["ship"][key] = {"file": os.path.basename(out), "sha256": sha256(out)}

    # tiled shipped stream (deep states across many tiles); digest only
    tiled = os.path.join("/tmp", "ship_x64.stream")
    with open(ship, "rb") as f:
        blob = f.read()
    with open(tiled, "wb") as f:
        f.write(blob * 64)
    out = os.path.join("/tmp", "ship_x64.u32")
    run([DRIVER, "dense", out, tiled] + dpaths("merged"))
    with open(out, "rb") as f:
        dense = f.read()
    manifest["ship_x64_merged"] = {"n": len(blob) * 64, "sha256": hashlib.sha256(dense).hexdigest(),
                                   "nonnull": sum(1 for i in range(0, len(dense), 4)
                                                  if dense[i:i + 4] != b"\0\0\0\0")}

    # (3) seeded synthetic streams (oracle/streamgen.h): digest + first records
    cases = [("et", 1, 0, 1 << 20), ("snort", 1, 0, 1 << 20), ("merged", 1, 0, 1 << 20),
             ("snort", 2, 1, 1 << 20), ("et", 3, 0, 64 << 20)]
    for key, seed, mode, n in cases:
        d = json.loads(run([DRIVER, "digest", str(seed), str(mode), str(n)] + dpaths(key)))
        d["dict"] = key
        manifest["digests"].append(d)

    # (4) parser known answers
    kat = os.path.join(DATA, "parser_kat.dict")
    with open(kat, "wb") as f:
        f.write(b"\n".join(PARSER_LINES) + b"\n")
    accepted = {}
    for ln in run([DRIVER, "parse", kat]).decode().split("\n"):
        if ln.strip():
            num, hx = ln.split(" ")
            accepted[num] = hx
    manifest["parser"]["parser_kat.dict"] = accepted
    for name in ("et.dict", "snort.dict"):
        lines = run([DRIVER, "parse", os.path.join(DATA, name)]).decode().split("\n")
        acc = [int(l.split(" ")[0]) for l in lines if l.strip()]
        with open(os.path.join(DATA, name), "rb") as f:
            total = f.read().count(b"\n")
        nonempty_rejected = []
        with open(os.path.join(DATA, name), "rb") as f:
            for i, raw in enumerate(f.read().split(b"\n")[:total], 1):
                if raw and i not in set(acc):
                    nonempty_rejected.append(i)
        manifest["parser"][name] = {"accepted": len(acc), "lines": total,
                                    "rejected_nonempty": nonempty_rejected,
                                    "sha256": hashlib.sha256("\n".join(lines).encode()).hexdigest()}

    # (5) KMP-RT known answer (Core/src/kmprt.c:303-326, commented-out test):
    # pattern AAAAAAAAAAAAAAAAAB over the 50-char text matches at 17 and 42.
    kd = os.path.join(DATA, "kmp_kat.dict")
    ks = os.path.join(DATA, "kmp_kat.stream")
    with open(kd, "wb") as f:
        f.write(b"AAAAAAAAAAAAAAAAAB\n")
    with open(ks, "wb") as f:
        f.write(b"AAAAAAAAAAAAAAAAABAAAAAABAAAAAAAAAAAAAAAAABAAAAAAA")
    out = os.path.join("/tmp", "kmp.u32")
    run([DRIVER, "dense", out, ks, kd])
    with open(out, "rb") as f:
        d = f.read()
    manifest["kmp_kat"] = [i // 4 for i in range(0, len(d), 4) if d[i:i + 4] != b"\0\0\0\0"]

    gen_tree(manifest)

    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print(json.dumps({k: manifest[k] for k in ("stats", "kmp_kat")}, indent=1))


if __name__ == "__main__":
    main()
