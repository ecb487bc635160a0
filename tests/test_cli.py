"""The drop-in CLI (`pm`, the reference's `exe`: main.c:7-24, -d/-s/-o/-v)."""
import os
import subprocess

import numpy as np
import pytest

import patternmatching_amd as pm
from oracle_lib import DATA, GOLDEN


def test_cli_usage_errors():
    r = subprocess.run([pm.CLI_PATH, "-o", "a", "-o", "b", "-d", "x"], capture_output=True, text=True)
    assert r.returncode != 0 and "more than one output file" in r.stderr  # parser.c:117-121
    r = subprocess.run([pm.CLI_PATH, "-q"], capture_output=True, text=True)
    assert r.returncode != 0 and "Unknown option -q" in r.stderr
    r = subprocess.run([pm.CLI_PATH, "-d"], capture_output=True, text=True)
    assert r.returncode != 0 and "must have argument" in r.stderr


@pytest.mark.gpu
def test_cli_et_shipped_stream(tmp_path):
    """BASELINE config 1 through the drop-in CLI: every GPU matcher, scored
    against the reliable instance (0 FP/FN/partial), dump == golden."""
    csv = tmp_path / "res.csv"
    dump = tmp_path / "m.u32"
    ship = os.path.join(DATA, "dictionaries_generated.stream")
    r = subprocess.run([pm.CLI_PATH, "-d", os.path.join(DATA, "et.dict"), "-s", ship, "-s", ship, "-o", str(csv),
                        "-m", str(dump), "-v", "-B", "4096"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    lines = csv.read_text().strip().split("\n")
    assert lines[0].startswith("Algorithm,Time (in secs),Total Memory Used,False Positive Rate,"
                               "False Negative Rate,Partial Success Rate")
    rows = {l.split(",")[0]: l.split(",") for l in lines[1:]}
    assert set(rows) == {"HIP Reverse-Trie", "HIP Aho-Corasick DFA", "HIP Auto (RT / AC per launch)"}
    for row in rows.values():
        assert row[3:6] == ["0.000000", "0.000000", "0.000000"]
        assert int(row[9]) == 2 * 10240
        assert len(row) == 12 and 0.0 < float(row[10]) < 1.0 and row[11] == "0"  # roofline frac, GPU id
    gold = np.fromfile(os.path.join(GOLDEN, "ship_et.u32"), dtype="<u4")
    got = np.fromfile(dump, dtype="<u4")
    assert np.array_equal(got, np.concatenate([gold, gold]))  # reset per stream file
    assert oct(os.stat(csv).st_mode & 0o777) == "0o644"
