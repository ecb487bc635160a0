"""The drop-in through the reference's own code (SURVEY
§8b): the plugin table slot is layout-compatible with Core/src/mps.h, the
INTEGRATION.md registration stub compiles against the reference's headers,
and the reference's unmodified program loop -- init_mps, measure_instances_stats
(read_char per byte, measure.c:292-294; the reliable AC and
measure_success_rate, :300-303) and write_stats_to_file -- runs the HIP
plugin exactly (oracle/ref_loop.c, oracle/mphip.c; built here by
oracle/Makefile from the reference's sources, the binary travels to the GPU
box with libpm.so)."""
import csv
import json
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SRC = "/root/reference/Core/src"
REF_LOOP = os.path.join(REPO, "oracle", "_ref", "ref_loop")
REF_LOOP_BATCHED = os.path.join(REPO, "oracle", "_ref", "ref_loop_batched")
DATA = os.path.join(REPO, "tests", "golden", "data")
needs_ref = pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference sources only in the build container")


@needs_ref
def test_plugin_slot_layout_matches_reference_mps_h():
    """oracle/abi_check.c: _Static_asserts of every MpsElem member's offset
    and size against PmMpsElem, pattern_id_t vs pm_pattern_id_t, MpsInstance."""
    r = subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "abicheck"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@needs_ref
def test_abi_check_fires_on_a_wrong_layout(tmp_path):
    """The check is not vacuous: a slot with two members swapped fails it."""
    src = open(os.path.join(REPO, "oracle", "abi_check.c")).read()
    hdr = open(os.path.join(REPO, "include", "pm_mps.h")).read()
    bad = hdr.replace("    void (*compile)(void*);\n    pm_pattern_id_t (*read_char)(void*, char);\n    size_t (*total_mem)(void*);",
                      "    void (*compile)(void*);\n    size_t (*total_mem)(void*);\n    pm_pattern_id_t (*read_char)(void*, char);")
    assert bad != hdr
    (tmp_path / "pm_mps.h").write_text(bad)
    (tmp_path / "abi_check.c").write_text(src)
    r = subprocess.run(["gcc", "-fsyntax-only", f"-I{REF_SRC}", f"-I{tmp_path}", str(tmp_path / "abi_check.c")],
                       capture_output=True, text=True)
    assert r.returncode != 0 and "offset of" in r.stderr


@needs_ref
def test_registration_stub_and_reference_loop_build():
    """mphip.c compiles against the reference's mps.h
    both ways: the unmodified enum, and with the maintainer's enum edit and
    read_block member."""
    r = subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "refloop", "refloopb"], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stderr
    assert os.path.exists(REF_LOOP) and os.path.exists(REF_LOOP_BATCHED)
    r = subprocess.run(["gcc", "-fsyntax-only", "-w", f"-I{REF_SRC}", f"-I{os.path.join(REPO, 'include')}",
                        "-DMPS_HIP_RT=3", "-DMPS_HIP_AC=4", "-DMPS_HIP_AUTO=5",
                        os.path.join(REPO, "oracle", "mphip.c")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@needs_ref
def test_batch_edit_of_the_reference_loop(tmp_path):
    """oracle/batch_measure.py makes exactly INTEGRATION.md §2's edit: the
    per-byte loop of measure.c:292-294 becomes one read_block call when the
    slot has one, the loop otherwise; everything else is unchanged."""
    r = subprocess.run(["python3", os.path.join(REPO, "oracle", "batch_measure.py"), os.path.join(REF_SRC, "measure.c")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    orig = open(os.path.join(REF_SRC, "measure.c")).read()
    edited = r.stdout
    assert "mps_read_block[inst->algo](obj, stream_buffer, (size_t)len_read, algo_results);" in edited
    assert edited.count("read_char_func(obj, stream_buffer[j])") == 1
    import difflib
    changed = [ln for ln in difflib.unified_diff(orig.splitlines(), edited.splitlines(), lineterm="", n=0)
               if ln[:1] in "+-" and not ln.startswith(("+++", "---"))]
    assert len(changed) <= 10, changed


def _ref_loop(tmp_path, dict_names, stream_path, bg, lmac=None, timeout=600, exe=REF_LOOP):
    out = tmp_path / "results.csv"
    # write_stats_to_file opens O_WRONLY | O_CREAT with no mode (measure.c:348;
    # SURVEY App. A 3): create the file first so it stays readable
    out.write_text("")
    os.chmod(out, 0o644)
    env = dict(os.environ, PM_REF_BG=bg)
    if lmac:
        env["PM_REF_LMAC"] = lmac
    args = [exe]
    for d in dict_names:
        args += ["-d", os.path.join(DATA, d)]
    args += ["-s", str(stream_path), "-o", str(out)]
    r = subprocess.run(args, capture_output=True, text=True, timeout=timeout, env=env, cwd=tmp_path)
    assert r.returncode == 0, (r.stdout[-1000:], r.stderr[-2000:])
    rows = list(csv.reader(open(out)))
    head = rows[0]
    return {row[0]: dict(zip(head, row)) for row in rows[1:] if row}


@pytest.mark.gpu
def test_reference_loop_runs_the_hip_plugin_exactly(tmp_path):
    """C1 (et.dict + the shipped stream) through the reference's own
    program: the HIP rows of its CSV show zero false-positive, false-negative
    and partial rates against the reference AC, and non-zero memory."""
    assert os.path.exists(REF_LOOP), "build it in the build container: make -C oracle refloop"
    res = _ref_loop(tmp_path, ["et.dict"], os.path.join(DATA, "dictionaries_generated.stream"), "rt", "auto")
    assert set(res) == {"Aho-Corasick", "HIP Auto (RT / AC per launch)", "HIP Reverse-Trie"}, res.keys()
    for name, row in res.items():
        assert float(row["False Positive Rate"]) == 0.0, (name, row)
        assert float(row["False Negative Rate"]) == 0.0, (name, row)
        assert float(row["Partial Success Rate"]) == 0.0, (name, row)
        assert int(row["Total Memory Used"]) > 0


@pytest.mark.gpu
def test_reference_loop_per_byte_rate(tmp_path):
    """The per-byte read_char rate through the reference's loop (clock()
    time of measure.c:290-297, 16 MiB of snort ASCII): the HIP kinds' host
    step against the reference AC in the same run; all exact."""
    import patternmatching_amd as pm
    n = 16 << 20
    stream = tmp_path / "ascii16M.stream"
    pm.gen_stream(n, seed=5, mode=0).tofile(stream)
    res = _ref_loop(tmp_path, ["snort.dict"], stream, "rt", "ac", timeout=900)
    rates = {}
    for name, row in res.items():
        assert float(row["False Positive Rate"]) == 0.0 and float(row["False Negative Rate"]) == 0.0, (name, row)
        assert float(row["Partial Success Rate"]) == 0.0, (name, row)
        rates[name] = n / max(float(row["Time (in secs)"]), 1e-9) / 1e6
    ev = os.environ.get("PM_EVIDENCE_DIR")
    if ev:
        os.makedirs(ev, exist_ok=True)
        with open(os.path.join(ev, "ref_loop_per_byte_rate.json"), "w") as f:
            json.dump({"bytes": n, "stream": "seed-5 ascii", "dict": "snort.dict", "MBps_per_core": rates,
                       "what": "reference program loop (oracle/ref_loop.c), read_char per byte, clock() time"}, f)
    assert rates["HIP Reverse-Trie"] >= rates["Aho-Corasick"], rates


# /root/reference/results.csv:2-3, the reference's published run
# `-d snort.dict -d et.dict -s dictionaries_generated.stream`:
# AC 716,744 states x 2,072 B + 24 B; LMAC's list nodes.
PUBLISHED_AC_MEMORY = 1485093592
PUBLISHED_LMAC_MEMORY = 40137664


@pytest.mark.gpu
@pytest.mark.parametrize("slots", [("auto", "rt"), ("auto", None)], ids=["bg_auto+lmac_rt", "bg_auto+lmac_ref"])
def test_reference_published_run_reproduced(tmp_path, slots):
    """The reference's published command, literally, through its own program
    with the batch call (oracle/_ref/ref_loop_batched): both dictionaries in
    results.csv's order and the shipped stream.  The AC row's Total Memory
    Used equals results.csv:2 (and, with the reference's LMAC kept in its
    slot, LMAC's equals results.csv:3); every row, the HIP ones included, has
    zero false-positive, false-negative and partial rates against the
    reference AC (measure.c:300-303)."""
    assert os.path.exists(REF_LOOP_BATCHED), "build it in the build container: make -C oracle refloopb"
    bg, lmac = slots
    res = _ref_loop(tmp_path, ["snort.dict", "et.dict"], os.path.join(DATA, "dictionaries_generated.stream"), bg,
                    lmac, exe=REF_LOOP_BATCHED)
    want = {"Aho-Corasick", "HIP Auto (RT / AC per launch)",
            "HIP Reverse-Trie" if lmac else "Low-Memory Aho-Corasick"}
    assert set(res) == want, res.keys()
    assert int(res["Aho-Corasick"]["Total Memory Used"]) == PUBLISHED_AC_MEMORY
    if not lmac:
        assert int(res["Low-Memory Aho-Corasick"]["Total Memory Used"]) == PUBLISHED_LMAC_MEMORY
    for name, row in res.items():
        assert float(row["False Positive Rate"]) == 0.0, (name, row)
        assert float(row["False Negative Rate"]) == 0.0, (name, row)
        assert float(row["Partial Success Rate"]) == 0.0, (name, row)
        assert int(row["Total Memory Used"]) > 0
    ev = os.environ.get("PM_EVIDENCE_DIR")
    if ev:
        os.makedirs(ev, exist_ok=True)
        tag = f"bg_{bg}_lmac_{lmac or 'ref'}"
        with open(tmp_path / "results.csv") as src, open(os.path.join(ev, f"published_run_{tag}.csv"), "w") as dst:
            dst.write(src.read())


@pytest.mark.gpu
def test_reference_loop_with_the_batch_call_is_exact(tmp_path):
    """The reference's program with INTEGRATION.md §2's batch call
    (oracle/_ref/ref_loop_batched): every 100 KiB chunk of the loop
    (measure.c:77, 284) goes to the GPU kernels through read_block, scored by
    the reference's own measure_success_rate against its AC -- C1 (et.dict +
    the shipped stream) and 16 MiB of snort ASCII, rt and auto slots: zero
    false-positive, false-negative and partial rates."""
    assert os.path.exists(REF_LOOP_BATCHED), "build it in the build container: make -C oracle refloopb"
    import patternmatching_amd as pm
    res = _ref_loop(tmp_path, ["et.dict"], os.path.join(DATA, "dictionaries_generated.stream"), "rt", "auto",
                    exe=REF_LOOP_BATCHED)
    assert set(res) == {"Aho-Corasick", "HIP Auto (RT / AC per launch)", "HIP Reverse-Trie"}, res.keys()
    n = 16 << 20
    stream = tmp_path / "ascii16M.stream"
    pm.gen_stream(n, seed=5, mode=0).tofile(stream)
    res2 = _ref_loop(tmp_path, ["snort.dict"], stream, "rt", "ac", timeout=900, exe=REF_LOOP_BATCHED)
    secs = {}
    for r in (res, res2):
        for name, row in r.items():
            assert float(row["False Positive Rate"]) == 0.0, (name, row)
            assert float(row["False Negative Rate"]) == 0.0, (name, row)
            assert float(row["Partial Success Rate"]) == 0.0, (name, row)
    for name, row in res2.items():
        secs[name] = float(row["Time (in secs)"])
    ev = os.environ.get("PM_EVIDENCE_DIR")
    if ev:
        os.makedirs(ev, exist_ok=True)
        with open(os.path.join(ev, "ref_loop_batched.json"), "w") as f:
            json.dump({"bytes": n, "stream": "seed-5 ascii", "dict": "snort.dict", "clock_seconds": secs,
                       "what": "reference program loop with INTEGRATION.md's batch call (oracle/_ref/ref_loop_batched): "
                               "read_block per 100 KiB chunk for the HIP slots, read_char per byte for the reference "
                               "AC; the CSV's Time column is clock(), process CPU time, which leaves out time the "
                               "thread sleeps waiting for the GPU"}, f)
