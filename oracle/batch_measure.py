#!/usr/bin/env python3
"""TEST INFRASTRUCTURE ONLY.  Prints the reference's Core/src/measure.c with
the edit INTEGRATION.md §2 asks a maintainer to make -- the per-byte loop at
measure.c:292-294 replaced by one read_block call when the algorithm's slot
has one, the loop otherwise -- for oracle/Makefile to compile from stdin
(`make refloopb`).  Nothing is written to disk: the edited source exists
only in the pipe to gcc; the result is one object under oracle/_ref/.

The slot's batch entry is the table `mps_read_block[MPS_SIZE]` (defined by
oracle/mphip.c under PM_READ_BLOCK_HOOK), which stands in for the optional
MpsElem member of INTEGRATION.md §2: adding a member to MpsElem would change
the layout every other reference object was compiled against.  Exits 1 if
either anchor is not found exactly once.  Usage: batch_measure.py MEASURE_C"""
import re
import sys

src = open(sys.argv[1]).read()
loop = re.compile(r"for \(j = 0; j < len_read; \+\+j\) \{\s*algo_results\[j\] = read_char_func\(obj, stream_buffer\[j\]\);\s*\}")
fn = "static void measure_single_instance_stats("
if len(loop.findall(src)) != 1 or src.count(fn) != 1:
    sys.exit("batch_measure.py: anchors not found exactly once in " + sys.argv[1])
src = loop.sub("if (mps_read_block[inst->algo])\n"
               "\t\t\t\tmps_read_block[inst->algo](obj, stream_buffer, (size_t)len_read, algo_results);\n"
               "\t\t\telse\n"
               "\t\t\t\tfor (j = 0; j < len_read; ++j) algo_results[j] = read_char_func(obj, stream_buffer[j]);", src)
src = src.replace(fn, "extern void (*mps_read_block[MPS_SIZE])(void*, const char*, size_t, pattern_id_t*);\n" + fn)
sys.stdout.write(src)
