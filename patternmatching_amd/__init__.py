"""patternmatching_amd -- MI355X-native streaming multi-pattern matcher.

A drop-in for the per-byte matcher path of yehonatan145/PatternMatching
(the ``mps_table`` plugin interface, Core/src/mps.h:71-80, driven by the
``-d/-s`` stream loop of Core/src/measure.c:241-311).  The scan runs in
hand-written HIP kernels for gfx950 (``csrc/pm_kernels.hip``) behind a
C-ABI (``include/pm_hip.h``); this package is the Python host mirror of that
interface:

    Dictionary      Core/src/PatternsTree.c:260-312 + parser.c:63-99
    HipMatcher      one MpsElem instance (create / add_pattern / compile /
                    read_char / read_block / reset / total_mem / free)
    gen_stream      the synthetic stream specification
"""
from ._lib import load, LIB_PATH, CLI_PATH  # noqa: F401
from .matcher import (  # noqa: F401
    Dictionary,
    HipMatcher,
    gen_stream,
    parse_line,
    KIND_RT,
    KIND_AC,
    KIND_AUTO,
)

__all__ = ["load", "Dictionary", "HipMatcher", "gen_stream", "parse_line", "KIND_RT", "KIND_AC", "KIND_AUTO",
           "LIB_PATH", "CLI_PATH"]
