#!/bin/bash
# Side-by-side sparse-DFA timing of library builds on ONE box:
# ab_dfa_forms.sh TAG lib1 lib2 ... (alternating, 2 passes; dfa_coded_sweep.py
# with the sparse form at the product shape).
set -o pipefail
OUT=gpurun_out/ab_$1; shift; mkdir -p $OUT
for pass in 1 2; do
  for lib in "$@"; do
    PM_LIBPM=$(pwd)/$lib timeout -k 10 300 python scripts/dfa_coded_sweep.py --forms 1 --lanes ${LANES:-512} --chains 1 \
        > $OUT/tmp.txt 2>&1 || { tail $OUT/tmp.txt; exit 1; }
    grep -v amdgpu $OUT/tmp.txt | grep -v "^{" | sed "s|^|$pass $lib |" | tee -a $OUT/ab.txt
  done
done
