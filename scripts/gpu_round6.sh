#!/bin/bash
# Round-6 measurement session: GPU tests, smoke, the default bench line, and
# for every leg of that line (headline C3, count only, deep, and each
# `configs` entry) one rocprofv3 --kernel-trace --stats run of the
# equivalent single-workload bench command plus the two PMC traffic passes
# (FETCH_SIZE, WRITE_SIZE; for the DFA legs TCP_TCC_READ_REQ_sum too: one
# counter per pass, --kernel-trace only).
# Usage: gpu_round5.sh TAG [legs...]   (legs default: all; "tests" / "bench"
# / a leg name).  Every GPU step has its own time limit; the first failure
# ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${1:-r06}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
shift
WANT=" ${*:-tests bench c3 count deep c2 c5 merged_lines merged_ship} "
export PM_EVIDENCE_DIR=$OUT
echo "== $(date) host cpus $(nproc) share ${OMP_NUM_THREADS:-?}"
if [[ $WANT == *" tests "* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 || { tail "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
if [[ $WANT == *" bench "* ]]; then
  timeout -k 10 900 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('C3', d['value'], 'kernel_ms', d['kernel_ms'], 'frac', d['roofline']['frac'], 'count', d['count_only']['kernel_ms'], 'deep', d['deep']['kernel_ms'], d['deep']['picked'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores']); print({k: (v['kernel_ms'], v['stream_gbps'], v['roofline']['frac'], v['kernel']) for k, v in d.get('configs', {}).items()})"
fi
cd /tmp && export TMPDIR=/tmp
# leg -> bench arguments (the equivalent single-workload run) and steps
declare -A ARGS=(
  [c3]="--steps 10"
  [count]="--mode count --steps 10"
  [deep]="--stream lines --kernel auto --steps 5"
  [c2]="--dict et --bytes 67108864 --steps 20"
  [c5]="--dict merged --bytes 4294967296 --steps 5"
  [merged_lines]="--dict merged --stream lines --kernel auto --steps 5"
  [merged_ship]="--dict merged --stream ship --kernel auto --steps 5"
)
for leg in c3 count deep c2 c5 merged_lines merged_ship; do
  [[ $WANT == *" $leg "* ]] || continue
  a=${ARGS[$leg]}
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$leg" -o bench -- \
      python3 "$ROOT/bench.py" --no-cpu --no-extra $a > "$OUT/bench_prof_$leg.json" 2> "$OUT/bench_prof_$leg.err" \
      || { tail "$OUT/bench_prof_$leg.err"; exit 1; }
  CTRS="FETCH_SIZE WRITE_SIZE"
  case $leg in deep|merged_lines|merged_ship) CTRS="$CTRS TCP_TCC_READ_REQ_sum";; esac
  for c in $CTRS; do
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/pmc_$leg/$c" -o c -- \
        python3 "$ROOT/bench.py" --no-cpu --no-extra ${a/--steps [0-9]*/--steps 3} --warmup 1 > "$OUT/pmc_${leg}_$c.log" 2>&1 \
        || { tail "$OUT/pmc_${leg}_$c.log"; exit 1; }
  done
  echo "leg $leg: $(python3 -c "import json; d=json.load(open('$OUT/bench_prof_$leg.json')); print(d['kernel_ms'], 'ms', d['value'], 'GB/s', d['config']['kernel'][:60])")"
done
python3 "$ROOT/scripts/collect_round5.py" "$OUT"
