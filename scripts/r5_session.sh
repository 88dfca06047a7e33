#!/bin/bash
# Round-5 GPU session: build, parity tests, A/B of the C3 kernels against
# variant libraries (scripts/ab/lib_NAME.so from scripts/ab_build.sh, listed in
# AB), smoke, bench.  Each GPU step has its own time limit; a crash or timeout
# ends the session.
set -u
OUT=${OUT:-gpurun_out/r5}
mkdir -p "$OUT"
step() {
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n ${TAILN:-12} "$OUT/$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping: $name $rc"; exit $rc; fi
    return 0
}
python -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1 || { echo build failed; tail "$OUT/build.log"; exit 1; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_gpu 420 python -u -m pytest tests -v -s -m gpu ${PYTEST_X:--x} --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
fi
# (A/B libraries: built beforehand with scripts/ab_build.sh, they travel in-tree)
for r in 1 2 3; do
  for v in ${AB:-}; do
    step ab_${v}_$r 120 python scripts/ab_kernels.py --lib scripts/ab/lib_$v.so --reps 10
  done
  [ -n "${AB:-}" ] && step ab_cur_$r 120 python scripts/ab_kernels.py --reps 10
done
[ -n "${EXTRA:-}" ] && step extra 300 $EXTRA
[ "${SKIP_SMOKE:-0}" != 1 ] && step smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
[ "${SKIP_BENCH:-0}" != 1 ] && step bench 420 python bench.py ${BENCH_ARGS:-}
echo session done
