# single-call compress latency of scripts/ab/lib_NAME.so builds, alternating,
# three rounds: bash scripts/dbg/single_ab.sh NAME...
set -u
for r in 1 2 3; do
  for v in "$@"; do
    echo "== $v $r"
    timeout -k 10 120 python scripts/ab_single.py --op compress --calls 40 --lib scripts/ab/lib_$v.so 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
