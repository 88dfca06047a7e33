#!/bin/bash
# Alternating A/B of prebuilt library variants (built in the container with
# scripts/ab_build.sh): ROUNDS passes over the libs, each one
# scripts/ab_kernels.py run (C3 compress and decode, median of REPS launches).
# Usage (GPU box): ROUNDS=3 REPS=20 bash scripts/ab_run.sh scripts/ab/lib_a.so scripts/ab/lib_b.so
set -u
ROUNDS=${ROUNDS:-3}; REPS=${REPS:-20}
for r in $(seq $ROUNDS); do
  for lib in "$@"; do
    timeout -k 10 120 python scripts/ab_kernels.py --lib $lib --reps $REPS 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
