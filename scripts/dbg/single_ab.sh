# single-call compress latency: the in-tree library against scripts/ab/lib_ehead.so
set -u
timeout -k 10 120 python scripts/ab_single.py --op compress --calls 30 --lib scripts/ab/lib_ehead.so || exit 1
timeout -k 10 120 python scripts/ab_single.py --op compress --calls 30 || exit 1
