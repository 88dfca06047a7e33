# Encoder dictionary traffic with and without the written-slot bitmap
# (VERDICT r5 item 2): L2 hits/misses, EA read requests, write requests,
# FETCH_SIZE and WRITE_SIZE and the SQ instruction counts per block, one
# rocprofv3 --pmc pass per counter set, builds scripts/ab/lib_e_occ0.so and
# lib_e_base.so (scripts/ab_build.sh).  GPU box: bash scripts/dbg/enc_occ_pmc.sh
set -eu
P1="TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
P2="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_WRITE_sum"
PMC="$P1" bash scripts/sq_changes.sh occ_l2 e_occ0 e_base
PMC="$P2" bash scripts/sq_changes.sh occ_ea e_occ0 e_base
PMC="FETCH_SIZE" bash scripts/sq_changes.sh occ_fetch e_occ0 e_base
PMC="WRITE_SIZE" bash scripts/sq_changes.sh occ_write e_occ0 e_base
bash scripts/sq_changes.sh occ_sq e_occ0 e_base
