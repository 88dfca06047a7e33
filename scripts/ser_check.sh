# table-walk decoder: its GPU tests, stamps and A/B, then SQ counters
T=${1:-s}
bash scripts/ser_run.sh $T && bash scripts/sq_ser.sh
