set -u
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 120 python scripts/diag_decode.py > gpurun_out/diag.log 2>&1 || { cat gpurun_out/diag.log; exit 1; }
cat gpurun_out/diag.log
bash scripts/profile_sq.sh cur || exit 1
bash scripts/profile_decode.sh r01b || exit 1
