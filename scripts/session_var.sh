set -u
mkdir -p gpurun_out
timeout -k 10 300 bash scripts/variants.sh "$@" > gpurun_out/variants.log 2>&1; rc=$?
cat gpurun_out/variants.log | grep -v amdgpu.ids; exit $rc
