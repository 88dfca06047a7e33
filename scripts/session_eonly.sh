set -u
python -c "import __graft_entry__ as g; g.build()" > /dev/null 2>&1 || exit 1
C=pomegranate_amd/csrc
for v in "rec:-DPOM_SLOTS=16 -DPOM_EXPERIMENT_RECORD" "replay:-DPOM_SLOTS=16 -DPOM_EXPERIMENT_REPLAY"; do
  n=${v%%:*}; f=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$C -Iinclude $f -c $C/lzo1x_decode_fast.hip -o /tmp/x_$n.o || exit 1
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o /tmp/lib_$n.so $C/lzo1x_kernels.o $C/lzo1x_encode_fast.o /tmp/x_$n.o $C/lzo_host.o $C/itb_codec.o $C/column_codec.o $C/xnet_frame.o -Wl,-Bsymbolic -lpthread || exit 1
done
timeout -k 10 120 python scripts/eonly.py /tmp/lib_rec.so /tmp/lib_replay.so 2>&1 | grep -v amdgpu.ids
