#!/bin/bash
# Build an A/B variant of liblzo_mi355x.so from the in-tree objects, with the
# encoder and/or decoder kernels taken from other source files and flags:
#   scripts/ab_build.sh NAME [enc=FILE] [dec=FILE] [encflags="-D..."] [decflags="-D..."]
# -> scripts/ab/lib_NAME.so (run it with: python scripts/ab_kernels.py --lib ...)
set -eu
name=$1; shift
C=pomegranate_amd/csrc
enc=$C/lzo1x_encode_fast.hip; dec=$C/lzo1x_decode_fast.hip; encflags=""; decflags=""
for kv in "$@"; do declare -- "$kv"; done
mkdir -p scripts/ab
HIPCC="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$C -Iinclude"
$HIPCC $encflags -c $enc -o /tmp/ab_enc_$name.o
$HIPCC $decflags -c $dec -o /tmp/ab_dec_$name.o
objs=$(ls $C/*.o | grep -v -e lzo1x_encode_fast.o -e lzo1x_decode_fast.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o scripts/ab/lib_$name.so /tmp/ab_enc_$name.o /tmp/ab_dec_$name.o $objs -Wl,-Bsymbolic -lpthread
echo "built scripts/ab/lib_$name.so"
