#!/bin/bash
# Build a variant of the product library with extra preprocessor flags (experiments only):
#   scripts/build_var.sh NAME "-DHPK_SPREAD=0 ..."  ->  loona_amd/libhpk_NAME.so (select with HPK_LIB)
set -e
cd "$(dirname "$0")/../loona_amd/csrc"
NAME=$1; FLAGS=$2
T=/tmp/hpkvar_$NAME; mkdir -p $T
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function"
$H $FLAGS -x hip --offload-arch=gfx950 -c -o $T/dec.o hpk_decode.hip
$H $FLAGS -x hip --offload-arch=gfx950 -c -o $T/ctx.o hpk_ctx.hip
$H $FLAGS -x hip --offload-arch=gfx950 -c -o $T/enc.o hpk_encode.hip
make -s hpk_cpu.o hpk_hpack.o hpk_h2.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../libhpk_$NAME.so hpk_cpu.o hpk_hpack.o hpk_h2.o $T/ctx.o $T/dec.o $T/enc.o
echo built loona_amd/libhpk_$NAME.so
