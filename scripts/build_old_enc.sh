#!/bin/bash
# (development) loona_amd/libhpk_NAME.so = the current library with hpk_encode.hip taken from git REV,
# for encode A/B runs: scripts/build_old_enc.sh NAME REV
set -e
cd "$(dirname "$0")/../loona_amd/csrc"
NAME=$1; REV=${2:-HEAD}
T=/tmp/hpkenc_$NAME; mkdir -p $T
git show $REV:loona_amd/csrc/hpk_encode.hip > $T/hpk_encode.hip
make -s hpk_cpu.o hpk_hpack.o hpk_h2.o hpk_ctx.o hpk_decode.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I. -x hip --offload-arch=gfx950 -c -o $T/enc.o $T/hpk_encode.hip
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../libhpk_$NAME.so hpk_cpu.o hpk_hpack.o hpk_h2.o hpk_ctx.o hpk_decode.o $T/enc.o
echo built loona_amd/libhpk_$NAME.so
