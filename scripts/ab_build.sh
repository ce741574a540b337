#!/bin/bash
# scripts/ab_build.sh NAME "-DFLAG=V ..." [kernel source] -- a variant of
# libmijpeg.so with mij_kernels.hip (or another version of it, e.g. from git
# show) compiled under extra defines, as ab/libmijpeg_NAME.so (for
# scripts/ab.sh; ab/ is git-ignored but travels to the GPU box).
set -e
cd "$(dirname "$0")/../jpeg-encoder-decoder_amd"
make -s csrc/mij_api.o csrc/mij_stream.o csrc/mij_detect.o csrc/mij_decode.o
mkdir -p ../ab
H="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../include -Icsrc -w"
SRC=$(realpath "${3:-csrc/mij_kernels.hip}")
/opt/rocm/bin/hipcc $H -Icsrc $2 -c "$SRC" -o /tmp/ab_k_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../ab/libmijpeg_$1.so /tmp/ab_k_$1.o \
    csrc/mij_api.o csrc/mij_stream.o csrc/mij_detect.o csrc/mij_decode.o
echo "ab/libmijpeg_$1.so"
