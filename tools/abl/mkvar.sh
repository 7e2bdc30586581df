#!/bin/bash
# development: a libifd variant that differs from the in-tree build only in conv_x3.o
# usage: tools/abl/mkvar.sh NAME "-DX3_EPI=1 ..." [other sources rebuilt with the same defines, e.g. "unet conv"]
#        -> tools/abl/libifd_NAME.so
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
P=$R/face-inpainting-diffusion-models_amd
make -s -C $P -j8 >/dev/null
T=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -mllvm -structurizecfg-skip-uniform-regions \
  -fno-slp-vectorize $2 -c $P/csrc/conv_x3.hip -o $T/conv_x3.o
for f in $3; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -mllvm -structurizecfg-skip-uniform-regions \
    $2 -c $P/csrc/$f.hip -o $T/$f.o
done
objs="$(for o in $P/build/*.o; do b=$(basename $o .o); [ -e $T/$b.o ] || echo $o; done) $T/*.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/tools/abl/libifd_$1.so $objs
rm -rf $T
echo "built tools/abl/libifd_$1.so ($2)"
