#!/bin/bash
# Build an A/B variant of libambrycrc.so for tools/ab_cases.sh:
#   tools/ab_build.sh <kernels.hip | -> <name>   ->  build/ab/<name>/libambrycrc.so
# <kernels.hip> replaces csrc/crc32_kernels.hip ("-": keep the in-tree one). AB_FLAGS adds knob
# overrides (-DAMBRY_X=v, csrc/build_knobs.h). Every A/B build is marked a probe build
# (-DAMBRY_AB_PROBE_BUILD: ambrycrc_version() says so and ambrycrc_init refuses it unless
# AMBRYCRC_ALLOW_PROBE=1) and carries the split group kernel (variant 32,
# tools/probes/group_kernels.hip).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
src=$1; name=$2
tree=$(mktemp -d)
mkdir -p $tree/ambry_amd $tree/include
cp -r $ROOT/ambry_amd/csrc $tree/ambry_amd/
cp $ROOT/include/*.h $tree/include/
if [ "$src" != "-" ]; then cp $src $tree/ambry_amd/csrc/crc32_kernels.hip; fi
cp $ROOT/tools/probes/group_kernels.hip $tree/ambry_amd/csrc/
mkdir -p $ROOT/build/ab/$name
cd $tree/ambry_amd
g++ -O3 -std=c++17 -fPIC -Wall -c -o host_crc.o csrc/host_crc.cpp
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DAMBRY_AB_PROBE_BUILD -DAMBRY_AB_SPLIT_GROUP ${AB_FLAGS:-} \
  -shared -o $ROOT/build/ab/$name/libambrycrc.so host_crc.o \
  csrc/ambrycrc.cpp csrc/ambrycrc_multi.cpp csrc/ambrycrc_put.cpp csrc/crc32_kernels.hip csrc/message_kernels.hip \
  csrc/put_kernels.hip csrc/ambrycrc_msg_cpu.cpp csrc/group_kernels.hip -ldl
rm -rf $tree
echo "built build/ab/$name/libambrycrc.so"
