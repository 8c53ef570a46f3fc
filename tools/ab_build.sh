#!/bin/bash
# Build libambrycrc.so with another crc32_kernels.hip for tools/ab_cases.sh:
#   tools/ab_build.sh <kernels.hip> <name>   ->  build/ab/<name>/libambrycrc.so
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
src=$1; name=$2
tree=$(mktemp -d)
mkdir -p $tree/ambry_amd $tree/include
cp -r $ROOT/ambry_amd/csrc $tree/ambry_amd/
cp $ROOT/include/*.h $tree/include/
cp $src $tree/ambry_amd/csrc/crc32_kernels.hip
mkdir -p $ROOT/build/ab/$name
cd $tree/ambry_amd
g++ -O3 -std=c++17 -fPIC -Wall -c -o host_crc.o csrc/host_crc.cpp
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 ${AB_FLAGS:-} -shared -o $ROOT/build/ab/$name/libambrycrc.so host_crc.o \
  csrc/ambrycrc.cpp csrc/ambrycrc_multi.cpp csrc/ambrycrc_put.cpp csrc/crc32_kernels.hip csrc/message_kernels.hip \
  csrc/put_kernels.hip csrc/ambrycrc_msg_cpu.cpp csrc/group_kernels.hip -ldl
rm -rf $tree
echo "built build/ab/$name/libambrycrc.so"
