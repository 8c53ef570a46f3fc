#!/bin/bash
# Build libambrycrc.so from the sources of a git revision (the A side of an A/B against the working
# tree), marked a probe build as tools/ab_build.sh marks its builds:
#   tools/ab_build_rev.sh <rev> <name>   ->  abtmp/<name>/libambrycrc.so
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rev=$1; name=$2
tree=$(mktemp -d)
git -C $ROOT archive $rev ambry_amd/csrc include | tar -x -C $tree
mkdir -p $ROOT/abtmp/$name
cd $tree/ambry_amd
g++ -O3 -std=c++17 -fPIC -Wall -c -o host_crc.o csrc/host_crc.cpp
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DAMBRY_AB_PROBE_BUILD ${AB_FLAGS:-} \
  -shared -o $ROOT/abtmp/$name/libambrycrc.so host_crc.o \
  csrc/ambrycrc.cpp csrc/ambrycrc_multi.cpp csrc/ambrycrc_put.cpp csrc/crc32_kernels.hip csrc/message_kernels.hip \
  csrc/put_kernels.hip csrc/ambrycrc_msg_cpu.cpp -ldl
rm -rf $tree
echo "built abtmp/$name/libambrycrc.so"
