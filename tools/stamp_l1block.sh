# Stamps build of libsad with only l1block.o rebuilt -DSAD_STAMPS=1 (the other
# objects from the normal build) -> abl/libsad_l1stamps.so; then time/stamp.
set -e
cd "$(dirname "$0")/.."
mkdir -p abl /tmp/l1st
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -munsafe-fp-atomics -DSAD_STAMPS=1 \
  -c synthetic-audio-detection_amd/csrc/l1block.hip -o /tmp/l1st/l1block.o
objs=$(ls build/csrc/*.o | grep -v l1block.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o abl/libsad_l1stamps.so $objs /tmp/l1st/l1block.o
