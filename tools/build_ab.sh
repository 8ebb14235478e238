#!/bin/bash
# Build otto-recommender_amd/libottohip_ab.so (the B side of tools/gpu_ab.sh) from the in-tree sources with extra
# compiler flags, e.g. tools/build_ab.sh -DOH_EMIT_NOCHECK; or from a git revision: tools/build_ab.sh --rev <rev>
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/otto-recommender_amd/csrc
EXTRA=""
if [ "$1" = "--rev" ]; then
  W=$(mktemp -d); git -C "$ROOT" archive "$2" otto-recommender_amd/csrc include | tar -x -C "$W"; SRC=$W/otto-recommender_amd/csrc; shift 2
fi
EXTRA="$*"
OBJ=$(mktemp -d)
for f in abi prims knn shard merge ingest retrieve candidates popularity; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$SRC/../../include" -Wno-unused-function \
    -Wno-unused-value -Wno-unused-result -munsafe-fp-atomics $([ $f = knn ] && echo -fno-honor-nans) $EXTRA -c -o "$OBJ/$f.o" "$SRC/$f.hip" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/otto-recommender_amd/libottohip_ab.so" "$OBJ"/*.o
rm -rf "$OBJ"
echo "built libottohip_ab.so ($EXTRA)"
