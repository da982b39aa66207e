# Build an A/B variant of libpcseg.so: the working tree's csrc with some files taken from a git
# ref, into pcseg/libpcseg_<name>.so (loaded via PCS_LIB=... by the A/B scripts only).
# usage: scripts/build_ab.sh <name> <git-ref> <csrc file> [<csrc file> ...]
#        (git-ref "-": no files replaced; extra hipcc flags in PCS_AB_FLAGS, e.g. -DPCS_GR_OCC=3)
set -eu
name=$1; ref=$2; shift 2
repo=$(cd "$(dirname "$0")/.." && pwd)
pkg=3d-semantic-segmentation-benchmark_amd
tmp=/tmp/pcs_ab_$name
rm -rf "$tmp"; mkdir -p "$tmp/x" "$tmp/include"
cp -r "$repo/$pkg/csrc" "$tmp/x/csrc"; rm -rf "$tmp/x/csrc/build"
cp "$repo/include/"*.h "$tmp/include/"
[ "$ref" = "-" ] || for f in "$@"; do git -C "$repo" show "$ref:$pkg/csrc/$f" > "$tmp/x/csrc/$f"; done
flags="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-variable"
make -s -C "$tmp/x/csrc" -j8 OUT="$repo/$pkg/pcseg/libpcseg_$name.so" BUILD="$tmp/build" CXXFLAGS="$flags ${PCS_AB_FLAGS:-}"
echo "built $pkg/pcseg/libpcseg_$name.so"
