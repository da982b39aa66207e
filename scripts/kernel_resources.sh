# Per-kernel VGPR/AGPR/scratch of the gfx950 code object inside libpcseg.so
set -e
SO=${1:-/root/repo/3d-semantic-segmentation-benchmark_amd/pcseg/libpcseg.so}
TMP=$(mktemp -d)
cd $TMP
/opt/rocm/lib/llvm/bin/clang-offload-bundler --list --type=o --input=$SO > targets.txt 2>/dev/null || true
T=$(grep gfx950 targets.txt | head -1)
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$SO --targets=$T --output=co.o
/opt/rocm/lib/llvm/bin/llvm-readelf --notes co.o | grep -E "\.name:|\.vgpr_count|\.agpr_count|\.private_segment_fixed_size|\.group_segment_fixed_size" | paste - - - - - | sed 's/  */ /g'
rm -rf $TMP
