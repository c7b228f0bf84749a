# builds the training-GEMM checker / bench (CPU here; run on the GPU box) from the library sources:
#   rows_check     parity of launch_tgemm (rows / cols kernels) vs a CPU double reference
#   rows_bench     per-shape timing
# (r06: the route / split constants are compile-time constants of the sources, no -D overrides; a
# variant is a modified copy of the sources, as tools/build_variant.sh builds them)
set -e
D=$(cd "$(dirname "$0")" && pwd)
L="$D/../../rethink_acoustic_image_enhancement_amd/csrc"
SRC="$L/train_rows.hip $L/train_cols.hip $L/train.hip"
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17"
$H -o "$D/rows_check" "$D/rows_check.cpp" $SRC
$H -o "$D/rows_bench" "$D/rows_bench.cpp" $SRC
