# builds the training-GEMM checkers / benches (CPU here; run on the GPU box) from the library sources:
#   rows_check     parity of launch_tgemm (rows / cols kernels) vs a CPU double reference
#   rows_check_b   the same through the generic kernel only (-DKDLAE_TRAIN_ROWS=0 -DKDLAE_TRAIN_COLS=0)
#   rows_bench*    per-shape timing, one binary per -D variant listed in $VARIANTS ("name:-DX=1 -DY=2")
set -e
D=$(cd "$(dirname "$0")" && pwd)
L="$D/../../rethink_acoustic_image_enhancement_amd/csrc"
SRC="$L/train_rows.hip $L/train_cols.hip $L/train.hip"
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17"
$H -o "$D/rows_check" "$D/rows_check.cpp" $SRC
$H -DKDLAE_TRAIN_ROWS=0 -DKDLAE_TRAIN_COLS=0 -o "$D/rows_check_b" "$D/rows_check.cpp" $SRC
$H -o "$D/rows_bench" "$D/rows_bench.cpp" $SRC
$H -DKDLAE_TRAIN_ROWS=0 -DKDLAE_TRAIN_COLS=0 -o "$D/rows_bench_generic" "$D/rows_bench.cpp" $SRC
for v in $VARIANTS; do
  n=${v%%:*}; f=${v#*:}
  $H ${f//,/ } -o "$D/rows_bench_$n" "$D/rows_bench.cpp" $SRC &
done
wait
