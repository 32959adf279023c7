# Per-shape GEMM timings of the LSTM step under different tile choices (diagnostic builds
# libreacher_big.so = the 32x32x2 128-tile kernel where it fits; the product = 16x16x4 64-tile everywhere).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in big product; do
  lib=libreacher_$v.so; [ $v = product ] && lib=libreacher.so
  RD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gc_$v -o run -- python3 scripts/bench_student_lstm.py 16384 > gpurun_out/gc_$v.log 2>&1 || exit 1
done
