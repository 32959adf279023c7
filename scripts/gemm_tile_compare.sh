cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in bt64 bt128; do
  RD_LIB=libreacher_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gc_$v -o run -- python3 scripts/bench_student_lstm.py 16384 > gpurun_out/gc_$v.log 2>&1 || exit 1
done
