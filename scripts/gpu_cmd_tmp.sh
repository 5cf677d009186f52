set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03j
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] || { grep -E "FAIL|Error" $OUT/pytest_gpu.log | head; exit 1; }
timeout -k 10 300 python scripts/probes/build_diag.py > $OUT/diag.txt 2> $OUT/diag.err || { tail $OUT/diag.err; exit 1; }
cat $OUT/diag.txt
GICP_BUILD_SPLIT=1 timeout -k 10 300 python scripts/probes/build_diag.py > $OUT/diag1.txt 2> $OUT/diag1.err || { tail $OUT/diag1.err; exit 1; }
cat $OUT/diag1.txt
timeout -k 10 300 python bench_odometry.py --frames 300 > $OUT/odo300.json 2> $OUT/odo.err || { tail $OUT/odo.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/odo300.json'));print({k:d[k] for k in ('value','frames_per_s','setup_ms_per_frame','align_ms_per_frame','iterations_per_frame')})"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o t --output-format csv -- python3 bench_odometry.py --frames 100 > $OUT/odo_prof.json 2> $OUT/odo_prof.err || { tail $OUT/odo_prof.err; exit 1; }
grep -E "k_corr|k_knn|k_graph|k_solve|build_tiles" $OUT/trace/t_kernel_stats.csv | cut -c1-130
