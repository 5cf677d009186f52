set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03k
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_odometry.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -8 $OUT/pytest.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python bench_odometry.py --frames 300 > $OUT/odo300.json 2> $OUT/odo.err || { tail $OUT/odo.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/odo300.json'));print({k:d[k] for k in ('value','frames_per_s','setup_ms_per_frame','align_ms_per_frame','iterations_per_frame')})"
timeout -k 10 300 python bench_odometry.py --frames 1000 > $OUT/odo1000.json 2> $OUT/odo1000.err || { tail $OUT/odo1000.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/odo1000.json'));print({k:d[k] for k in ('value','frames_per_s','setup_ms_per_frame','align_ms_per_frame','iterations_per_frame','frame_error','drift')})"
