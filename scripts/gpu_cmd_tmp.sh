set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03l
mkdir -p $OUT
for r in 1 2; do
for v in "GICP_BUILD_SPLIT=1" "GICP_BUILD_SPLIT=4"; do
env $v timeout -k 10 300 python bench_odometry.py --frames 500 > $OUT/odo_${v}_$r.json 2> $OUT/odo.err || { tail $OUT/odo.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/odo_${v}_$r.json'));print('$v', {k:round(d[k],3) for k in ('value','frames_per_s','setup_ms_per_frame','align_ms_per_frame')})"
done
done
