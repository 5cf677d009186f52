set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tr}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o t --output-format csv -- python3 bench.py --no-cpu-baseline ${@:2} > $OUT/bench.json 2> $OUT/trace.err || { echo trace failed; tail $OUT/trace.err; exit 1; }
python3 scripts/trace_iters.py $OUT/trace 30 > $OUT/iterations.txt
cat $OUT/iterations.txt
