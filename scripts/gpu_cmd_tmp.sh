set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03m
mkdir -p $OUT
GICP_LIB_VARIANT=stamps timeout -k 10 300 python scripts/pass_diag.py 1000000 12 > $OUT/diag.txt 2> $OUT/stamps.txt || { tail $OUT/stamps.txt; exit 1; }
tail -14 $OUT/diag.txt
grep -E "all |slowest|median|mean cycles" $OUT/stamps.txt | head -60 | cut -c1-400
timeout -k 10 400 python scripts/twod_1m_vs_oracle.py > $OUT/twod_1m.json 2> $OUT/twod.err || { tail $OUT/twod.err; exit 1; }
cat $OUT/twod_1m.json
