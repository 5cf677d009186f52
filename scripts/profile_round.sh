#!/bin/bash
# Round profile of the DRIVER's bench command (bench.py --gpus 1 --steps $STEPS --warmup $WARMUP, default
# 20 / 5: 205 k_corr launches): kernel-trace stats, per-iteration trace, PMC passes (instruction mix, waits)
# and the HBM-side traffic summary keyed by (workload, steps, warmup), mean and per pass; then the bench
# line of the same command (which reads the traffic just measured).
# Usage: scripts/profile_round.sh OUTNAME PROFILEDIR   (e.g. r04_prof profiles/r04)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-prof}
PD=${2:-profiles/r05}
STEPS=${STEPS:-20}
WARMUP=${WARMUP:-5}
CMD="bench.py --gpus 1 --steps $STEPS --warmup $WARMUP"
mkdir -p $OUT $PD
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o t --output-format csv -- python3 $CMD > $OUT/bench_under_rocprof.json 2> $OUT/trace.err || { echo trace failed; exit 1; }
python3 scripts/trace_iters.py $OUT/trace $STEPS > $OUT/iterations.txt
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" \
           "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d $OUT/pmc/p$i -o pmc --output-format csv -- python3 $CMD > $OUT/pmc_p$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
python3 scripts/pmc_summary.py $OUT/pmc > $OUT/pmc_summary.txt
python3 scripts/pmc_traffic.py $OUT/pmc $OUT/pmc_traffic.json k_corr 3d_room_1000k_1000k_k20 $WARMUP $STEPS
cp $OUT/pmc_traffic.json $PD/pmc_traffic.json   # (on the box: read by the bench line below; gpurun_out/ is what comes back)
timeout -k 10 300 python3 $CMD > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail $OUT/bench.err; exit 1; }
echo done
