#!/bin/bash
# The round's side lines (after scripts/profile_round.sh): C2, the 2-D segment scenes, the C5 stream
# (staged and synchronous), per-pass instruction counts of the default bench.  Output: gpurun_out/$1/
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-extras}
mkdir -p $OUT
timeout -k 10 300 python bench.py --n 100000 > $OUT/bench_c2.json 2> $OUT/c2.err || { echo c2 failed; exit 1; }
timeout -k 10 300 python bench.py --dim 2 --n 1000000 --no-cpu-baseline > $OUT/bench_2d_1m.json 2> $OUT/2d1m.err || { echo 2d 1m failed; exit 1; }
timeout -k 10 300 python bench.py --dim 2 --n 100000 --no-cpu-baseline > $OUT/bench_2d_100k.json 2> $OUT/2d100k.err || { echo 2d 100k failed; exit 1; }
timeout -k 10 400 python bench_odometry.py > $OUT/bench_odometry_staged.json 2> $OUT/odo.err || { echo odometry failed; exit 1; }
timeout -k 10 400 python bench_odometry.py --copy > $OUT/bench_odometry_staged_copy.json 2> $OUT/odo_copy.err || { echo odometry copy failed; exit 1; }
timeout -k 10 400 python bench_odometry.py --sync > $OUT/bench_odometry_sync.json 2> $OUT/odo_sync.err || { echo odometry sync failed; exit 1; }
mkdir -p $OUT/pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES -d $OUT/pmc/p1 -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/pmc/p1.log 2>&1 || { echo pmc failed; exit 1; }
python3 scripts/pmc_passes.py $OUT/pmc/p1 > $OUT/pmc_passes.txt
for f in bench_c2 bench_2d_1m bench_2d_100k; do python3 -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',round(d['value'],1),d['unit'],'k_corr',round(d['roofline']['kernel_avg_ms']*1e3,1),'us')"; done
cat $OUT/bench_odometry_staged.json | head -c 600; echo
timeout -k 10 300 python scripts/full_output_cost.py > $OUT/full_output_cost.json 2> $OUT/foc.err || { echo full_output_cost failed; tail $OUT/foc.err; exit 1; }
cat $OUT/full_output_cost.json
timeout -k 10 300 python bench_small.py > $OUT/bench_c1.json 2> $OUT/c1.err || { echo c1 failed; exit 1; }
timeout -k 10 300 python3 bench.py --shard-sim 8 --no-cpu-baseline > $OUT/bench_shard_sim8.json 2> $OUT/sim8.err || { echo sim8 failed; exit 1; }
timeout -k 10 300 python3 bench.py --gpus 2 --share-gpu --no-cpu-baseline --steps 20 > $OUT/share2.log 2> $OUT/share2.err || { echo share failed; exit 1; }
tail -1 $OUT/share2.log > $OUT/bench_share2_peer.json
timeout -k 10 300 python3 bench.py --gpus 2 --share-gpu --no-cpu-baseline --n 20000 --steps 100 > $OUT/share2s.log 2> $OUT/share2s.err || { echo share small failed; exit 1; }
tail -1 $OUT/share2s.log > $OUT/bench_share2_peer_20k.json
timeout -k 10 300 python3 bench.py --shard-sim 2 --no-cpu-baseline --n 20000 --steps 100 > $OUT/bench_shard_sim2_20k.json 2> $OUT/sim2s.err || { echo sim2 small failed; exit 1; }
