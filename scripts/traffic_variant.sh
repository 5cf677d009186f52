#!/bin/bash
# HBM-side traffic per k_corr pass of the driver's command for one library variant (the two PMC passes of
# scripts/profile_round.sh that pmc_traffic.py reads), e.g. to compare a layout change's bytes:
#   scripts/traffic_variant.sh OUTNAME VARIANT      (VARIANT "" = the default build)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:?out}
V=${2:-}
CMD="bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
mkdir -p $OUT
i=2
for set in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  GICP_LIB_VARIANT=$V timeout -k 10 300 rocprofv3 --pmc $set -d $OUT/pmc/p$i -o pmc --output-format csv -- python3 $CMD > $OUT/pmc_p$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
python3 scripts/pmc_traffic.py $OUT/pmc $OUT/pmc_traffic.json k_corr 3d_room_1000k_1000k_k20 5 20
