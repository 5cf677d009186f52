set -o pipefail
mkdir -p gpurun_out/tl
GICP_LIB_VARIANT=tl GICP_STAMPS_DUMP=gpurun_out/tl/st timeout -k 10 200 python scripts/pass_diag.py 1000000 30 > gpurun_out/tl/diag.txt 2>&1 || exit 1
for k in 30 31 35 40 42 45 51 55; do echo "== dump $k"; python scripts/timeline.py gpurun_out/tl/st.$k 4 0; done > gpurun_out/tl/timeline.txt
# keep the first pass of the timed registration (and the next) for the launch-order analysis
for k in $(ls gpurun_out/tl/ | sed -n 's/^st\.\([0-9]*\)$/\1/p'); do [ $k = 30 ] || [ $k = 31 ] || rm -f gpurun_out/tl/st.$k; done
