set -o pipefail
mkdir -p gpurun_out/stamps
GICP_LIB_VARIANT=stamps timeout -k 10 200 python scripts/pass_diag.py 1000000 30 > gpurun_out/stamps/diag.txt 2> gpurun_out/stamps/stamps.txt || exit 1
