set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03d
timeout -k 10 300 python scripts/probes/full_output_profile.py > gpurun_out/r03d/prof.txt 2> gpurun_out/r03d/prof.err || { tail gpurun_out/r03d/prof.err; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_odometry.py -x -v --timeout 600 --timeout-method thread -k "2d or full_size_stream" > gpurun_out/r03d/pytest.log 2>&1; rc=$?; tail -12 gpurun_out/r03d/pytest.log; exit $rc
