#!/bin/bash
# round 5: walkers-first hot slots -- schedule invariance test, A/B of the slot count on the driver command,
# per-pass tail breakdown with and without
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05h
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_extensions.py -k walkers > $OUT/test.log 2>&1 || { echo test failed; tail -30 $OUT/test.log; exit 1; }
tail -2 $OUT/test.log
for r in 1 2; do
  for h in 0 64 128 256; do
    GICP_HOT_SLOTS=$h timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/b_${h}_$r.json 2> $OUT/b_${h}_$r.err || { echo bench $h failed; tail $OUT/b_${h}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b_${h}_$r.json'));print('hot $h rep $r',round(d['value'],1),'it/s',round(d['ms_per_step']*1e3,1),'us/step')"
  done
done
for h in 0 128; do
  GICP_HOT_SLOTS=$h GICP_LIB_VARIANT=tail timeout -k 10 300 python3 scripts/tail_run.py --steps 20 --reps 2 > $OUT/tail_1m_$h.txt 2> $OUT/tail_$h.err || { echo tail failed; tail $OUT/tail_$h.err; exit 1; }
done
python3 - <<'PY'
import re
for h in (0, 128):
    L = open(f"gpurun_out/r05h/tail_1m_{h}.txt").read().splitlines()
    ev = [float(l.split()[1]) for l in L if re.match(r"^\s+\d+\s+\d", l)][:20]
    print(h, "event per pass", " ".join(f"{x:.0f}" for x in ev), "sum", round(sum(ev)))
PY
