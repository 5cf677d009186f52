#!/bin/bash
# bench.py (default workload, cold start) under environment variants, interleaved, one GPU call:
#   scripts/bench_variants.sh OUTDIR REPS "ENV1" "ENV2" ...      (use "X=0" for the default build)
#   BENCH_ARGS="--n 100000" selects another workload
set -o pipefail
OUT=gpurun_out/$1; REPS=$2; shift 2
mkdir -p $OUT
for r in $(seq 1 $REPS); do
  i=0
  for v in "$@"; do
    i=$((i+1))
    env $v timeout -k 10 200 python bench.py --no-cpu-baseline $BENCH_ARGS > $OUT/v${i}_r$r.json 2> $OUT/v${i}_r$r.err || { echo "variant $v failed"; tail $OUT/v${i}_r$r.err; exit 1; }
  done
done
python - "$OUT" "$REPS" "$@" <<'PY'
import sys, json
out, reps, vs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
for i, v in enumerate(vs, 1):
    for r in range(1, reps + 1):
        d = json.load(open(f"{out}/v{i}_r{r}.json"))
        p = d["passes"]
        print(f"{v:28s} r{r} {d['value']:8.1f} it/s  k_corr {d['roofline']['kernel_avg_ms']*1e3:6.1f} us  moving {p['moving_pass_us']:6.1f}"
              f"  converged {p['converged_pass_us']:5.1f}  warm {d['warm_start']['value']:8.1f}")
    print("   per-iteration:", " ".join(f"{x:.0f}" for x in p["k_corr_us_per_iteration"]))
PY
