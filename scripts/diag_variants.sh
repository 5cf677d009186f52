#!/bin/bash
# pass_diag.py under environment variants, one GPU call: scripts/diag_variants.sh OUTDIR "ENV1" "ENV2" ...
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
i=0
for v in "$@"; do
  i=$((i+1))
  echo "== $v" > $OUT/v$i.txt
  env $v timeout -k 10 200 python scripts/pass_diag.py >> $OUT/v$i.txt 2>&1 || { echo "variant $v failed"; tail $OUT/v$i.txt; exit 1; }
done
python - "$OUT" $i <<'PY'
import sys, re
out, n = sys.argv[1], int(sys.argv[2])
for k in range(1, n + 1):
    L = open(f"{out}/v{k}.txt").read().splitlines()
    t = [float(re.search(r"pass +\d+ +(\d+) us", l).group(1)) for l in L if l.startswith("pass")]
    print(L[0], "sum", sum(t), "first10", sum(t[:10]), "mid10", sum(t[10:20]), "last10", sum(t[20:]))
PY
