#!/bin/bash
# r03: the walk's fixed cost -- walk / pass time against batch size (cfg1, cfg3)
set -o pipefail
O=gpurun_out/${1:-r03_floor}; mkdir -p $O
for c in "1 1024" "1 8192" "1 32768" "3 1024" "3 16384"; do
  set -- $c
  timeout -k 10 240 python -u bench.py --cfg $1 --topics $2 --steps 50 --warmup 5 --no-cpu-baseline --no-e2e --windows "" > $O/b_$1_$2.json 2> $O/b_$1_$2.err || exit 1
  python - $O/b_$1_$2.json <<'PY' >> $O/summary.txt
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
r=d['roofline']; c=d['config']
print(c['workload'][:5], c['global_batch'], 'step', d['ms_per_step'], 'kern', r.get('kernels_ms'), 'onepass', c.get('one_pass_at_a_time',{}).get('ms_per_step'))
PY
done
cat $O/summary.txt
