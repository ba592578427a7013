# grouped k_scatter: PMC traffic and stall counters on cfg2, and a cfg1 A/B against the direct
# stores (r06, profiles/r06/scatter/)
set -o pipefail
cd /root/repo
bash tools/job.sh scat3 stall=2:k_scatter_grp prof=2 || exit 1
O=gpurun_out/scat3
B="--no-cpu-baseline --no-e2e --nif= --no-subscribe"
for i in 1 2; do
  for v in grp direct; do
    if [ $v = direct ]; then export EMQXGM_SCATTER_DIRECT=1; else unset EMQXGM_SCATTER_DIRECT; fi
    for c in 1 2; do
      timeout -k 10 300 python -u bench.py --cfg $c $B > $O/b_c${c}_${v}_$i.json 2> $O/b_c${c}_${v}_$i.log || exit 1
      echo "$v c$c $i $(python3 -c "import json;d=json.load(open('$O/b_c${c}_${v}_$i.json'));print(d['value'],d['ms_per_step'],d['kernels_ms'])")"
    done
  done
done
