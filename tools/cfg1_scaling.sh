# cfg1 walk time against the batch size (a walk bound by its heaviest topics' chains stays flat as
# the batch shrinks; one bound by throughput shrinks with it), plus the census walk's per-wave
# timeline (tools/wave_times.py).  GPU box: bash tools/cfg1_scaling.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/cfg1_scaling; mkdir -p $O
A="--cfg 1 --no-cpu-baseline --no-e2e --nif= --no-subscribe --steps 100 --warmup 10"
for t in 100000 50000 25000 12500 6250; do
  (cd $R && timeout -k 10 240 python -u bench.py $A --topics $t > $O/t$t.json 2> $O/t$t.log) || exit 1
done
(cd $R && EMQXGM_WAVE_TIMES=$O/wt1.bin timeout -k 10 240 python -u bench.py $A --steps 5 > $O/census.json 2> $O/census.log) &&
python3 $R/tools/wave_times.py $O/wt1.bin > $O/wave_times.txt
