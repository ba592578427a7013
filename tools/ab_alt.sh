# Alternating A/B of the in-tree engine against ablib/lib_<V>.so, each run kept: cfg C, N rounds.
# GPU box: bash tools/ab_alt.sh TAG V C N
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; V=$2; C=$3; N=${4:-3}; mkdir -p $O
A="--no-cpu-baseline --no-e2e --nif= --no-subscribe --steps 100 --warmup 10"
cp $R/emqx_amd/libemqx_gpumatch.so $O/base.so || exit 1
for i in $(seq $N); do
  for v in base $V; do
    cp $([ $v = base ] && echo $O/base.so || echo $R/ablib/lib_$v.so) $R/emqx_amd/libemqx_gpumatch.so || exit 1
    (cd $R && timeout -k 10 300 python -u bench.py --cfg $C $A > $O/${v}_$i.json 2> $O/${v}_$i.log) || { cp $O/base.so $R/emqx_amd/libemqx_gpumatch.so; exit 1; }
  done
done
cp $O/base.so $R/emqx_amd/libemqx_gpumatch.so; rm -f $O/base.so
for f in $O/*_[0-9]*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$(basename $f)', round(d['value']/1e9,3), d['ms_per_step'], d['roofline']['kernels_ms']['k_walk'])"; done
