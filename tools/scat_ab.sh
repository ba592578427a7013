set -o pipefail
cd /root/repo
O=gpurun_out/${TAG:-scat1}; mkdir -p $O
B="--no-cpu-baseline --no-e2e --nif= --no-subscribe"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
for i in 1 2; do
  for v in grp direct; do
    if [ $v = direct ]; then export EMQXGM_SCATTER_DIRECT=1; else unset EMQXGM_SCATTER_DIRECT; fi
    for c in ${CFGS:-2 3}; do
      timeout -k 10 300 python -u bench.py --cfg $c $B > $O/b_c${c}_${v}_$i.json 2> $O/b_c${c}_${v}_$i.log || exit 1
      echo "$v c$c $i $(python3 -c "import json,sys;d=json.load(open('$O/b_c${c}_${v}_$i.json'));print(d['value'],d['ms_per_step'])")"
    done
  done
done
unset EMQXGM_SCATTER_DIRECT
cd /tmp && export TMPDIR=/tmp
true
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /root/repo/$O/onepass_c3 -o run --output-format csv -- python3 /root/repo/bench.py --cfg 3 --no-pipeline $B --settle-s 0 --steps 20 --warmup 3 > /root/repo/$O/onepass_c3.json 2>&1 || exit 1
echo done
