# r06: k_exact with LDS-staged names (A/B against ablib/lib_xglob.so, the global-read probe) and
# the grouped scatter at 8 waves per SIMD against the direct stores on cfg3 (profiles/r06/exact/)
set -o pipefail
cd /root/repo
O=gpurun_out/${TAG:-xab1}; mkdir -p $O
B="--no-cpu-baseline --no-e2e --nif= --no-subscribe"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
bash tools/job.sh ${TAG:-xab1} ab=2:0,4:0,3:0/xglob || exit 1
cat $O/ab_summary.txt
for i in 1 2; do
  for v in grp direct; do
    if [ $v = direct ]; then export EMQXGM_SCATTER_DIRECT=1; else unset EMQXGM_SCATTER_DIRECT; fi
    timeout -k 10 300 python -u bench.py --cfg 3 $B > $O/s_c3_${v}_$i.json 2> $O/s_c3_${v}_$i.log || exit 1
    echo "$v c3 $i $(python3 -c "import json;d=json.load(open('$O/s_c3_${v}_$i.json'));print(d['value'],d['ms_per_step'])")"
  done
done
