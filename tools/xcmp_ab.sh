# r06: route-key confirmation a dword at a time (A/B against ablib/lib_bytecmp.so, the byte loop)
set -o pipefail
cd /root/repo
O=gpurun_out/xcmp; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
bash tools/job.sh xcmp ab=2:0,4:0/bytecmp stall=2:k_exact || exit 1
cat $O/ab_summary.txt
