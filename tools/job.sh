#!/bin/bash
# The one GPU-box job runner (replaces r01-r03's one-off lease scripts).  Runs its steps in
# order, each under its own time limit, and stops at the first failure.  Output under
# gpurun_out/TAG/.
#
#   tools/job.sh TAG STEP [STEP ...]
#
# steps:
#   tests[=PYTEST_ARGS]     python -m pytest tests -m gpu (default: the whole GPU suite); ARGS:
#                           commas for spaces
#   smoke                   __graft_entry__.smoke()
#   bench=CFG[:TOPICS[:ARGS]]  bench.py --cfg CFG (default bench line, or --topics TOPICS);
#                           ARGS: extra bench arguments, commas for spaces
#   onepass=CFG             rocprofv3 --kernel-trace --stats over bench.py --no-pipeline (the
#                           roofline's kernel time: one pass at a time)
#   prof=CFG[:ARGS]         rocprofv3 kernel stats + the PMC passes (one counter group per
#                           run: FETCH_SIZE; WRITE_SIZE + L2 hit/miss; TCP->TCC requests), then
#                           tools/pmc_summary.py; ARGS: extra bench arguments, commas for spaces
#                           (the output directories then carry them in their names)
#   sq=CFG[:TOPICS]         PMC issue counters of k_walk (SQ_* groups)
#   ab=SPECS/VARIANTS       A/B of engine builds ablib/lib_<V>.so (tools/ab_build.sh) against
#                           the in-tree one, base first and last; SPECS "cfg:topics,..." (0 =
#                           default topics), VARIANTS "v1,v2"
#   load=CFG[:FILTERS]      the concurrent publish entry's load (bench.py --only-nif)
#   latency                 tools/latency_probe.hip (built on the box): the dependent-step floor
#   winlat[=ARGS]           tools/window_latency.py (one window at a time); ARGS commas (r04:
#                           HSA_ENABLE_SDMA=0, blit-kernel copies, was slower: profiles/r04/latency)
#   wintrace[=ARGS]         rocprofv3 kernel + memory-copy + HIP runtime traces of
#                           tools/window_latency.py (the timeline of one window at a time)
#   dist[=filters|both]     bench.py's N=2 path with two ranks sharing this box's one GPU over
#                           gloo (RCCL refuses two ranks on one device): the control flow at full
#                           size, not a timing; "filters" makes the filter-sharded layout the
#                           headline
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:?usage: tools/job.sh TAG STEP...}
shift
O=$R/gpurun_out/$TAG
mkdir -p $O
KRE="k_walk|k_tok|k_exact|k_scatter|k_verify|k_scan"
NOCPU="--no-cpu-baseline --no-e2e --nif="
PROF="$NOCPU --settle-s 0 --no-subscribe"  # profiled runs: every launch is profiled, so no settle phase

step_tests() {
  local args=${1:-tests,-m,gpu}
  args=${args//,/ }
  (cd $R && timeout -k 10 1000 python -u -m pytest $args -x -v --timeout 300 --timeout-method thread) \
    > $O/pytest.log 2>&1
  local rc=$?
  tail -3 $O/pytest.log
  return $rc
}

step_smoke() {
  (cd $R && timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()') > $O/smoke.log 2>&1
}

step_bench() {
  local cfg=${1%%:*} rest= topics= extra=
  [ "$1" != "$cfg" ] && rest=${1#*:}
  topics=${rest%%:*}
  [ "$rest" != "$topics" ] && extra=${rest#*:}
  local T=""; [ -n "$topics" ] && [ "$topics" != 0 ] && T="--topics $topics"
  local tag=${extra//[^a-zA-Z0-9=]/_}
  local name=bench_c${cfg}_${topics:-0}${tag:+_$tag}
  (cd $R && timeout -k 10 900 python -u bench.py --cfg $cfg $T ${extra//,/ }) > $O/$name.json 2> $O/$name.log
}

step_onepass() {
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/onepass_c$1 -o run --output-format csv \
    -- python3 $R/bench.py --cfg $1 --no-pipeline $PROF --steps 20 --warmup 3 \
    > $O/onepass_c$1.json 2> $O/onepass_c$1.log
}

step_prof() {
  local c=${1%%:*} extra= steps=5
  [ "$1" != "$c" ] && extra=${1#*:}
  local tag=${extra//[^a-zA-Z0-9=]/_}
  local d=cfg$c${tag:+_$tag}
  extra=${extra//,/ }
  [ $c = 3 ] && steps=10
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats_$d -o run --output-format csv \
    -- python3 $R/bench.py --cfg $c $PROF $extra --steps $steps --warmup 2 \
    > $O/stats_$d.json 2> $O/stats_$d.log || return 1
  local i=0 grp
  for grp in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
             "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
    i=$((i+1))
    timeout -s KILL 400 rocprofv3 --pmc $grp --kernel-include-regex "$KRE" -d $O/pmc_$d/p$i -o run \
      --output-format csv -- python3 $R/bench.py --cfg $c $PROF $extra --steps 3 --warmup 1 \
      > $O/pmc_${d}_p$i.log 2>&1 || return 1
  done
  python3 $R/tools/pmc_summary.py $O/pmc_$d > $O/pmc_${d}_summary.txt 2>&1
}

step_sq() {
  local c=${1%%:*} topics=
  [ "$1" != "$c" ] && topics="--topics ${1#*:}"
  local i=0 grp
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
             "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-include-regex "k_walk" -d $O/sq_cfg$c/p$i -o run \
      --output-format csv -- python3 $R/bench.py --cfg $c $topics $PROF --steps 3 --warmup 1 \
      > $O/sq_cfg${c}_p$i.log 2>&1 || return 1
  done
  python3 $R/tools/pmc_summary.py $O/sq_cfg$c > $O/sq_cfg${c}_summary.txt 2>&1
}

step_stall() {
  # memory-subsystem stall counters of one kernel: issue/wait split (SQ),
  # address/data path busy and stalls (TA, TD), L1 pending and translation stalls (TCP)
  local c=${1%%:*} k=k_walk i=0 grp
  [ "$1" != "$c" ] && k=${1#*:}
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
             "SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
             "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_ADDR_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 400 rocprofv3 --pmc $grp --kernel-include-regex "$k" -d $O/stall_cfg$c/p$i -o run \
      --output-format csv -- python3 $R/bench.py --cfg $c $PROF --steps 3 --warmup 1 \
      > $O/stall_cfg${c}_p$i.log 2>&1 || return 1
  done
  python3 $R/tools/pmc_summary.py $O/stall_cfg$c > $O/stall_cfg${c}_summary.txt 2>&1
}

step_ab() {
  local specs=${1%%/*} variants=${1#*/} V spec
  cp $R/emqx_amd/libemqx_gpumatch.so $R/ablib/lib_base.so || return 1
  for V in base ${variants//,/ } base; do
    cp $R/ablib/lib_$V.so $R/emqx_amd/libemqx_gpumatch.so || return 1
    for spec in ${specs//,/ }; do
      local c=${spec%%:*} t=${spec##*:} T=""
      [ "$t" != 0 ] && T="--topics $t"
      (cd $R && timeout -k 10 300 python -u bench.py --cfg $c $T $NOCPU --steps 50 --warmup 5) \
        > $O/${V}_c${c}_${t}.json 2> $O/${V}_c${c}_${t}.log || { cp $R/ablib/lib_base.so $R/emqx_amd/libemqx_gpumatch.so; return 1; }
    done
  done
  cp $R/ablib/lib_base.so $R/emqx_amd/libemqx_gpumatch.so
  python3 $R/tools/ab_lib_summary.py $O > $O/ab_summary.txt 2>&1
}

step_load() {
  local c=${1%%:*} f=
  [ "$1" != "$c" ] && f="--filters ${1#*:}"
  (cd $R && timeout -k 10 600 python -u bench.py --cfg $c $f --only-nif) > $O/load_c$c.json 2> $O/load_c$c.log
}

step_latency() {
  hipcc --offload-arch=gfx950 -O3 $R/tools/latency_probe.hip -o $O/latency_probe || return 1
  timeout -k 10 180 $O/latency_probe > $O/latency_probe.txt 2>&1
  local rc=$?
  rm -f $O/latency_probe
  cat $O/latency_probe.txt
  return $rc
}

step_winlat() {
  local extra=${1//,/ } tag=${1//[^a-zA-Z0-9=]/_}
  (cd $R && timeout -k 10 300 python -u tools/window_latency.py $extra) > $O/winlat${tag:+_$tag}.json \
    2> $O/winlat${tag:+_$tag}.log
}

step_wintrace() {
  local extra=${1//,/ }
  timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d $O/wintrace \
    -o run --output-format csv -- python3 $R/tools/window_latency.py $extra \
    > $O/wintrace.json 2> $O/wintrace.log
}

step_dist() {
  local extra=""
  [ "$1" = filters ] && extra="--shard filters"
  [ "$1" = both ] && extra="--filter-shard"
  (cd $R && EMQXGM_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 $extra \
    --steps 5 --warmup 1) > $O/dist_n2${1:+_$1}.json 2> $O/dist_n2${1:+_$1}.log
}

for s in "$@"; do
  name=${s%%=*}
  arg=
  [ "$s" != "$name" ] && arg=${s#*=}
  echo "[job] $name $arg"
  step_$name "$arg"
  rc=$?
  if [ $rc != 0 ]; then
    echo "[job] step $s failed: $rc"
    exit $rc
  fi
done
echo "[job] done"
