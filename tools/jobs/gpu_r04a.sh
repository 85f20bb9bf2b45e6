#!/bin/bash
# Round-4 call A: captured-RCCL abort diagnosis.  Runs the overlap child
# (tests/_rccl_graph_child.py) under HIP error logging and RCCL INFO, in the
# default capture mode and in thread_local / relaxed, with the graphs dumped
# as dot files; then one short cfg2 bench to confirm the box.  Every child has
# its own time limit; a child abort is recorded and the next variant runs (an
# abort is a host-side SIGABRT, not a GPU fault), any timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04a
mkdir -p $OUT
export MASTER_ADDR=127.0.0.1
run_child() {  # name, then env assignments
  local name=$1; shift
  env "$@" AMD_LOG_LEVEL=1 NCCL_DEBUG=INFO MASTER_PORT=$((29600 + RANDOM % 300)) \
    MDE_GRAPH_DOT_DIR=$OUT/dot_$name timeout -k 10 240 python3 -u tests/_rccl_graph_child.py overlap \
    > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 3 $OUT/$name.log
  if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then exit $rc; fi
  return 0
}
run_child global1 MDE_GRAPH_CAPTURE_MODE=global
run_child global2 MDE_GRAPH_CAPTURE_MODE=global
run_child thread_local1 MDE_GRAPH_CAPTURE_MODE=thread_local
run_child thread_local2 MDE_GRAPH_CAPTURE_MODE=thread_local
run_child relaxed1 MDE_GRAPH_CAPTURE_MODE=relaxed
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 10 > $OUT/bench_gd.log 2>&1
echo "bench rc=$?"
tail -n 2 $OUT/bench_gd.log
