# Round-end measurement set (one GPU-box pass): the GPU test suite, smoke,
# per-schema bench lines (every leg), rocprofv3 kernel stats and
# FETCH_SIZE / WRITE_SIZE passes per schema (tools/prof_summary.py layout).
# Every GPU step has its own time limit; the first failure ends the pass.
#   gpurun -- 'TAG=r03z bash tools/gpu/round_end.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-round_end}
mkdir -p "$O"
{ nproc; python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)))'; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; } > "$O/host.txt" 2>&1
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -20 "$O/pytest_gpu.log"; exit 1; }
  tail -1 "$O/pytest_gpu.log"
  timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke()' > "$O/smoke.log" 2>&1 || exit 1
fi
timeout -k 10 400 python3 -u bench.py > "$O/bench_rec128.log" 2>&1 || exit 1
echo "[bench] rec128 done $(date +%T)"
for s in numerics recvar rpc vecrec containertest rp_list; do
  extra=""
  [ "$s" = recvar ] && extra="$extra --msgs"
  [ "$s" = rpc ] && extra="$extra --msgs --rpc"
  timeout -k 10 300 python3 -u bench.py --schema "$s" $extra > "$O/bench_$s.log" 2>&1 || exit 1
  echo "[bench] $s done $(date +%T)"
done
B="bench.py --no-cpu-baseline --no-large --no-cold --no-host-inclusive --no-plain --no-shard --steps 10 --warmup 3"
for s in rec128 numerics recvar rpc vecrec containertest rp_list; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/stats_$s" -o k --output-format csv -- python3 $B --schema "$s" > "$O/stats_$s.log" 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch_$s" -o k --output-format csv -- python3 $B --schema "$s" > "$O/fetch_$s.log" 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$O/write_$s" -o k --output-format csv -- python3 $B --schema "$s" > "$O/write_$s.log" 2>&1 || exit 1
  echo "[prof] $s done $(date +%T)"
done
