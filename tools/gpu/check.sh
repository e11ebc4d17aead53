# One GPU-box pass: host facts, the GPU test suite, smoke, the headline bench
# and its rocprofv3 kernel stats.  Every GPU step has its own time limit and
# the steps are chained, so the first failure ends the pass.
#   gpurun -- 'bash tools/gpu/check.sh'          (TAG names the output dir)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-check}
mkdir -p "$O"
{ nproc; python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)))'; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; } > "$O/host.txt" 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > "$O/pytest_gpu.log" 2>&1 \
  && timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke()' > "$O/smoke.log" 2>&1 \
  && timeout -k 10 300 python3 -u bench.py ${BENCH_ARGS:-} > "$O/bench.log" 2>&1 \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline > "$O/prof.log" 2>&1
rc=$?
tail -2 "$O/pytest_gpu.log"
tail -1 "$O/bench.log"
exit $rc
