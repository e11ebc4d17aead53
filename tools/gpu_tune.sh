set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TUNE_N=16777216 TUNE_ROUNDS=3 timeout -k 10 400 python3 tools/tune/tune_fixed.py > gpurun_out/tune16m.log 2>&1 || { tail gpurun_out/tune16m.log; exit 1; }
head -16 gpurun_out/tune16m.log
TUNE_N=1048576 TUNE_ROUNDS=5 timeout -k 10 300 python3 tools/tune/tune_fixed.py > gpurun_out/tune1m.log 2>&1 || { tail gpurun_out/tune1m.log; exit 1; }
head -12 gpurun_out/tune1m.log
timeout -k 10 300 python3 bench.py --cold --host-inclusive --no-cpu-baseline > gpurun_out/bench_cold1m.log 2>&1 && tail -1 gpurun_out/bench_cold1m.log
