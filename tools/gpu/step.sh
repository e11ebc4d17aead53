# One GPU-box pass of chosen steps, each under its own time limit, chained
# so that the first failure ends the pass.  Output under gpurun_out/$TAG.
#   gpurun -- 'TAG=x STEPS="copy tests:tests/test_deep.py,tests/test_kat.py bench:--schema,rpc" bash tools/gpu/step.sh'
#   (test paths and bench/prof arguments comma-separated; "tests" alone = the whole suite;
#    pmc:<schema> = kernel stats + FETCH_SIZE + WRITE_SIZE passes, tools/prof_summary.py layout)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-step}
mkdir -p "$O"
for st in ${STEPS:-tests bench}; do
  name=${st%%:*}; arg=${st#*:}; [ "$arg" = "$st" ] && arg=""
  echo "[step] $st $(date +%T)"
  case $name in
    copy) timeout -k 10 120 ./tools/probe/copy_ceiling 256 2048 4096 > "$O/copy_ceiling.log" 2>&1 ;;
    tests) ta=${arg:-tests}; timeout -k 10 900 python3 -u -m pytest ${ta//,/ } -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest_$(echo "${arg:-all}" | tr '/,.' '___').log" 2>&1 ;;
    smoke) timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke()' > "$O/smoke.log" 2>&1 ;;
    bench) timeout -k 10 400 python3 -u bench.py ${arg//,/ } > "$O/bench_${arg//[ ,-]/_}.log" 2>&1 ;;
    pmc) B="bench.py --no-cpu-baseline --no-large --no-cold --no-host-inclusive --no-plain --steps 10 --warmup 3 --schema $arg"
         timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/stats_$arg" -o k --output-format csv -- python3 $B > "$O/stats_$arg.log" 2>&1 &&
         timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch_$arg" -o k --output-format csv -- python3 $B > "$O/fetch_$arg.log" 2>&1 &&
         timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$O/write_$arg" -o k --output-format csv -- python3 $B > "$O/write_$arg.log" 2>&1 ;;
    cppbench) timeout -k 10 300 ./oracle/_ref/dropin_test bench ${arg:-1048576} > "$O/cppbench.log" 2>&1 ;;
    prof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_${arg//[ ,-]/_}" -o run --output-format csv -- python3 bench.py --no-cpu-baseline ${arg//,/ } > "$O/prof_${arg//[ ,-]/_}.log" 2>&1 ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
  rc=$?
  echo "[step] $st rc=$rc $(date +%T)"
  [ $rc -ne 0 ] && { tail -n 30 "$O"/*.log; exit $rc; }
done
tail -n 3 "$O"/*.log
