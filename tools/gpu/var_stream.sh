# One-pass encode check: its GPU tests, the var parity tests, then bench
# lines and rocprofv3 kernel stats of recvar and rpc.  Each GPU step has its
# own time limit; the first failure ends the pass.  Output: gpurun_out/$TAG.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-vs}
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest ${TESTS:-tests/test_stream_encode.py} -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
for s in ${SCH:-recvar rpc}; do
  timeout -k 10 240 python3 -u bench.py --schema $s --no-cpu-baseline --no-large --steps 30 --warmup 5 ${BENCH_ARGS:-} > "$O/bench_$s.log" 2>&1 || { tail -20 "$O/bench_$s.log"; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/bench_$s.log') if l.startswith('{')][-1]); print('$s', d['value'], 'enc', d.get('encode_ms'), 'dec', d.get('decode_ms'), 'frac', d['roofline']['frac'])"
  if [ -n "${PROF:-1}" ]; then
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/prof_$s" -o run --output-format csv -- python3 bench.py --schema $s --no-cpu-baseline --no-large --steps 30 --warmup 5 > "$O/prof_$s.log" 2>&1 || { tail -20 "$O/prof_$s.log"; exit 1; }
    f=$(find "$O/prof_$s" -name '*kernel_stats.csv' | head -1)
    [ -n "$f" ] && head -12 "$f" | cut -d, -f1-4,7-8
  fi
done
