# rec128's rocprof stats and FETCH/WRITE passes without the shard leg (round_end.sh's B).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06end2; mkdir -p $O
B="bench.py --no-cpu-baseline --no-large --no-cold --no-host-inclusive --no-plain --no-shard --steps 10 --warmup 3"
s=rec128
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/stats_$s" -o k --output-format csv -- python3 $B --schema "$s" > "$O/stats_$s.log" 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch_$s" -o k --output-format csv -- python3 $B --schema "$s" > "$O/fetch_$s.log" 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$O/write_$s" -o k --output-format csv -- python3 $B --schema "$s" > "$O/write_$s.log" 2>&1 || exit 1
echo done
