# round 4: numerics fixed group kernel sweep (workgroups, chunks in flight, non-temporal stores), one box
mkdir -p gpurun_out/r04bf
B="python -u bench.py --schema numerics --steps 30 --warmup 5 --no-cpu-baseline --no-large --no-cold --no-host-inclusive --no-plain"
for o in "" "--plan-opt grp_blocks=1024" "--plan-opt grp_blocks=4096" "--plan-opt grp_blocks=8192" "--plan-opt grp_unroll=1" "--plan-opt grp_unroll=2" "--plan-opt grp_unroll=4" "--plan-opt grp_nontemporal=1" "--plan-opt grp_blocks=4096 --plan-opt grp_nontemporal=1" ""; do
  echo "== $o" >> gpurun_out/r04bf/sweep.log
  timeout -k 10 120 $B $o 2>/dev/null | tail -1 >> gpurun_out/r04bf/sweep.log || exit 1
done
