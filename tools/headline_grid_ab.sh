BA="--warmup 5 --steps 20 --no-extras --no-sharded --no-pipe --no-train --no-shard-train --no-cascade --cpu-seconds 0 --sim-ranks 0"
for r in 1 2; do for g in 0 3072 6144 9216; do
  if [ $g = 0 ]; then unset RF_FUSED_GRID_CAP; else export RF_FUSED_GRID_CAP=$g; fi
  echo "grid_cap=$g r$r $(timeout -k 10 200 python bench.py $BA 2>/dev/null | python tools/bench_brief.py /dev/stdin | head -1)" || exit 1
done; done
