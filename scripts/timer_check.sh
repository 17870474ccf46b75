set -e
mkdir -p gpurun_out/tm
for r in 1 2; do
  for w in 0 20; do
    HPK_WARM=$w timeout -k 10 180 python scripts/dec_time.py config5 20 | sed "s/^/{\"warm\": $w, \"row\": /; s/\$/}/" >> gpurun_out/tm/dec.jsonl
  done
done
for r in 1 2; do
  for wl in config3 config3_text; do
    HPK_WARM=3 timeout -k 10 180 python scripts/dec_time.py $wl 10 >> gpurun_out/tm/c3.jsonl
  done
done
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu --no-config2 --no-config3 --no-config4 --no-compact > gpurun_out/tm/bench.json 2> gpurun_out/tm/bench.err
