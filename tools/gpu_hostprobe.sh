mkdir -p gpurun_out/hp
for gph in 1 0; do
  FLOCK_SC_PIPELINE_GRAPHS=$gph timeout -k 10 120 python tools/host_cost.py > gpurun_out/hp/host_g$gph.txt 2>&1 || exit 1
  FLOCK_SC_PIPELINE_GRAPHS=$gph timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/hp/bench_g$gph.json 2>/dev/null || exit 1
  echo "graphs=$gph"; grep -v amdgpu gpurun_out/hp/host_g$gph.txt; grep -o '"ms_per_step": [0-9.]*' gpurun_out/hp/bench_g$gph.json
done
