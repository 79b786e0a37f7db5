# rocprofv3 kernel trace of a config-3 bench (no policy loop, no CPU baseline) + the per-step timeline summary
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/tl && mkdir -p gpurun_out/tl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o run -- python bench.py --steps 80 --warmup 10 --policy-steps 0 --no-cpu-baseline "$@" > gpurun_out/tl/bench.json 2> gpurun_out/tl/bench.err || exit 1
f=$(find gpurun_out/tl -name "*kernel_trace.csv" | head -1)
python tools/trace_timeline.py "$f" > gpurun_out/tl/timeline.txt
cat gpurun_out/tl/timeline.txt
