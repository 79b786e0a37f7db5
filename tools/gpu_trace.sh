# rocprofv3 kernel trace of a short config-3 bench (timeline of the learner chain vs the env step)
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace -o run -- python bench.py --steps 30 --warmup 5 > gpurun_out/trace_bench.json 2> gpurun_out/trace.err
find gpurun_out/trace -name "*kernel_trace.csv" | head -3
