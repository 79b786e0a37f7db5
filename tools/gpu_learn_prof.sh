set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python tools/gap_probe.py > gpurun_out/gap_probe.txt 2>&1; echo "rc(gap)=$?"
GRAPH=1 ITERS=300 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/learnprof -o run --output-format csv -- python3 tools/prof_sc.py > gpurun_out/learnprof.log 2>&1; echo "rc(prof)=$?"
