set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tr_pipe -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 40 --warmup 10 > gpurun_out/tr_pipe.log 2>&1; echo "rc=$?"
