set -u
OUT=gpurun_out/vdn; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name 2>&1; local rc=$?; echo "rc($name)=$rc"; if [ $rc -ne 0 ]; then tail -30 $OUT/$name; exit $rc; fi; }
step pytest.txt 300 python -u -m pytest tests/test_gpu_learn_kernels.py tests/test_gpu_torch_ops_learn.py tests/test_gpu_learners.py tests/test_gpu_learners_scale.py -m gpu -q --timeout 120 --timeout-method thread
tail -2 $OUT/pytest.txt
step vdn_profile.txt 300 python tools/vdn_profile.py
head -3 $OUT/vdn_profile.txt
step bench_config4.json 300 python bench.py --config 4 --no-cpu-baseline
head -c 400 $OUT/bench_config4.json
echo ALLDONE
