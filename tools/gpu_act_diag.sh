# timing-only variants of the act kernel (FLOCK_ACT_DIAG: 1 no LN1 stats, 2 no epilogue, 4 no B fetch, 7 none)
set -o pipefail
B=$PWD/marl_range_flocking_amd/_build
cp $B/libflock_amd.so $B/libflock_amd_base.so
for v in ${VARIANTS:-base d1 d2 d4 d7 base}; do
  cp $B/libflock_amd_$v.so $B/libflock_amd.so
  echo -n "$v: "; timeout -k 10 120 python tools/act_bench.py 2>/dev/null || { cp $B/libflock_amd_base.so $B/libflock_amd.so; exit 1; }
done
cp $B/libflock_amd_base.so $B/libflock_amd.so
