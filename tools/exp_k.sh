export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --warmup 40000 --steps 20000"
P="env SIT_LIBRARY=build_diag/libsit_phases.so python tools/diag_paths.py --warmup 40000"
tools/gpu_steps.sh \
 k50 120 $B --chunk 50 --- k100 120 $B --chunk 100 --- k400 120 $B --chunk 400 --- k2000 120 $B --chunk 2000 --- \
 ph200 120 $P --chunk 200 --launches 20 --- ph1000 120 $P --chunk 1000 --launches 4
