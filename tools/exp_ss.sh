export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --launch-trace"
tools/gpu_steps.sh \
 base_ss 120 $B --warmup 40000 --steps 20000 --- \
 base_ss_c1000 120 $B --warmup 40000 --steps 20000 --chunk 1000 --- \
 e32_ss 120 env SIT_LIBRARY=build_diag/libsit_e32.so $B --warmup 40000 --steps 20000 --- \
 e16_ss 120 env SIT_LIBRARY=build_diag/libsit_e16.so $B --warmup 40000 --steps 20000 --- \
 base_early 120 $B --warmup 200 --steps 20000
