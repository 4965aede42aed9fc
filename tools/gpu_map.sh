export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --launch-trace"
tools/gpu_steps.sh \
 map 300 python -u -m pytest tests/test_gpu_map.py -x -v --timeout 200 --timeout-method thread --- \
 pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --- \
 base_ss 120 $B --warmup 40000 --steps 20000 --- \
 base_ss_c1000 120 $B --warmup 40000 --steps 20000 --chunk 1000 --- \
 slow 300 env SIT_LIBRARY=build_diag/libsit_phases.so python tools/diag_slow.py --- \
 ph200 120 env SIT_LIBRARY=build_diag/libsit_phases.so python tools/diag_paths.py --warmup 40000 --chunk 200 --launches 10
