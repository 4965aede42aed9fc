#!/bin/bash
export TMPDIR=/tmp
tools/gpu_steps.sh \
 pol_tests 400 python -u -m pytest tests/test_gpu_policy.py -x -v --timeout 300 --timeout-method thread --- \
 pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --- \
 bench 200 python bench.py --no-cpu-baseline --- \
 bench_pol 200 python bench.py --no-cpu-baseline --mode policy --- \
 bench_pol_g1 200 python bench.py --no-cpu-baseline --mode policy --groups 1 --- \
 bench_pol_c64 200 python bench.py --no-cpu-baseline --mode policy --chunk 64 --- \
 bench_pol_c16 200 python bench.py --no-cpu-baseline --mode policy --chunk 16 --- \
 bench_pol_g4 200 python bench.py --no-cpu-baseline --mode policy --groups 4
for f in bench bench_pol bench_pol_g1 bench_pol_c64 bench_pol_c16 bench_pol_g4; do grep -h '^{' gpurun_out/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$f', '%.3e'%d['value'], '%.3f us/step'%(d['ms_per_step']*1e3), c.get('env_step_fraction'), d['roofline']['launch_ms'])"; done
