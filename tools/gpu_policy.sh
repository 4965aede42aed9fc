export TMPDIR=/tmp
tools/gpu_steps.sh \
 pol_tests 400 python -u -m pytest tests/test_gpu_policy.py -x -v --timeout 300 --timeout-method thread --- \
 bench_pol 200 python bench.py --no-cpu-baseline --mode policy --- \
 bench_pol_g1 200 python bench.py --no-cpu-baseline --mode policy --groups 1 --- \
 bench_pol_c64 200 python bench.py --no-cpu-baseline --mode policy --chunk 64 --- \
 bench_pol_c64g1 200 python bench.py --no-cpu-baseline --mode policy --chunk 64 --groups 1 --- \
 prof_c5 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --mode policy
rm -f gpurun_out/prof_c5/run_kernel_trace.csv
for f in bench_pol bench_pol_g1 bench_pol_c64 bench_pol_c64g1; do grep -h '^{' gpurun_out/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$f', '%.3e'%d['value'], '%.3f us/step'%(d['ms_per_step']*1e3), c.get('env_step_fraction'), d['roofline']['launch_ms'])"; done
