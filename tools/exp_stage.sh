export TMPDIR=/tmp
tools/gpu_steps.sh \
 cur200 120 env SIT_LIBRARY=build_diag/libsit_cur.so python bench.py --no-cpu-baseline --chunk 200 --- \
 legld200 120 env SIT_LIBRARY=build_diag/libsit_legld.so python bench.py --no-cpu-baseline --chunk 200 --- \
 cur32 120 env SIT_LIBRARY=build_diag/libsit_cur.so python bench.py --no-cpu-baseline --chunk 32 --- \
 legld32 120 env SIT_LIBRARY=build_diag/libsit_legld.so python bench.py --no-cpu-baseline --chunk 32 --- \
 curpol 120 env SIT_LIBRARY=build_diag/libsit_cur.so python bench.py --no-cpu-baseline --mode policy --- \
 legldpol 120 env SIT_LIBRARY=build_diag/libsit_legld.so python bench.py --no-cpu-baseline --mode policy --- \
 ph 120 env SIT_LIBRARY=build_diag/libsit_phases.so python tools/diag_paths.py --warmup 40000 --chunk 200 --launches 5
for f in cur200 legld200 cur32 legld32 curpol legldpol; do grep -h '^{' gpurun_out/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', '%.4e'%d['value'], '%.3f us/step'%(d['ms_per_step']*1e3))"; done
grep "prologue" gpurun_out/ph.log
