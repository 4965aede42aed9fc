export TMPDIR=/tmp
tools/gpu_steps.sh \
 pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --- \
 smoke 120 python -c "import __graft_entry__ as g; g.smoke()" --- \
 bench 300 python bench.py --- \
 prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline
