# round 6 end: the driver's round-end GPU steps on this tree — GPU suite, smoke(), default bench
set -u
mkdir -p gpurun_out
T=${1:-r6z}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
