set -o pipefail
mkdir -p gpurun_out/v1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/v1/pytest.log 2>&1; rc=$?; tail -8 gpurun_out/v1/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v1/smoke.log 2>&1 || { tail -20 gpurun_out/v1/smoke.log; exit 1; }
tail -1 gpurun_out/v1/smoke.log
timeout -k 10 300 python bench.py --cpu-baseline-seconds 5 > gpurun_out/v1/bench.json 2> gpurun_out/v1/bench.err || { tail -20 gpurun_out/v1/bench.err; exit 1; }
cat gpurun_out/v1/bench.json
