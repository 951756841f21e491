set -o pipefail
mkdir -p gpurun_out/q
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/q/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/q/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-baseline-seconds 2 > gpurun_out/q/bench.json 2> gpurun_out/q/bench.err || { tail -20 gpurun_out/q/bench.err; exit 1; }
cat gpurun_out/q/bench.json
FLOAM_DEBUG_STAMPS=1 timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --no-roofline > gpurun_out/q/bench_stamps.json 2> gpurun_out/q/bench_stamps.err || { tail -20 gpurun_out/q/bench_stamps.err; exit 1; }
grep stamps gpurun_out/q/bench_stamps.err
