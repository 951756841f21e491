set -o pipefail
bash tools/gpu_ab.sh base i4 i6 base || exit 1
cp floam_amd/libfloam_amd_base.so floam_amd/libfloam_amd.so
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/tl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl/p -o run -- python3 bench.py --steps 20 --cpu-baseline-seconds 0 --no-roofline --no-secondary > gpurun_out/tl/log 2>&1 || { tail gpurun_out/tl/log; exit 1; }
ls -R gpurun_out/tl | head
