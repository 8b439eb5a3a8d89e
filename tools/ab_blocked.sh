# Blocked-kernel check: GPU tests of the blocked paths, the in-kernel timeline, the headline bench.
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -m pytest tests/test_gpu.py -x -q -k "persistent_iterations or auto_native or blocked_xgmi or checkpoint_resumes or graft_smoke" > gpurun_out/ab/tests.log 2>&1 && \
timeout -k 10 120 python tools/blocked_timeline.py 300 > gpurun_out/ab/tl.json 2>gpurun_out/ab/tl.err && \
timeout -k 10 180 python bench.py --steps 20 --warmup 3 > gpurun_out/ab/bench.json 2>gpurun_out/ab/bench.err
echo rc=$?
