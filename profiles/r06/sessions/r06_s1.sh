set -o pipefail
mkdir -p gpurun_out/s1
timeout -k 10 120 python -u tools/coldstart_probe.py tsp1080 > gpurun_out/s1/cold_jit.json 2> gpurun_out/s1/cold_jit.err &&
RTX_JIT=0 timeout -k 10 120 python -u tools/coldstart_probe.py tsp1080 > gpurun_out/s1/cold_nojit.json 2> gpurun_out/s1/cold_nojit.err &&
PROBE_HIPRTC=0 timeout -k 10 120 python -u tools/coldstart_probe.py tsp1080 > gpurun_out/s1/cold_jit_nohiprtc.json 2> gpurun_out/s1/cold_jit_nohiprtc.err &&
timeout -k 10 180 python -u tools/graph_gather_probe.py tsp1080 2000 > gpurun_out/s1/graph.json 2> gpurun_out/s1/graph.err &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s1/pytest_gpu.log 2>&1
echo done
