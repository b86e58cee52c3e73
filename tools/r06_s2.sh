# round 6 session 2: the new GPU tests, the frame-graph probe, cold start, bench lines
set -o pipefail
mkdir -p gpurun_out/s2
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_frame_loop.py tests/test_gpu_jit_cache.py "tests/test_gpu_parity.py::test_edits_between_renders_match_oracle" "tests/test_gpu_parity.py::test_camera_changes_rerender" > gpurun_out/s2/pytest_new.log 2>&1 &&
timeout -k 10 180 python -u tools/graph_gather_probe.py tsp1080 2000 > gpurun_out/s2/graph.json 2> gpurun_out/s2/graph.err &&
timeout -k 10 120 python -u tools/coldstart_probe.py tsp1080 > gpurun_out/s2/cold_tsp.json 2> gpurun_out/s2/cold_tsp.err &&
timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 > gpurun_out/s2/bench.json 2> gpurun_out/s2/bench.err &&
MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 timeout -k 10 300 python -u bench.py --pipeline --steps 2000 --warmup 20 --no-cpu-baseline > gpurun_out/s2/bench_pipeline.json 2> gpurun_out/s2/bench_pipeline.err
echo done
