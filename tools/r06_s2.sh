# round 6 session 2: the new GPU tests, the frame-graph probe, cold start, bench lines
set -o pipefail
mkdir -p gpurun_out/s2
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_frame_loop.py tests/test_gpu_jit_cache.py "tests/test_gpu_parity.py::test_edits_between_renders_match_oracle" "tests/test_gpu_parity.py::test_camera_changes_rerender" "tests/test_gpu_parity.py::test_device_face_bins_equal_host" "tests/test_gpu_parity.py::test_codegen_options_render_the_default_bytes" "tests/test_gpu_parity.py::test_heavy_tiles_equal_walk" > gpurun_out/s2/pytest_new.log 2>&1 &&
timeout -k 10 180 python -u tools/graph_gather_probe.py tsp1080 2000 > gpurun_out/s2/graph.json 2> gpurun_out/s2/graph.err &&
timeout -k 10 120 python -u tools/coldstart_probe.py tsp1080 > gpurun_out/s2/cold_tsp.json 2> gpurun_out/s2/cold_tsp.err &&
RTX_SETUP_LOG=1 timeout -k 10 180 python -u tools/setup_probe.py blob1080 > gpurun_out/s2/setup_blob.json 2> gpurun_out/s2/setup_blob.err &&
RTX_SETUP_LOG=1 RTX_DEV_BINS=0 timeout -k 10 180 python -u tools/setup_probe.py blob1080 > gpurun_out/s2/setup_blob_host.json 2> gpurun_out/s2/setup_blob_host.err &&
timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 > gpurun_out/s2/bench.json 2> gpurun_out/s2/bench.err &&
timeout -k 10 300 python -u bench.py --config blob1080 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/s2/bench_blob.json 2> gpurun_out/s2/bench_blob.err &&
MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 timeout -k 10 300 python -u bench.py --pipeline --steps 2000 --warmup 20 --no-cpu-baseline > gpurun_out/s2/bench_pipeline.json 2> gpurun_out/s2/bench_pipeline.err
echo done
